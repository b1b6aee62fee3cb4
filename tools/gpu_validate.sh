source tools/gpu_step.sh
run_step 400 gpu_tests python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run_step 300 bench python -u bench.py
run_step 300 coder_bench python -u tools/coder_bench.py
echo ALLDONE
