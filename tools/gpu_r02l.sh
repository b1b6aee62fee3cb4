source tools/gpu_step.sh
run_step 400 t_new python -u -m pytest -v --tb=short --timeout 300 --timeout-method thread tests/test_gpu_net.py tests/test_gpu_threads.py tests/test_gpu_coder.py
echo ALLDONE
