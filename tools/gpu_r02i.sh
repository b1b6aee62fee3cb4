source tools/gpu_step.sh
run_step 400 wbast2 python -u tools/op_determinism.py --reps 16 --wba-stages
run_step 300 probe_fix python -u tools/determinism_probe.py --reps 4 --no-poison --single-stream
run_step 300 attn_tests python -u -m pytest -x -q --timeout 200 tests/test_gpu_attn.py
echo ALLDONE
