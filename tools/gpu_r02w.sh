source tools/gpu_step.sh
run_step 400 t_split python -u -m pytest -q --tb=short --timeout 300 --timeout-method thread tests/test_gpu_split.py -s
run_step 200 cb_split6 python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128,conv5x5s2@128
run_step 200 b_split6 python -u bench.py --no-extras --precision fp32x6
echo ALLDONE
