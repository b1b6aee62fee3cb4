source tools/gpu_step.sh
run_step 200 acc3 python -u tools/split_accuracy.py
run_step 200 acc7 python -u tools/split_accuracy.py --k 7
run_step 200 cb_s1 python -u tools/conv_bench.py --dtype fp32x3 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128,conv5x5s2@128
LIC_SPLIT_NO192=1 run_step 200 cb_s1_128 python -u tools/conv_bench.py --dtype fp32x3 --auto-only --only wnsa3x3@64,wnsa7x7@64
run_step 200 cb_s2 python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128,conv5x5s2@128
run_step 400 t_split python -u -m pytest -q --tb=short --timeout 300 --timeout-method thread tests/test_gpu_split.py -s
echo ALLDONE
