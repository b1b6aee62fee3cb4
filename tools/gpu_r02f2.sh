source tools/gpu_step.sh
run_step 200 cb_base python -u tools/conv_bench.py --dtype fp32x3 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128
LIC_SPLIT_W4=1 run_step 200 cb_w4 python -u tools/conv_bench.py --dtype fp32x3 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128
LIC_SPLIT_W4=1 run_step 200 acc_w4 python -u tools/split_accuracy.py
echo ALLDONE
