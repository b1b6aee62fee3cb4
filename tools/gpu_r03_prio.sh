source tools/gpu_step.sh
mkdir -p gpurun_out/r03prio
S=wnsa3x3@64,rbws_conv2@128,wnsa7x7@64,qkv1x1@64
run_step 300 r03prio/wgrad_tests python -u -m pytest tests/test_gpu_wgrad.py -x -q --timeout 200 --timeout-method thread
run_step 200 r03prio/wgrad_bench python -u tools/wgrad_bench.py
run_step 120 r03prio/base python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $S
LIC_LIB=tools/native/liblic_prio1.so run_step 120 r03prio/prio1 python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $S
LIC_LIB=tools/native/liblic_prio2.so run_step 120 r03prio/prio2 python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $S
run_step 120 r03prio/base2 python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $S
echo ALLDONE
