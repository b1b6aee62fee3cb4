source tools/gpu_step.sh
mkdir -p gpurun_out/r03bench2
run_step 300 r03bench2/test_split python -u -m pytest tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread
run_step 120 r03bench2/conv_base python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only wnsa3x3@64,rbws_conv2@128,qkv1x1@64,wnsa7x7@64
LIC_LIB=tools/native/liblic_wdnt.so run_step 120 r03bench2/conv_nt python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only wnsa3x3@64,rbws_conv2@128,qkv1x1@64,wnsa7x7@64
LIC_LIB=tools/native/liblic_wdnt.so run_step 90 r03bench2/pmc_FETCH_nt timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03bench2/pmc_FETCH_nt -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
run_step 600 r03bench2/bench python3 bench.py
echo ALLDONE
