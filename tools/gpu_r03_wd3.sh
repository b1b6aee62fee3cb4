source tools/gpu_step.sh
mkdir -p gpurun_out/r03wd3
run_step 300 r03wd3/test_split_ops python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread -k matches_fp32 -s
run_step 120 r03wd3/bench_fp32x6 python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only wnsa3x3@64,rbws_conv2@128,rbneck3x3_96@64
echo ALLDONE
