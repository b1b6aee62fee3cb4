# r03: weights-direct split kernel (conv_split_wd.hip): op parity, conv timings, end-to-end fp32x6 parity
source tools/gpu_step.sh
mkdir -p gpurun_out/r03wd
run_step 300 r03wd/test_split_ops python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread -k matches_fp32 -s
run_step 120 r03wd/bench_fp32x6 python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only wnsa3x3@64,rbws_conv2@128,wnsa7x7@64,conv5x5s2@128,rbneck3x3_96@64,qkv1x1@64,wnsa3x3@16,cc3x3_336_224@16
run_step 300 r03wd/test_split_net python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread -k "net_parity and fp32x6 and net_ga-1" -s

run_step 300 r03wd/trace_fp32x6 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03wd/trace_fp32x6 -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
run_step 200 r03wd/bench_fp32x6_noextra python3 bench.py --precision fp32x6 --no-extras --steps 20 --warmup 3
echo ALLDONE2
