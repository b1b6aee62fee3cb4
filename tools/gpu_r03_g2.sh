source tools/gpu_step.sh
mkdir -p gpurun_out/r03g2
run_step 300 r03g2/test_split_ops python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread -k "matches_fp32 or transpose" -s
run_step 120 r03g2/bench_fp32x6 python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only wnsa3x3@16,cc3x3_224_128@16,cc3x3_128_48@16,ru3x3_64@16,ru1x1_128_64@16,ru1x1_64_128@16,lin512_128@16
run_step 400 r03g2/test_split_net python -u -m pytest tests/test_gpu_split.py -v --timeout 300 --timeout-method thread -k "net_parity and fp32x6" -s
run_step 200 r03g2/bench_fp32x6_noextra python3 bench.py --precision fp32x6 --no-extras --steps 20 --warmup 3
echo ALLDONE
