source tools/gpu_step.sh
# round 4: 192-channel tiles for the 6 / 4-tap phases; stride-2 phases on small maps (hyper analysis)
mkdir -p gpurun_out/r04o
for v in 0 1; do
  LIC_WD_BN192=$v run_step 200 r04o/conv_bn$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only conv5x5s2@128,conv5x5s2@32 --iters 30
done
run_step 600 r04o/net python -u -m pytest tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_net.py tests/test_gpu_coder.py -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider
run_step 200 r04o/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
LIC_S2_PHASE_MIN_PIX=16384 run_step 300 r04o/bench_a python3 bench.py --no-extras --precision fp32x6
run_step 300 r04o/bench_b python3 bench.py --no-extras --precision fp32x6
echo ALLDONE
