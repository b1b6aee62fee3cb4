source tools/gpu_step.sh
# round 4: 96-channel 16x16-px tiles for the ResidualBottleneck 3x3 at 64^2 (LIC_WD_BN96) + parity
mkdir -p gpurun_out/r04q
for v in 0 1; do
  LIC_WD_BN96=$v run_step 200 r04q/conv_bn96_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only rbneck3x3_96@64,wnsa3x3@16 --iters 30
done
run_step 300 r04q/split python -u -m pytest tests/test_gpu_split.py tests/test_gpu_configs.py -m gpu -q --timeout 170 --timeout-method thread -p no:cacheprovider
LIC_WD_BN96=0 run_step 300 r04q/bench_0 python3 bench.py --no-extras --precision fp32x6
run_step 300 r04q/bench_1 python3 bench.py --no-extras --precision fp32x6
echo ALLDONE
