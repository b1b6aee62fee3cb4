source tools/gpu_step.sh
# round 4: 96-channel tap-group tiles for the 16x16 latents' 192-channel 3x3 (LIC_WD_BN96) + parity
mkdir -p gpurun_out/r04p
for v in 0 1; do
  LIC_WD_BN96=$v run_step 200 r04p/conv_bn96_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa3x3@16,cc3x3_336_224@16,wnsa7x7@16 --iters 30
done
run_step 600 r04p/net python -u -m pytest tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_net.py tests/test_gpu_coder.py -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider
run_step 200 r04p/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
LIC_WD_BN96=0 run_step 300 r04p/bench_0 python3 bench.py --no-extras --precision fp32x6
run_step 300 r04p/bench_1 python3 bench.py --no-extras --precision fp32x6
echo ALLDONE
