source tools/gpu_step.sh
# round 4: fused WinBasedAttention incl. proj + shortcut (bit-exactness, timing, bench A/B) and the
# 4-wave one-per-SIMD 192-channel 3x3 experiment (LIC_WD_BN192=3)
mkdir -p gpurun_out/r04l
run_step 300 r04l/attn python -u -m pytest tests/test_gpu_attn.py -m gpu -q -x --timeout 160 --timeout-method thread -p no:cacheprovider
run_step 120 r04l/wba python -u tools/wba_bench.py
LIC_WD_BN192=3 run_step 200 r04l/split3 python -u -m pytest tests/test_gpu_split.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "test_split_conv_matches_fp32 and 192-192-3-1"
for v in 1 3 1 3; do
  LIC_WD_BN192=$v run_step 200 r04l/conv_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa3x3@64,rbws_conv2@128 --iters 30
done
run_step 500 r04l/net python -u -m pytest tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_net.py tests/test_gpu_coder.py -m gpu -q -x --timeout 170 --timeout-method thread -p no:cacheprovider
LIC_FUSED_WBA=0 run_step 300 r04l/bench_unfused python3 bench.py --no-extras --precision fp32x6
run_step 300 r04l/bench_fused python3 bench.py --no-extras --precision fp32x6
echo ALLDONE
