source tools/gpu_step.sh
# round 4: fused fp32x6 qkv + window attention (csrc/wba_split.hip): bit-exactness, timing, bench A/B
mkdir -p gpurun_out/r04j
run_step 300 r04j/attn python -u -m pytest tests/test_gpu_attn.py tests/test_capi.py -m "gpu or not gpu" -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
run_step 120 r04j/wba python -u tools/wba_bench.py
run_step 500 r04j/net python -u -m pytest tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_net.py tests/test_gpu_coder.py -m gpu -q -x --timeout 170 --timeout-method thread -p no:cacheprovider
LIC_FUSED_WBA=0 run_step 300 r04j/bench_unfused python3 bench.py --no-extras --precision fp32x6
run_step 300 r04j/bench_fused python3 bench.py --no-extras --precision fp32x6
echo ALLDONE
