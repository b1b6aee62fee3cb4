source tools/gpu_step.sh
# round 4: 192-channel 3x3 on 4 waves at one per SIMD (LIC_WD_BN192=3) vs the 8-wave tiles (=1)
mkdir -p gpurun_out/r04k
LIC_WD_BN192=3 run_step 200 r04k/split3 python -u -m pytest tests/test_gpu_split.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "test_split_conv_matches_fp32 and 192-192-3-1"
for v in 1 3 1 3; do
  LIC_WD_BN192=$v run_step 200 r04k/conv_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa3x3@64,rbws_conv2@128 --iters 30
done
echo ALLDONE
