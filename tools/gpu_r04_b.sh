source tools/gpu_step.sh
# round 4: the 192-channel WD 3x3 experiment (LIC_WD_BN192=1: 8 waves, =2: 4 waves at one per SIMD)
# + the failing parity tests with the conditioned rate bar
mkdir -p gpurun_out/r04b
for v in 0 1 2; do
  LIC_WD_BN192=$v run_step 200 r04b/conv_bn192_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa3x3@64,rbws_conv2@128,rbneck3x3_96@64 --iters 30
done
LIC_WD_BN192=1 run_step 200 r04b/split_bn192_1 python -u -m pytest tests/test_gpu_split.py -m gpu -q -k "test_split_conv_matches_fp32 and 192-192-3-1" --timeout 120 --timeout-method thread -p no:cacheprovider
LIC_WD_BN192=2 run_step 200 r04b/split_bn192_2 python -u -m pytest tests/test_gpu_split.py -m gpu -q -k "test_split_conv_matches_fp32 and 192-192-3-1" --timeout 120 --timeout-method thread -p no:cacheprovider
run_step 600 r04b/gpu_tests python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_net.py tests/test_gpu_split.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "forward or net_parity or kodak"
echo ALLDONE
