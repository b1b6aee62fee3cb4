source tools/gpu_step.sh
# round 4: 192-channel 7x7 A/B, RCCL-captured training step test, end-to-end A/B, kernel trace
mkdir -p gpurun_out/r04c
for v in 0 1; do
  LIC_WD_BN192=$v run_step 200 r04c/conv_bn192_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128 --iters 30
done
LIC_WD_BN192=1 run_step 200 r04c/split_bn192_1 python -u -m pytest tests/test_gpu_split.py -m gpu -q -k "test_split_conv_matches_fp32 and (192-192-3-1 or 192-192-7-1)" --timeout 120 --timeout-method thread -p no:cacheprovider
for v in 0 1 2; do
  LIC_WD_VT=$v run_step 200 r04c/conv_vt_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only qkv1x1@64,proj1x1@64,c1x1@128 --iters 30
done
LIC_WD_VT=1 run_step 200 r04c/split_vt_1 python -u -m pytest tests/test_gpu_split.py -m gpu -q -k "test_split_conv_matches_fp32 and 1-1-0-0-0-0" --timeout 120 --timeout-method thread -p no:cacheprovider
LIC_WD_VT=2 run_step 200 r04c/split_vt_2 python -u -m pytest tests/test_gpu_split.py -m gpu -q -k "test_split_conv_matches_fp32 and 1-1-0-0-0-0" --timeout 120 --timeout-method thread -p no:cacheprovider
run_step 300 r04c/split_all python -u -m pytest tests/test_gpu_split.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
LIC_WD_GEO=0 run_step 200 r04c/conv_s2_nogeo python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only conv5x5s2@128,conv5x5s2@32 --iters 30
run_step 200 r04c/conv_s2_geo python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only conv5x5s2@128,conv5x5s2@32 --iters 30
run_step 400 r04c/dist_graph python -u -m pytest tests/test_gpu_dist_train.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k graph_step
for v in 0 1; do
  LIC_WD_BN192=$v run_step 300 r04c/bench_bn192_$v python3 bench.py --no-extras --precision fp32x6
done
run_step 300 r04c/trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04c/trace -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
echo ALLDONE
