source tools/gpu_step.sh
# round 4: small-map 1x1 convs on the 8x8-px virtual-tap tiles (LIC_WD_SMALL1X1_ALL) -- timing + parity;
# the fixed fused-WBA / RCCL-capture tests
mkdir -p gpurun_out/r04n
for v in 0 1; do
  LIC_WD_SMALL1X1_ALL=$v run_step 200 r04n/conv_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only lin128_512@16,lin512_128@16,qkv1x1@16,gdn1x1@32,in1x1_320_128@16 --iters 30
done
run_step 300 r04n/attn_dist python -u -m pytest tests/test_gpu_attn.py tests/test_gpu_dist_train.py -m gpu -q -x --timeout 165 --timeout-method thread -p no:cacheprovider
run_step 600 r04n/net python -u -m pytest tests/test_gpu_split.py tests/test_gpu_resunit.py tests/test_gpu_configs.py tests/test_gpu_net.py tests/test_gpu_coder.py -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider
run_step 200 r04n/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
LIC_WD_SMALL1X1_ALL=0 run_step 300 r04n/bench_0 python3 bench.py --no-extras --precision fp32x6
run_step 300 r04n/bench_1 python3 bench.py --no-extras --precision fp32x6
echo ALLDONE
