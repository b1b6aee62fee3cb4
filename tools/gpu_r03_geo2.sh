source tools/gpu_step.sh
# GEO 1 for 7x7 and the virtual-tap 1x1 configs: parity + timing (vs LIC_WD_GEO=0)
mkdir -p gpurun_out/r03geo2
run_step 400 r03geo2/test python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_resunit.py -x -q --timeout 120 --timeout-method thread
SH=wnsa3x3@64,wnsa7x7@64,wnsa7x7@16,conv5x5s2@32,qkv1x1@64,proj1x1@64,gdn1x1@128,lin512_128@16,ru1x1_128_64@16,cc1x1_128_32@16,wnsa3x3@16
run_step 150 r03geo2/bench_geo python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
LIC_WD_GEO=0 run_step 150 r03geo2/bench_gen python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
run_step 300 r03geo2/bench python3 bench.py --precision fp32x6
echo ALLDONE
