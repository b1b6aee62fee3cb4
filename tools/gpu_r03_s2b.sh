source tools/gpu_step.sh
# round 3 session 2: training after the uniform-wave-index fix, wgrad, small 1x1 A/B, split tests
mkdir -p gpurun_out/r03s2b
run_step 300 r03s2b/split_tests python3 -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread -k "4-"
run_step 200 r03s2b/wgrad python -u tools/wgrad_bench.py
run_step 300 r03s2b/train_graph python -u train_net_unet.py --bench --steps 20 --warmup 5
SH=lin512_128@16,lin128_512@16,in1x1_320_128@16,cc1x1_128_32@16,ru1x1_64_128@16
run_step 120 r03s2b/small1x1_wd python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
LIC_WD_SMALL1X1=0 run_step 120 r03s2b/small1x1_gemm python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
echo ALLDONE
