source tools/gpu_step.sh
mkdir -p gpurun_out/r03wg
run_step 400 r03wg/tests python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_attn.py -x -v --timeout 200 --timeout-method thread
run_step 400 r03wg/split_tests python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread -k "matches_fp32"
run_step 200 r03wg/bench_tiled python -u tools/wgrad_bench.py
LIC_WGRAD_TR=0 run_step 200 r03wg/bench_generic python -u tools/wgrad_bench.py
run_step 300 r03wg/train_tiled python -u train_net_unet.py --bench --steps 10 --warmup 3
LIC_WGRAD_TR=0 run_step 300 r03wg/train_generic python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 300 r03wg/conv_bench python -u tools/conv_bench.py --dtype fp32x6
echo ALLDONE
