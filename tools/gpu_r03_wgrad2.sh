source tools/gpu_step.sh
mkdir -p gpurun_out/r03wg2
run_step 400 r03wg2/tests python -u -m pytest tests/test_gpu_wgrad.py -x -v --timeout 200 --timeout-method thread
run_step 200 r03wg2/bench_tiled python -u tools/wgrad_bench.py
run_step 300 r03wg2/train_graph python -u train_net_unet.py --bench --steps 20 --warmup 5 --graph
run_step 300 r03wg2/train_eager python -u train_net_unet.py --bench --steps 20 --warmup 5
echo ALLDONE
