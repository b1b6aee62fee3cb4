source tools/gpu_step.sh
mkdir -p gpurun_out/r03s2
run_step 400 r03s2/split_tests python -u -m pytest tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread
run_step 400 r03s2/train_tests python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread
run_step 600 r03s2/bench python3 bench.py --precision fp32x6
run_step 300 r03s2/train_graph python -u train_net_unet.py --bench --steps 20 --warmup 5 --graph
echo ALLDONE
