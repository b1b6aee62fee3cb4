source tools/gpu_step.sh
# round 4: strided-view weight packs (training re-packs): training parity tests, bench, kernel trace
mkdir -p gpurun_out/r04v
run_step 400 r04v/train_tests python -u -m pytest tests/test_gpu_train_net.py tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread
run_step 300 r04v/train_bench_graph python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 300 r04v/prof_train rocprofv3 --kernel-trace --stats -d gpurun_out/r04v/prof -o run -- python3 train_net_unet.py --bench --steps 5 --warmup 2
echo ALLDONE
