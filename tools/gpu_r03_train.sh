source tools/gpu_step.sh
mkdir -p gpurun_out/r03train
run_step 600 r03train/tests python -u -m pytest tests/test_gpu_dist_train.py tests/test_gpu_train_net.py -x -v --timeout 400 --timeout-method thread -k "allreduce or bf16" -s
echo ALLDONE
