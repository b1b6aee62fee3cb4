source tools/gpu_step.sh
run_step 600 t_train python -u -m pytest -q --tb=short --timeout 300 --timeout-method thread tests/test_gpu_train_net.py tests/test_gpu_train.py -s -k "hipgraph or attn or table or unet"
echo ALLDONE
