source tools/gpu_step.sh
run_step 600 t_ops python -u -m pytest -q --tb=short --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_ops2.py tests/test_gpu_halo_small.py tests/test_gpu_attn.py tests/test_gpu_train.py
echo ALLDONE
