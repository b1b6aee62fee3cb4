source tools/gpu_step.sh
run_step 600 t_bf16 python -u -m pytest -q -x --tb=short --timeout 300 --timeout-method thread -k "bfloat16 or bf16" tests/test_gpu_ops.py tests/test_gpu_ops2.py tests/test_gpu_halo_small.py tests/test_gpu_attn.py tests/test_gpu_train.py tests/test_gpu_train_net.py -s
run_step 300 train_bench_bf16 python -u train_net_unet.py --bench --steps 5 --warmup 2
echo ALLDONE
