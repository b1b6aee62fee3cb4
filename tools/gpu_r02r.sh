source tools/gpu_step.sh
run_step 600 t_train python -u -m pytest -q -x --tb=short --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_train_net.py -s
run_step 300 tb_bf16 python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 300 trace_train rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_train -o trace -- python3 train_net_unet.py --bench --steps 5 --warmup 2
echo ALLDONE
