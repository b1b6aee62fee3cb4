source tools/gpu_step.sh
run_step 600 t_graph python -u -m pytest -q -x --tb=short --timeout 300 --timeout-method thread tests/test_gpu_train_net.py -k "graph" -s
run_step 300 trace_train rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_train -o trace -- python3 train_net_unet.py --bench --steps 5 --warmup 2
echo ALLDONE
