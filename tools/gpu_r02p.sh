source tools/gpu_step.sh
run_step 600 t_graph python -u -m pytest -q -x --tb=short --timeout 300 --timeout-method thread tests/test_gpu_train_net.py tests/test_gpu_train.py -k "graph or rate or noise or train_step" -s
run_step 300 tb_eager python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 300 tb_graph python -u train_net_unet.py --bench --steps 10 --warmup 3 --graph
echo ALLDONE
