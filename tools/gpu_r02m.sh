source tools/gpu_step.sh
run_step 600 t_train python -u -m pytest -v -s --tb=short --timeout 400 --timeout-method thread tests/test_gpu_train_net.py
run_step 300 train_bench_unet python -u train_net_unet.py --bench --steps 5 --warmup 2 --arch net_unet_ha_hs --precision fp16
echo ALLDONE
