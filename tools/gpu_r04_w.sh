source tools/gpu_step.sh
# round 4: fused Adam (one multi-tensor kernel per step) vs the foreach capturable path, same box
mkdir -p gpurun_out/r04w
run_step 300 r04w/train_fused_adam python -u train_net_unet.py --bench --steps 10 --warmup 3
LIC_FUSED_ADAM=0 run_step 300 r04w/train_foreach_adam python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 300 r04w/train_fused_adam2 python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 300 r04w/prof_train rocprofv3 --kernel-trace -d gpurun_out/r04w/prof -o run -- python3 train_net_unet.py --bench --steps 5 --warmup 2
echo ALLDONE
