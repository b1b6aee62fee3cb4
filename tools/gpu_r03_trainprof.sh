source tools/gpu_step.sh
mkdir -p gpurun_out/r03tp
export TMPDIR=/tmp
run_step 400 r03tp/prof_tiled rocprofv3 --kernel-trace --stats -d gpurun_out/r03tp/tiled -o run -- python3 -u train_net_unet.py --bench --steps 5 --warmup 2
LIC_WGRAD_TR=0 run_step 400 r03tp/prof_generic rocprofv3 --kernel-trace --stats -d gpurun_out/r03tp/generic -o run -- python3 -u train_net_unet.py --bench --steps 5 --warmup 2
run_step 300 r03tp/train_tiled2 python -u train_net_unet.py --bench --steps 20 --warmup 5
LIC_WGRAD_TR=0 run_step 300 r03tp/train_generic2 python -u train_net_unet.py --bench --steps 20 --warmup 5
echo ALLDONE
