source tools/gpu_step.sh
mkdir -p gpurun_out/r03b3
export TMPDIR=/tmp
run_step 600 r03b3/bench python3 bench.py
run_step 400 r03b3/prof_train_graph rocprofv3 --kernel-trace --stats -d gpurun_out/r03b3/train_graph -o run -- python3 -u train_net_unet.py --bench --steps 5 --warmup 3 --graph
echo ALLDONE
