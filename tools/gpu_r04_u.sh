source tools/gpu_step.sh
# round 4: config-5 training step (net_unet_ha_hs bf16, B=8, hipGraph-captured default) on HEAD
mkdir -p gpurun_out/r04u
run_step 300 r04u/train_bench_graph python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 300 r04u/wba_bench python -u tools/wba_bench.py
echo ALLDONE
