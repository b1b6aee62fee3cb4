source tools/gpu_step.sh
mkdir -p gpurun_out/r03prof
run_step 300 r03prof/layers_fp32x6 python3 tools/layer_profile.py --precision fp32x6 --top 70
run_step 300 r03prof/trace_fp32x6 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03prof/trace_fp32x6 -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
echo ALLDONE
