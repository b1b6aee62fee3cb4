source tools/gpu_step.sh
mkdir -p gpurun_out/r03prof3
export TMPDIR=/tmp
run_step 300 r03prof3/trace_fp32x6 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03prof3/trace_fp32x6 -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
run_step 300 r03prof3/layers python3 tools/layer_profile.py --precision fp32x6
echo ALLDONE
