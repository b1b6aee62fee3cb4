source tools/gpu_step.sh
mkdir -p gpurun_out/r03prof2
run_step 120 r03prof2/g1_base python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only qkv1x1@64,proj1x1@64,gdn1x1@128
LIC_LIB=tools/native/liblic_g1alt0.so run_step 120 r03prof2/g1_alt0 python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only qkv1x1@64,proj1x1@64,gdn1x1@128
run_step 300 r03prof2/trace_fp32x6 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03prof2/trace_fp32x6 -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
echo ALLDONE
