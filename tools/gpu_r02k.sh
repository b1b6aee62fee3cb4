source tools/gpu_step.sh
run_step 900 gpu_tests python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread
run_step 120 trace_conv_fp32 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_conv_fp32 -o trace -- python3 tools/conv_bench.py --dtype fp32 --iters 20 --auto-only --only wnsa3x3@64
echo ALLDONE
