source tools/gpu_step.sh
mkdir -p gpurun_out/r03full
run_step 1000 r03full/gpu_tests python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run_step 300 r03full/trace_fp32x6 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03full/trace_fp32x6 -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
echo ALLDONE
