# r03: split tests, PMC traffic of the fp32x6 roofline kernel, full default bench line
source tools/gpu_step.sh
mkdir -p gpurun_out/r03bench
run_step 300 r03bench/test_split python -u -m pytest tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread
for c in FETCH_SIZE WRITE_SIZE; do
  run_step 90 r03bench/pmc_$c timeout -s KILL 80 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r03bench/pmc_$c -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
done
run_step 60 r03bench/pmc_summary python3 tools/pmc_summary.py gpurun_out/r03bench/pmc_FETCH_SIZE gpurun_out/r03bench/pmc_WRITE_SIZE conv_split_wd_kernel "conv_split_wd_kernel fp32x6 conv3x3 192->192 @64x64 B=32" "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64" gpurun_out/r03bench/pmc_conv3x3_64_f32x6.json
run_step 600 r03bench/bench python3 bench.py
echo ALLDONE
