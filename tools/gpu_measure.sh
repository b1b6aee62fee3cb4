# bench + rocprof evidence for the headline (fp32) and the fp16 extra; outputs under gpurun_out/
source tools/gpu_step.sh
run_step 400 bench python -u bench.py
for dt in fp32 fp16; do
  for c in FETCH_SIZE WRITE_SIZE; do
    run_step 90 pmc_${dt}_${c} timeout -s KILL 80 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${dt}_${c} -o pmc -- python3 tools/conv_bench.py --dtype $dt --iters 5 --auto-only --only wnsa3x3@64
  done
done
run_step 200 trace_fp32 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_fp32 -o trace -- python3 bench.py --profile --steps 5 --warmup 2
echo ALLDONE
