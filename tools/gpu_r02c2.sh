source tools/gpu_step.sh
run_step 500 t_split python -u -m pytest -q --tb=short --timeout 300 --timeout-method thread tests/test_gpu_split.py -s
run_step 200 acc3 python -u tools/split_accuracy.py
run_step 200 cb_s1 python -u tools/conv_bench.py --dtype fp32x3 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128,conv5x5s2@128
for c in FETCH_SIZE WRITE_SIZE; do
  run_step 90 pmc_fp32x3_${c} timeout -s KILL 80 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_fp32x3_${c} -o pmc -- python3 tools/conv_bench.py --dtype fp32x3 --iters 5 --auto-only --only wnsa3x3@64
done
run_step 200 trace_x3 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_x3 -o trace -- python3 bench.py --profile --steps 5 --warmup 2 --precision fp32x3
run_step 700 bench_all python -u bench.py
echo ALLDONE
