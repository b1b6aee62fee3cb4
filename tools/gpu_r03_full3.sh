source tools/gpu_step.sh
mkdir -p gpurun_out/r03full3
run_step 600 r03full3/bench python3 bench.py
run_step 90 r03full3/pmc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03full3/pmc_fetch -o f -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
run_step 90 r03full3/pmc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r03full3/pmc_write -o w -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
run_step 300 r03full3/trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03full3/trace -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
run_step 1000 r03full3/gpu_tests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
run_step 300 r03full3/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
echo ALLDONE
