source tools/gpu_step.sh
# ConvT phases on compile-time grids (ascending taps): full suite, bench, ConvT timings
mkdir -p gpurun_out/r03convt
run_step 500 r03convt/gpu_tests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
run_step 200 r03convt/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 600 r03convt/bench python3 bench.py
run_step 300 r03convt/trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03convt/trace -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
echo ALLDONE
