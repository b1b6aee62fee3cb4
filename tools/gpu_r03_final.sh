source tools/gpu_step.sh
# round 3 closing state: full GPU suite, smoke, headline bench, kernel trace of the timed replays
mkdir -p gpurun_out/r03final
run_step 500 r03final/gpu_tests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
run_step 200 r03final/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 600 r03final/bench python3 bench.py
run_step 300 r03final/trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03final/trace -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
echo ALLDONE
