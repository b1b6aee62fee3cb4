source tools/gpu_step.sh
# round 4 state of HEAD: full GPU suite, smoke, headline bench, kernel trace of the timed replays
mkdir -p gpurun_out/r04m
run_step 900 r04m/gpu_tests python -u -X faulthandler -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider
run_step 200 r04m/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 400 r04m/bench python3 -X faulthandler bench.py
run_step 300 r04m/trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m/trace -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
echo ALLDONE
