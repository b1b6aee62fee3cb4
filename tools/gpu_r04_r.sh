source tools/gpu_step.sh
# round 4 closing state: 7-tap rows on 96-channel tiles (A/B), full GPU suite, smoke, headline bench,
# kernel trace of the timed replays
mkdir -p gpurun_out/r04r
for v in 0 1; do
  LIC_WD_BN96=$v run_step 200 r04r/conv_bn96_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa7x7@16,wnsa3x3@16,rbneck3x3_96@64 --iters 30
done
run_step 900 r04r/gpu_tests python -u -X faulthandler -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider
run_step 200 r04r/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 400 r04r/bench python3 -X faulthandler bench.py
run_step 300 r04r/trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04r/trace -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
echo ALLDONE
