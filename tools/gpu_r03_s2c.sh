source tools/gpu_step.sh
# patch path for the image's first conv; full suite; headline bench
mkdir -p gpurun_out/r03s2c
run_step 200 r03s2c/patch_tests python3 -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread -k "patch"
run_step 500 r03s2c/gpu_tests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
run_step 200 r03s2c/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 600 r03s2c/bench python3 bench.py
LIC_PATCHES=0 run_step 200 r03s2c/bench_nopatch python3 bench.py --precision fp32x6 --no-extras
echo ALLDONE
