source tools/gpu_step.sh
# round 4, first GPU call: the new fp32x6 parity tests (cfg3 / cfg4 / B=32 round trip), the
# measured-bits rate bar, the fused-bias wgrad tests, smoke (strict 0 flips), the headline bench
mkdir -p gpurun_out/r04a
run_step 900 r04a/gpu_tests python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_net.py tests/test_gpu_split.py tests/test_gpu_coder.py tests/test_gpu_wgrad.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider
run_step 200 r04a/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 600 r04a/bench python3 bench.py
echo ALLDONE
