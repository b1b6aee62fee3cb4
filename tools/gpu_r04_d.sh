source tools/gpu_step.sh
# round 4: correctness of the new WD paths (tap split, s2 GEO, 192-ch tiles, first conv), slice-loop
# conv A/B, then the bench segfault hunt (faulthandler), serial vs concurrent ResidualUnits
mkdir -p gpurun_out/r04d
run_step 400 r04d/split_all python -u -m pytest tests/test_gpu_split.py tests/test_gpu_resunit.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider
for v in 0 1; do
  LIC_WD_TAPSPLIT=$v run_step 200 r04d/conv_tapsplit_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa3x3@16,cc3x3_224_128@16,cc3x3_336_224@16,ru3x3_64@16 --iters 30
done
run_step 300 r04d/net_tests python -u -X faulthandler -m pytest tests/test_gpu_net.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "fp32_parity and not kodak"
run_step 300 r04d/bench_serial python3 -X faulthandler bench.py --no-extras --precision fp32x6 --steps 5
LIC_CONCURRENT_RU=1 run_step 300 r04d/bench_side python3 -X faulthandler bench.py --no-extras --precision fp32x6 --steps 5
echo ALLDONE
