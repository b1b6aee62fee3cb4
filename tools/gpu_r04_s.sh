source tools/gpu_step.sh
# round 4: conv_a of the 16x16 Win_noShift_Attention blocks / SWAtten on a side stream (LIC_CONCURRENT_RU=1)
mkdir -p gpurun_out/r04s
run_step 300 r04s/bench_0 python3 -X faulthandler bench.py --no-extras --precision fp32x6
LIC_CONCURRENT_RU=1 run_step 300 r04s/bench_1 python3 -X faulthandler bench.py --no-extras --precision fp32x6
LIC_CONCURRENT_RU=1 run_step 400 r04s/net python -u -X faulthandler -m pytest tests/test_gpu_split.py tests/test_gpu_net.py tests/test_gpu_determinism.py tests/test_gpu_coder.py -m gpu -q -x --timeout 170 --timeout-method thread -p no:cacheprovider
run_step 300 r04s/bench_0b python3 -X faulthandler bench.py --no-extras --precision fp32x6
LIC_CONCURRENT_RU=1 run_step 300 r04s/bench_1b python3 -X faulthandler bench.py --no-extras --precision fp32x6
echo ALLDONE
