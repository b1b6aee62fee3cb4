source tools/gpu_step.sh
# round 4: virtual-tap 1x1 with one sign flip per launch + unrolled 6-tile epilogue: parity + timing + bench
mkdir -p gpurun_out/r04i
run_step 400 r04i/split python -u -m pytest tests/test_gpu_split.py tests/test_gpu_resunit.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
run_step 200 r04i/conv python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only qkv1x1@64,proj1x1@64,c1x1@128,wnsa3x3@64 --iters 30
run_step 500 r04i/net python -u -m pytest tests/test_gpu_net.py tests/test_gpu_configs.py tests/test_gpu_coder.py -m gpu -v -x --timeout 170 --timeout-method thread -p no:cacheprovider
run_step 300 r04i/bench python3 bench.py --no-extras --precision fp32x6
echo ALLDONE
