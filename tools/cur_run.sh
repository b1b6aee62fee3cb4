bash tools/gpu.sh r05q \
 'c16tests|300|python -u -m pytest tests/test_gpu_conv16.py tests/test_gpu_attn.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider' \
 'gdn|120|python -u tools/conv_bench.py --dtype fp16 --auto-only --gdn gdn --only gdn1x1@128,gdn1x1@32' \
 'cb7|120|python -u tools/conv_bench.py --dtype fp16 --auto-only --only wnsa7x7@64,wnsa3x3@64' 'cb7off|120|env LIC_CONV16_7X7=0 python -u tools/conv_bench.py --dtype fp16 --auto-only --only wnsa7x7@64' 'bench16|300|python -u bench.py --precision fp16 --no-extras' \
 'profa|300|rocprofv3 --kernel-trace -d gpurun_out/r05q/prof_a -o run -- python3 bench.py --precision fp16 --profile --profile-a-model --steps 5 --warmup 1'
