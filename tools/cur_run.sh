bash tools/gpu.sh r05zb \
 'c16tests|300|python -u -m pytest tests/test_gpu_conv16.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider' \
 'cb|120|python -u tools/conv_bench.py --dtype fp16 --auto-only --only wnsa3x3@16,cc3x3_224_128@16,cc3x3_336_224@16' \
 'bench16|300|python -u bench.py --precision fp16 --no-extras'
