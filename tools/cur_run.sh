bash tools/gpu.sh r05x \
 'c16tests|300|python -u -m pytest tests/test_gpu_conv16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider' \
 'gdn|120|python -u tools/conv_bench.py --dtype fp16 --auto-only --gdn gdn --only gdn1x1@128,gdn1x1@32' \
 'gdnr1|120|python -u tools/conv_bench.py --dtype fp16 --auto-only --gdn gdn_r1 --only gdn1x1@128' \
 'cb1|120|python -u tools/conv_bench.py --dtype fp16 --auto-only --only proj1x1@64,c1x1@128,qkv1x1@64,qkv1x1@16' \
 'bench16|300|python -u bench.py --precision fp16 --no-extras'
