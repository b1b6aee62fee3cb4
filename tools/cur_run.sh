bash tools/gpu.sh r05w \
 'c16tests|300|python -u -m pytest tests/test_gpu_conv16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider' \
 'cb|150|python -u tools/conv_bench.py --dtype fp16 --auto-only --only wnsa3x3@64,rbws_conv2@128,wnsa7x7@64,conv5x5s2@128,rbneck3x3_96@64' \
 'cbnorot|150|env LIC_C16_ROT=0 python -u tools/conv_bench.py --dtype fp16 --auto-only --only wnsa3x3@64,rbws_conv2@128,wnsa7x7@64,conv5x5s2@128,rbneck3x3_96@64' \
 'bench16|300|python -u bench.py --precision fp16 --no-extras'
