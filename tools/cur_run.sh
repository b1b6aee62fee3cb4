# The GPU call of the moment (overwritten per call; results under gpurun_out/<tag>/).
bash tools/gpu.sh r05e \
 'g16one|90|python -u -m pytest tests/test_gpu_conv16.py -x -v --timeout 60 --timeout-method thread -p no:cacheprovider -k "test_gemm16_vs_torch_fp32 and 192-192-1-16"' \
 'cbq|90|python -u tools/conv_bench.py --dtype fp16 --auto-only --only proj1x1@64,qkv1x1@64,gdn1x1@128,wnsa3x3@64' \
 'c16tests|400|python -u -m pytest tests/test_gpu_conv16.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider' \
 'cb_new|200|python -u tools/conv_bench.py --dtype fp16 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128,rbneck3x3_96@64,conv5x5s2@128,qkv1x1@64,proj1x1@64,gdn1x1@128' \
 'bench16|300|python -u bench.py --precision fp16 --no-extras' \
 'layers16|300|python -u tools/layer_profile.py --precision fp16 --what a_model'
