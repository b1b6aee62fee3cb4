# The GPU call of the moment (overwritten per call; results under gpurun_out/<tag>/).
bash tools/gpu.sh r05k \
 'c16tests|300|python -u -m pytest tests/test_gpu_conv16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider' \
 'cb16|120|python -u tools/conv_bench.py --dtype fp16 --auto-only --only qkv1x1@64,proj1x1@64,gdn1x1@128,qkv1x1@16,gdn1x1@32' \
 'bench16|300|python -u bench.py --precision fp16 --no-extras' \
 'layers16|300|python -u tools/layer_profile.py --precision fp16 --what a_model' \
 'probe|120|python -u tools/capture_fork_probe.py'
