# The GPU call of the moment (overwritten per call; results under gpurun_out/<tag>/).
bash tools/gpu.sh r05i \
 'c16tests|300|python -u -m pytest tests/test_gpu_conv16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider' \
 'st6|120|env LIC_LIB=tools/native/liblic_c16stamp.so python -u tools/conv16_stamps.py wnsa3x3 rbws_conv2' \
 'stnost|120|env LIC_LIB=tools/native/liblic_c16nost.so python -u tools/conv16_stamps.py wnsa3x3 rbws_conv2' \
 'cb16|120|python -u tools/conv_bench.py --dtype fp16 --auto-only --only wnsa3x3@64,rbws_conv2@128,conv5x5s2@128' \
 'bench16|300|python -u bench.py --precision fp16 --no-extras' \
 'ops|600|python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_ops2.py tests/test_gpu_train.py tests/test_gpu_train_net.py tests/test_gpu_wgrad.py -x -q --timeout 170 --timeout-method thread -p no:cacheprovider' \
 'train|300|python -u train_net_unet.py --bench --steps 10 --warmup 3'
