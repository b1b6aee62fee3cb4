source tools/gpu_step.sh
run_step 200 acc3 python -u tools/split_accuracy.py
run_step 200 acc7 python -u tools/split_accuracy.py --k 7
LIC_LIB=tools/native/liblic_p0.so run_step 200 acc3_p0 python -u tools/split_accuracy.py
LIC_LIB=tools/native/liblic_p0.so run_step 200 acc7_p0 python -u tools/split_accuracy.py --k 7
run_step 200 cb_s1 python -u tools/conv_bench.py --dtype fp32x3 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128
LIC_LIB=tools/native/liblic_p0.so run_step 200 cb_s1_p0 python -u tools/conv_bench.py --dtype fp32x3 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128
run_step 400 t_split python -u -m pytest -q --tb=line --timeout 300 --timeout-method thread tests/test_gpu_split.py -s -k net_parity
LIC_LIB=tools/native/liblic_p0.so run_step 400 t_split_p0 python -u -m pytest -q --tb=line --timeout 300 --timeout-method thread tests/test_gpu_split.py -s -k net_parity
echo ALLDONE
