source tools/gpu_step.sh
run_step 300 t_ops python -u -m pytest -q -x --tb=short --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_ops2.py tests/test_gpu_net.py
run_step 200 b_def python -u bench.py --no-extras --precision fp32
LIC_LIB=tools/native/liblic_h1x1none.so run_step 200 b_none python -u bench.py --no-extras --precision fp32
LIC_LIB=tools/native/liblic_h1x1all.so run_step 200 b_all16 python -u bench.py --no-extras --precision fp16
run_step 200 b_def16 python -u bench.py --no-extras --precision fp16
run_step 300 t_graph python -u -m pytest -q -x --tb=short --timeout 300 --timeout-method thread tests/test_gpu_train_net.py -k graph -s
echo ALLDONE
