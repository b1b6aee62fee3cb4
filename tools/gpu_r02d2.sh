source tools/gpu_step.sh
run_step 500 t_split python -u -m pytest -q --tb=short --timeout 300 --timeout-method thread tests/test_gpu_split.py -s
run_step 200 b_x3 python -u bench.py --no-extras --precision fp32x3
run_step 300 lp_x3 python -u tools/layer_profile.py --precision fp32x3 --top 30
echo ALLDONE
