source tools/gpu_step.sh
run_step 300 lp_x3 python -u tools/layer_profile.py --precision fp32x3 --top 40
run_step 600 bench_all python -u bench.py
echo ALLDONE
