source tools/gpu_step.sh
run_step 200 lp_a16 python -u tools/layer_profile.py --what a_model --precision fp16 --top 30
run_step 200 lp_a32 python -u tools/layer_profile.py --what a_model --precision fp32 --top 30
run_step 200 lp_f32 python -u tools/layer_profile.py --precision fp32 --top 40
echo ALLDONE
