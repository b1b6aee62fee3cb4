source tools/gpu_step.sh
# round 4: per-layer breakdowns (eager, serialised op timing): fp16 a_model (the north star's fp16 leg),
# fp32x6 full forward
mkdir -p gpurun_out/r04t
run_step 300 r04t/layers_f16_amodel python -u tools/layer_profile.py --precision fp16 --what a_model --top 40
run_step 300 r04t/layers_fp32x6 python -u tools/layer_profile.py --precision fp32x6 --top 45
echo ALLDONE
