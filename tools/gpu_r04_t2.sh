source tools/gpu_step.sh
# round 4: per-layer breakdowns again with layer_profile charging nested ops their self time
mkdir -p gpurun_out/r04t2
run_step 300 r04t2/layers_f16_amodel python -u tools/layer_profile.py --precision fp16 --what a_model --top 40
run_step 300 r04t2/layers_fp32x6 python -u tools/layer_profile.py --precision fp32x6 --top 45
echo ALLDONE
