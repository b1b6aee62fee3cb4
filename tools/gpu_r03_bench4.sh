source tools/gpu_step.sh
mkdir -p gpurun_out/r03b4
run_step 600 r03b4/bench python3 bench.py
run_step 300 r03b4/layers_f16_amodel python3 tools/layer_profile.py --precision fp16 --what a_model
run_step 300 r03b4/layers_f16 python3 tools/layer_profile.py --precision fp16
echo ALLDONE
