source tools/gpu_step.sh
mkdir -p gpurun_out/r04p
run_step 300 r04p/add_probe python -u tools/train_add_probe.py
echo ALLDONE
