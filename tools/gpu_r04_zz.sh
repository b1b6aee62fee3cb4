source tools/gpu_step.sh
# round 4: headline bench re-check on another box (r04z's box ran the unchanged roofline kernel 20 % slow)
mkdir -p gpurun_out/r04zz
run_step 200 r04zz/conv python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa3x3@64 --iters 30
run_step 400 r04zz/bench python3 -X faulthandler bench.py
echo ALLDONE
