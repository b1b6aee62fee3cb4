# 8x8 x 64 split tile capped at 80 KB LDS (two workgroups per CU): latent conv timings, GPU suite, bench + trace.
source tools/gpu_step.sh
mkdir -p gpurun_out/prof4
S16=ru3x3_64@16,wnsa3x3@16,cc3x3_224_128@16,cc3x3_128_48@16,cc3x3_336_224@16
run_step 200 cb16_x3b rocprofv3 --kernel-trace --stats -d gpurun_out/cb16_x3b -o run -- python3 tools/conv_bench.py --dtype fp32x3 --auto-only --iters 50 --only $S16
run_step 900 gpu_tests4 python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread
run_step 200 smoke4 python -u -c "import __graft_entry__ as g; g.smoke()"
run_step 400 bench4 python -u bench.py
run_step 300 prof4 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run -- python3 bench.py --no-extras --steps 10 --warmup 3
echo ALLDONE
