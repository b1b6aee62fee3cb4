# Round-2 closing validation of HEAD: 16x16-latent conv kernel times (exact fp32 vs fp32x3 split),
# GPU suite, smoke, default bench, rocprof kernel trace of the headline leg, coder bench.
source tools/gpu_step.sh
mkdir -p gpurun_out/prof
S16=ru3x3_64@16,wnsa3x3@16,cc3x3_224_128@16,cc3x3_128_48@16,cc3x3_336_224@16,ru1x1_128_64@16,ru1x1_64_128@16,lin512_128@16
run_step 200 cb16_fp32 rocprofv3 --kernel-trace --stats -d gpurun_out/cb16_fp32 -o run -- python3 tools/conv_bench.py --dtype fp32 --auto-only --iters 50 --only $S16
run_step 200 cb16_fp32x3 rocprofv3 --kernel-trace --stats -d gpurun_out/cb16_fp32x3 -o run -- python3 tools/conv_bench.py --dtype fp32x3 --auto-only --iters 50 --only $S16
run_step 900 gpu_tests python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread
run_step 200 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
run_step 400 bench python -u bench.py
run_step 300 prof rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-extras --steps 10 --warmup 3
run_step 200 coder python -u tools/coder_bench.py
echo ALLDONE
