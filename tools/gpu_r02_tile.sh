# 8x8 x 192 split tile for stride-2 / large-halo convolutions: full GPU suite, smoke, headline bench + trace.
source tools/gpu_step.sh
mkdir -p gpurun_out/prof3
run_step 900 gpu_tests3 python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread
run_step 200 smoke3 python -u -c "import __graft_entry__ as g; g.smoke()"
run_step 400 bench3 python -u bench.py
run_step 300 prof3 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run -- python3 bench.py --no-extras --steps 10 --warmup 3
echo ALLDONE
