set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { echo "TESTS FAILED"; tail -5 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH FAILED; exit 1; }
timeout -k 10 300 python -u eval_net.py --synthetic-kodak --graph --precision fp16 > gpurun_out/kodak_sweep.log 2>&1 || { echo SWEEP FAILED; exit 1; }
timeout -k 10 200 python -u bench.py --no-extras --post-processing --steps 5 --warmup 2 > gpurun_out/bench_han.log 2>&1 || { echo HAN BENCH FAILED; exit 1; }
timeout -k 10 200 python -u tools/coder_bench.py > gpurun_out/coder_bench.log 2>&1 || { echo CODER BENCH FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --profile --steps 5 > gpurun_out/prof.log 2>&1 || { echo PROF FAILED; exit 1; }
echo ALLDONE
