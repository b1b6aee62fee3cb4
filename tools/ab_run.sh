set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn.py tests/test_gpu_net.py -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
timeout -k 10 120 python -u tools/attn_bench.py > gpurun_out/attn.log 2>&1 || { echo ATTN FAILED; tail gpurun_out/attn.log; exit 1; }
cat gpurun_out/attn.log
timeout -k 10 200 python -u bench.py --no-extras --steps 30 > gpurun_out/ab.log 2>&1 || { echo BENCH FAILED; tail gpurun_out/ab.log; exit 1; }; tail -1 gpurun_out/ab.log | cut -c1-120
