set -o pipefail
mkdir -p gpurun_out/prof_train
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_net.py -v --timeout 250 --timeout-method thread > gpurun_out/train3.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" gpurun_out/train3.log | tail; exit 1; }
tail -1 gpurun_out/train3.log
timeout -k 10 240 python -u train_net_unet.py --bench --steps 10 --warmup 3 > gpurun_out/train_bench_f16.log 2>&1 || { echo "BENCH16 FAILED"; tail -20 gpurun_out/train_bench_f16.log; exit 1; }
tail -1 gpurun_out/train_bench_f16.log
timeout -k 10 240 python -u train_net_unet.py --bench --steps 5 --warmup 2 --precision fp32 > gpurun_out/train_bench_f32.log 2>&1 || { echo "BENCH32 FAILED"; tail -20 gpurun_out/train_bench_f32.log; exit 1; }
tail -1 gpurun_out/train_bench_f32.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run -- python3 train_net_unet.py --bench --steps 5 --warmup 2 > gpurun_out/prof_train.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/prof_train.log; exit 1; }
echo ALLDONE
