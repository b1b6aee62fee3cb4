# round-end measurement call: headline bench, replay-only traces, PMC pairs (tools/gpu.sh steps)
T=${1:-r05s}
bash tools/gpu.sh $T \
 "bench|600|python -u bench.py" \
 "profh|300|rocprofv3 --kernel-trace -d gpurun_out/$T/prof_h -o run -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 1" \
 "profa|300|rocprofv3 --kernel-trace -d gpurun_out/$T/prof_a -o run -- python3 bench.py --precision fp16 --profile --profile-a-model --steps 5 --warmup 1" \
 "pmcF16|150|timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$T/pmcF16 -o run -- python3 tools/conv_bench.py --dtype fp16 --auto-only --iters 5 --only wnsa3x3@64" \
 "pmcW16|150|timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$T/pmcW16 -o run -- python3 tools/conv_bench.py --dtype fp16 --auto-only --iters 5 --only wnsa3x3@64" \
 "pmcF6|150|timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$T/pmcF6 -o run -- python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 5 --only wnsa3x3@64" \
 "pmcW6|150|timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$T/pmcW6 -o run -- python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 5 --only wnsa3x3@64"
