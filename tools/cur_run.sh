T=r05z
bash tools/gpu.sh $T \
 "pmcF|150|timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$T/pmcF -o run -- python3 tools/conv_bench.py --dtype fp16 --auto-only --iters 5 --only proj1x1@64,c1x1@128,wnsa3x3@16" \
 "pmcW|150|timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$T/pmcW -o run -- python3 tools/conv_bench.py --dtype fp16 --auto-only --iters 5 --only proj1x1@64,c1x1@128,wnsa3x3@16" \
 "pmcS|150|timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM --output-format csv -d gpurun_out/$T/pmcS -o run -- python3 tools/conv_bench.py --dtype fp16 --auto-only --iters 5 --only proj1x1@64,wnsa3x3@16"
