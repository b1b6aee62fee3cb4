source tools/gpu_step.sh
mkdir -p gpurun_out/r03xcd
export TMPDIR=/tmp
S=wnsa3x3@64,rbws_conv2@128,wnsa7x7@64,qkv1x1@64,conv5x5s2@128,wnsa3x3@16
run_step 300 r03xcd/split_tests python -u -m pytest tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread -k matches_fp32
run_step 120 r03xcd/xcd python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $S
LIC_WD_XCD=0 run_step 120 r03xcd/noxcd python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $S
run_step 120 r03xcd/xcd2 python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $S
run_step 90 r03xcd/pmc_fetch timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03xcd/pmc_fetch -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
run_step 90 r03xcd/pmc_write timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r03xcd/pmc_write -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
echo ALLDONE
