source tools/gpu_step.sh
# WD kernel, compile-time 3x3 addressing (GEO 1): parity + timing vs the general path + counters
mkdir -p gpurun_out/r03geo
run_step 400 r03geo/test python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_resunit.py -x -q --timeout 120 --timeout-method thread -k "split_conv or resunit"
SH=wnsa3x3@64,rbws_conv2@128,rbneck3x3_96@64,wnsa3x3@16,cc3x3_224_128@16,cc3x3_128_32@16,qkv1x1@64
run_step 150 r03geo/bench_geo python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
LIC_WD_GEO=0 run_step 150 r03geo/bench_gen python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
run_step 150 r03geo/bench_geo2 python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
run_step 90 r03geo/sq1 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r03geo/sq1 -o sq1 -- python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 5 --only wnsa3x3@64
run_step 90 r03geo/sq2 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM --output-format csv -d gpurun_out/r03geo/sq2 -o sq2 -- python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 5 --only wnsa3x3@64
echo ALLDONE
