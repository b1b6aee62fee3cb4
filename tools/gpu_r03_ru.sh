source tools/gpu_step.sh
# fused ResidualUnit: parity + timing; then the WD-kernel ablations / counters
mkdir -p gpurun_out/r03ru gpurun_out/r03wdabl4
run_step 300 r03ru/test python3 -u -m pytest tests/test_gpu_resunit.py -x -v --timeout 120 --timeout-method thread
run_step 120 r03ru/bench python3 tools/resunit_bench.py
SH=wnsa3x3@64,wnsa3x3@16,ru3x3_64@16
run_step 150 r03wdabl4/base python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
for v in 1 2 4 8 16 15 32; do
  LIC_LIB=tools/native/liblic_wdabl$v.so run_step 150 r03wdabl4/abl$v python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
done
run_step 90 r03wdabl4/sq1 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r03wdabl4/sq1 -o sq1 -- python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 5 --only wnsa3x3@64
run_step 90 r03wdabl4/sq2 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM --output-format csv -d gpurun_out/r03wdabl4/sq2 -o sq2 -- python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 5 --only wnsa3x3@64
echo ALLDONE
