# r03: where the weights-direct fp32x6 conv spends its time (ablation builds + SQ counters)
source tools/gpu_step.sh
mkdir -p gpurun_out/r03wdabl
SH=wnsa3x3@64,rbws_conv2@128
run_step 120 r03wdabl/abl_base python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
for v in nosplit nob onlymfma; do
  LIC_LIB=tools/native/liblic_wd_$v.so run_step 120 r03wdabl/abl_$v python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
done
run_step 90 r03wdabl/pmc1 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/r03wdabl/pmc1 -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
run_step 90 r03wdabl/pmc2 timeout -s KILL 80 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r03wdabl/pmc2 -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
run_step 90 r03wdabl/pmc3 timeout -s KILL 80 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/r03wdabl/pmc3 -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
echo ALLDONE
