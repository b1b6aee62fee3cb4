# r03: where the fp32x6 split conv spends its time (ablation builds, PMC pass); outputs under gpurun_out/r03abl/
source tools/gpu_step.sh
mkdir -p gpurun_out/r03abl
SH=wnsa3x3@64,wnsa3x3@16,cc3x3_336_224@16,ru3x3_64@16
for v in base nodma noepi nosplit nomfma nofrag onlymfma; do
  LIC_LIB=tools/native/liblic_$v.so run_step 120 r03abl/abl_$v python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
done
run_step 120 r03abl/ref_fp32x3 python3 tools/conv_bench.py --dtype fp32x3 --auto-only --iters 30 --only $SH
run_step 120 r03abl/ref_fp32 python3 tools/conv_bench.py --dtype fp32 --auto-only --iters 30 --only $SH
run_step 60 r03abl/counters rocprofv3 -L
LIC_LIB=tools/native/liblic_base.so run_step 90 r03abl/pmc1 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/r03abl/pmc1 -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
LIC_LIB=tools/native/liblic_base.so run_step 90 r03abl/pmc2 timeout -s KILL 80 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r03abl/pmc2 -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
echo ALLDONE
