source tools/gpu_step.sh
# round 4: counters of the 192-channel WD 3x3 (roofline kernel) and the virtual-tap 1x1 (qkv), B=32
mkdir -p gpurun_out/r04f
for S in wnsa3x3@64 qkv1x1@64; do
  T=${S%%@*}
  run_step 90 r04f/${T}_sq1 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r04f/${T}_sq1 -o sq1 -- python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 5 --only $S
  run_step 90 r04f/${T}_sq2 timeout -s KILL 80 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM --output-format csv -d gpurun_out/r04f/${T}_sq2 -o sq2 -- python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 5 --only $S
  run_step 90 r04f/${T}_tcp timeout -s KILL 80 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/r04f/${T}_tcp -o tcp -- python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 5 --only $S
  run_step 90 r04f/${T}_fetch timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04f/${T}_fetch -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only $S
  run_step 90 r04f/${T}_write timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r04f/${T}_write -o pmc -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only $S
done
echo ALLDONE
# ablations (timing only; outputs wrong): WD_ABL 8 no epilogue, 1 no in-loop split/halo prefetch, 2 no B loads, 16 no MFMA
SH=wnsa3x3@64,qkv1x1@64,proj1x1@64,c1x1@128
run_step 150 r04f/abl_base python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
for v in 8 1 2 16; do
  LIC_LIB=tools/native/liblic_vtabl$v.so run_step 150 r04f/abl$v python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
done
run_step 175 r04f/rccl_graph python -u -m pytest tests/test_gpu_dist_train.py::test_graph_step_with_rccl_allreduce_matches_eager -v -s --timeout 165 --timeout-method thread -p no:cacheprovider
echo ALLDONE2
