source tools/gpu_step.sh
# round 4: LDS weight ring (LB) for the 192-channel WD 3x3 / 7x7 -- correctness, A/B vs the register path, bench
mkdir -p gpurun_out/r04g
run_step 300 r04g/split_lb python -u -m pytest tests/test_gpu_split.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "test_split_conv_matches_fp32"
for v in 1 2 1; do
  LIC_WD_BN192=$v run_step 200 r04g/conv_bn192_$v python -u tools/conv_bench.py --dtype fp32x6 --auto-only --only wnsa3x3@64,wnsa7x7@64,rbws_conv2@128 --iters 30
done
run_step 300 r04g/bench python3 bench.py --no-extras --precision fp32x6
run_step 90 r04g/sq1 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r04g/sq1 -o sq1 -- python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 5 --only wnsa3x3@64
echo ALLDONE
