source tools/gpu_step.sh
mkdir -p gpurun_out/r03wdabl3
SH=wnsa3x3@64,rbws_conv2@128
run_step 120 r03wdabl3/abl_base python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
for v in halo0; do
  LIC_LIB=tools/native/liblic_wd_$v.so run_step 120 r03wdabl3/abl_$v python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
done
echo ALLDONE
