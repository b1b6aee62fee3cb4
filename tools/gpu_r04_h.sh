source tools/gpu_step.sh
# round 4: 192-channel WD 3x3 ablations on one box (timing only): base, L2-resident halo (32), no split (1), no B loads (2)
mkdir -p gpurun_out/r04h
SH=wnsa3x3@64,rbws_conv2@128
run_step 150 r04h/base python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
for v in 32 1 2; do
  LIC_LIB=tools/native/liblic_bigabl$v.so run_step 150 r04h/abl$v python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
done
run_step 150 r04h/base2 python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
echo ALLDONE
