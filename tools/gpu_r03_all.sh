source tools/gpu_step.sh
# round-3 session-2 validation: full GPU suite, headline bench, PMC of the roofline kernel, kernel trace, layer timings
mkdir -p gpurun_out/r03all
run_step 500 r03all/gpu_tests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
run_step 200 r03all/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 600 r03all/bench python3 bench.py
SH=wnsa3x3@64,wnsa7x7@64,wnsa7x7@16,conv5x5s2@32,qkv1x1@64,proj1x1@64,gdn1x1@128,wnsa3x3@16,cc3x3_224_128@16,rbws_conv2@128,conv5x5s2@128
run_step 150 r03all/conv_geo python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
LIC_WD_GEO=0 run_step 150 r03all/conv_gen python3 tools/conv_bench.py --dtype fp32x6 --auto-only --iters 30 --only $SH
run_step 90 r03all/pmc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03all/pmc_fetch -o f -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
run_step 90 r03all/pmc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r03all/pmc_write -o w -- python3 tools/conv_bench.py --dtype fp32x6 --iters 5 --auto-only --only wnsa3x3@64
run_step 300 r03all/trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03all/trace -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
LIC_FUSED_RU=0 run_step 200 r03all/bench_noru python3 bench.py --precision fp32x6 --no-extras
echo ALLDONE
