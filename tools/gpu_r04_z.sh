source tools/gpu_step.sh
# round 4 closing: 32-bit pack index math; pack tests, full GPU suite, smoke, headline bench, training
mkdir -p gpurun_out/r04z
timeout -k 10 200 python -u -m pytest tests/test_gpu_pack.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04z/pack.log 2>&1 || { echo "PACK TESTS FAILED"; tail -30 gpurun_out/r04z/pack.log; exit 1; }
tail -1 gpurun_out/r04z/pack.log
run_step 900 r04z/gpu_tests python -u -X faulthandler -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider
run_step 200 r04z/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 400 r04z/bench python3 -X faulthandler bench.py
run_step 300 r04z/train_plan python -u train_net_unet.py --bench --steps 10 --warmup 3
LIC_PACK_PLAN=0 run_step 300 r04z/train_noplan python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 300 r04z/prof_train rocprofv3 --kernel-trace -d gpurun_out/r04z/prof -o run -- python3 train_net_unet.py --bench --steps 5 --warmup 2
echo ALLDONE
