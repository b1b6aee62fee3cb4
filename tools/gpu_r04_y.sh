source tools/gpu_step.sh
# round 4: PackPlan (all of a training step's weight packs in one lic_pack_taps_batch launch)
mkdir -p gpurun_out/r04y
timeout -k 10 200 python -u -m pytest tests/test_gpu_pack.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04y/pack.log 2>&1 || { echo "PACK TESTS FAILED"; tail -30 gpurun_out/r04y/pack.log; exit 1; }
tail -1 gpurun_out/r04y/pack.log
run_step 400 r04y/train_tests python -u -m pytest tests/test_gpu_train_net.py tests/test_gpu_train.py tests/test_gpu_dist_train.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
run_step 300 r04y/train_plan python -u train_net_unet.py --bench --steps 10 --warmup 3
LIC_PACK_PLAN=0 run_step 300 r04y/train_noplan python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 300 r04y/train_plan2 python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 200 r04y/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 300 r04y/prof_train rocprofv3 --kernel-trace -d gpurun_out/r04y/prof -o run -- python3 train_net_unet.py --bench --steps 5 --warmup 2
echo ALLDONE
