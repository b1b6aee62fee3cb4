source tools/gpu_step.sh
# round 4: lic_pack_taps (one launch per weight pack) -- pack bit-exactness first, then the full GPU
# suite, smoke, headline bench and the training step with its kernel trace
mkdir -p gpurun_out/r04x
timeout -k 10 200 python -u -m pytest tests/test_gpu_pack.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04x/pack.log 2>&1 || { echo "PACK TESTS FAILED"; tail -30 gpurun_out/r04x/pack.log; exit 1; }
tail -1 gpurun_out/r04x/pack.log
run_step 900 r04x/gpu_tests python -u -X faulthandler -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider
run_step 200 r04x/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 400 r04x/bench python3 -X faulthandler bench.py
run_step 300 r04x/train_bench python -u train_net_unet.py --bench --steps 10 --warmup 3
run_step 300 r04x/prof_train rocprofv3 --kernel-trace -d gpurun_out/r04x/prof -o run -- python3 train_net_unet.py --bench --steps 5 --warmup 2
echo ALLDONE
