source tools/gpu_step.sh
mkdir -p gpurun_out/r03full2
run_step 1000 r03full2/gpu_tests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
run_step 300 r03full2/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 400 r03full2/train_default python -u train_net_unet.py --bench --steps 20 --warmup 5
echo ALLDONE
