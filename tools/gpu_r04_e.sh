source tools/gpu_step.sh
# round 4 (session 2) state of HEAD: full GPU suite (the RCCL graph-capture test on its own, last), smoke,
# headline bench, kernel trace of the timed replays
mkdir -p gpurun_out/r04e
G=tests/test_gpu_dist_train.py::test_graph_step_with_rccl_allreduce_matches_eager
run_step 900 r04e/gpu_tests python -u -X faulthandler -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider --deselect $G
run_step 200 r04e/smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
run_step 400 r04e/bench python3 -X faulthandler bench.py
run_step 300 r04e/trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04e/trace -o trace -- python3 bench.py --precision fp32x6 --profile --steps 5 --warmup 2
run_step 175 r04e/rccl_graph python -u -m pytest $G -v -s --timeout 165 --timeout-method thread -p no:cacheprovider
echo ALLDONE
