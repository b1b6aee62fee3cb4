source tools/gpu_step.sh
run_step 900 gpu_tests python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread
run_step 200 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
echo ALLDONE
