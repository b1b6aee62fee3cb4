source tools/gpu_step.sh
run_step 200 acc3 python -u tools/split_accuracy.py
run_step 200 acc3p python -u tools/split_accuracy.py --positive
run_step 200 acc7 python -u tools/split_accuracy.py --k 7
run_step 200 b_split6 python -u bench.py --no-extras --precision fp32x6
echo ALLDONE
