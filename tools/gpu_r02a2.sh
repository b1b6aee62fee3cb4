source tools/gpu_step.sh
run_step 300 na_ga python -u tools/split_net_accuracy.py
run_step 300 na_unet python -u tools/split_net_accuracy.py --arch net_unet_ha_hs
echo ALLDONE
