set -o pipefail
mkdir -p gpurun_out
for cfg in 256:0 192:0 128:0 256:256 192:256 256:0; do m=${cfg%%:*}; n=${cfg#*:}
LIC_HALO_MID=$m LIC_HALO_N32=$n timeout -k 10 200 python -u bench.py --no-extras --steps 30 > gpurun_out/ab.log 2>&1 || { echo BENCH FAILED; tail gpurun_out/ab.log; exit 1; }; echo "mid=$m n32=$n $(tail -1 gpurun_out/ab.log | cut -c1-120)"; done
