# One parametrised GPU-box runner (replaces the per-call tools/gpu_r0x_*.sh scripts).
# usage: bash tools/gpu.sh TAG 'name|seconds|command' ['name|seconds|command' ...]
# Each step runs under its own time limit (tools/gpu_step.sh: a timeout / abort / crash ends the
# script, an ordinary failure is recorded and the next step runs); logs go to gpurun_out/TAG/name.log.
# Environment for one step: prefix the command with `env VAR=VALUE` (never after a profiler's `--`).
source tools/gpu_step.sh
tag=$1
shift
mkdir -p "gpurun_out/$tag"
for st in "$@"; do
  IFS='|' read -r name secs cmd <<< "$st"
  eval "run_step $secs $tag/$name $cmd"
done
echo ALLDONE
