# source me: run_step SECONDS LOGNAME cmd...  — runs one GPU step under its own time limit;
# a non-zero ordinary exit is recorded and the script goes on, a timeout / abort / crash ends it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run_step() {
  local secs=$1 log=$2; shift 2
  echo "== $log: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$log.log" 2>&1
  local rc=$?
  echo "   rc=$rc; $(tail -c 600 gpurun_out/$log.log | tail -3)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $log (rc=$rc)"; exit $rc; fi
  return 0
}
