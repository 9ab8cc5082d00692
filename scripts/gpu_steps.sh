#!/bin/bash
# Helper for gpurun calls: run named steps in order, each under its own
# timeout; keep going after an ordinary failure (exit 1-5: a failed test or
# assertion), stop the whole call after anything crash-like (timeout 124,
# kill 137, abort 134, segfault 139, ...), so nothing else touches the GPU.
#   source scripts/gpu_steps.sh; step NAME SECONDS cmd args...
mkdir -p gpurun_out
step() {
  local name=$1 t=$2
  shift 2
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a gpurun_out/steps.log
  case $rc in
    0|1|2|3|4|5) return 0 ;;
    *) echo "STOP: $name exited $rc"; exit "$rc" ;;
  esac
}
