#!/bin/bash
# End-to-end rate with the record array reused by every call (an rx loop's
# pattern) against a fresh array per call (the earlier measurement).
source scripts/gpu_steps.sh
export TMPDIR=/tmp
for r in 1 2; do
  step e2e_reuse_$r 200 python tools/e2e.py
  step e2e_fresh_$r 200 env E2E_FRESH_OUT=1 python tools/e2e.py
done
step e2e_trace_staged 200 env E2E_CFGS=c64 E2E_MODES=staged rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/e2e_tr_staged -o run --output-format csv -- python tools/e2e.py
cat gpurun_out/steps.log
