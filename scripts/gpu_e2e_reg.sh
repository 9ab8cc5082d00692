#!/bin/bash
# Registered record arrays: host-batch GPU tests, then the end-to-end rate
# with the record array registered against reused-but-unregistered.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gt_host 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "host or ring or staged or pool or direct or example or registered"
for r in 1 2; do
  step e2e_reg_$r 200 env E2E_REG_OUT=1 python tools/e2e.py
  step e2e_reuse_$r 200 python tools/e2e.py
done
cat gpurun_out/steps.log
