#!/bin/bash
# Host path: end-to-end rate of C64, current library against the previous
# build and a 1 MiB copy-out piece variant, interleaved processes.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
export E2E_CFGS=c64
for r in 1 2 3 4; do
  step e2e_new_$r 200 python tools/e2e.py
  step e2e_old_$r 200 env E2E_LIB=abl/old/libpptkrx.so python tools/e2e.py
  step e2e_p1m_$r 200 env E2E_LIB=abl/p1m/libpptkrx.so python tools/e2e.py
done
cat gpurun_out/steps.log
