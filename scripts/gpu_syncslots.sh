#!/bin/bash
# pptk_rx_batch over 2 vs 4 slots (PPTK_RX_SYNC_SLOTS), 1 M-frame calls,
# records registered, interleaved.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
for r in 1 2; do
  for k in 2 4; do
    step e2e_s${k}_$r 200 env E2E_REG_OUT=1 PPTK_RX_SYNC_SLOTS=$k python tools/e2e.py
  done
done
cat gpurun_out/steps.log
