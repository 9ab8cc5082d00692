#!/bin/bash
# Binned CMIX with coarser length groups (PPTK_RX_BIN_BOUNDS) against batch
# order, each in its own process (the knob is read once), twice over.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
for r in 1 2; do
  step bb_default_$r 200 python tools/opbench.py binned_ab --steps 10 --warmup 2
  step bb_241_$r 200 env PPTK_RX_BIN_BOUNDS=241,241,241,241,1521 python tools/opbench.py binned_ab --steps 10 --warmup 2
  step bb_113_$r 200 env PPTK_RX_BIN_BOUNDS=113,113,113,113,1521 python tools/opbench.py binned_ab --steps 10 --warmup 2
  step bb_497_$r 200 env PPTK_RX_BIN_BOUNDS=497,497,497,497,1521 python tools/opbench.py binned_ab --steps 10 --warmup 2
  step bb_241_1009_$r 200 env PPTK_RX_BIN_BOUNDS=241,241,241,1009,1521 python tools/opbench.py binned_ab --steps 10 --warmup 2
  step bb_one_$r 200 env PPTK_RX_BIN_BOUNDS=0,0,0,0,1521 python tools/opbench.py binned_ab --steps 10 --warmup 2
done
cat gpurun_out/steps.log
