#!/bin/bash
# SQ instruction counters of one config under diagnostic tune flags
# (PPTK_RX_TUNE, include/pptk_rx.h: 16 = skip the per-frame phase, 8 = skip
# record stores), e.g.  gpurun -- bash profiles/r03/scripts/gpu_sq_diag.sh cmix 32 48 40
source scripts/gpu_steps.sh
export TMPDIR=/tmp
c=$1
shift
for t in "$@"; do
  PPTK_RX_TUNE=$t step sq_${c}_$t 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex rx_kernel -d gpurun_out/sq_${c}_$t -o run --output-format csv -- python bench.py --only $c --steps 2 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0
done
cat gpurun_out/steps.log
