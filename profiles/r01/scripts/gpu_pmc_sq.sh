#!/bin/bash
# SQ instruction counters (VALU/SALU/LDS/VMEM per dispatch) for one config:
#   gpurun -- bash profiles/r01/scripts/gpu_pmc_sq.sh c64
source scripts/gpu_steps.sh
export TMPDIR=/tmp
c=${1:-c64}
step pmc_sq_$c 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex rx_kernel -d gpurun_out/pmc_sq_$c -o run --output-format csv -- python bench.py --only $c --steps 2 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --settle 0
cat gpurun_out/steps.log
