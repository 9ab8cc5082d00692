#!/bin/bash
# Branch-free GATHER descriptors + length-group launches: parity, A/B against
# the previous build (build/ab_old), then a short bench.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
export AB_LIBS=old=build/ab_old/libpptkrx.so,sip64=build/ab_sip64/libpptkrx.so
step gputests 900 python -m pytest tests -x -q -m gpu
step ab_cmix 300 python tools/ab.py cmix 3:33 old:3:33 4:33 5:33 11:33
step ab_cmix_mixed 300 env AB_MIXED=1 AB_LIBS= python tools/ab.py cmix -1:-1 3:33 11:33 -1:0 -1:1
step ab_c1500g 300 python tools/ab.py c1500g 3:33 old:3:33
step ab_c64 300 python tools/ab.py c64 0:0 sip64:0:0 old:0:0 0:32 1:0
step bench 600 python bench.py --steps 10 --warmup 2 --cpu-seconds 4
step pmc_c64 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex rx_kernel -d gpurun_out/pmc_c64_a -o run --output-format csv -- python bench.py --only c64 --steps 2 --warmup 1 --no-cpu --no-check --no-membench --settle 0
cat gpurun_out/steps.log
