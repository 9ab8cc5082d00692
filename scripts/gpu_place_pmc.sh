#!/bin/bash
# Record-buffer placement experiment under PMC (tools/place_probe.py --matrix):
# fabric destination of L2 misses (local DRAM vs GMI) and TLB behaviour of
# the C1500 launch into each of 10 separately allocated record buffers.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
step place_pmc1 200 rocprofv3 --pmc TCC_EA0_WRREQ_WRITE_DRAM_sum TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_GMI_32B_sum --kernel-include-regex rx_kernel -d $O/p1 -o run --output-format csv -- python tools/place_probe.py --matrix 10 --reps 1
step place_pmc2 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_sum --kernel-include-regex rx_kernel -d $O/p2 -o run --output-format csv -- python tools/place_probe.py --matrix 10 --reps 1
cat gpurun_out/steps.log
