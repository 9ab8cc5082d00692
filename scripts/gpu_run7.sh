#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step ab_diag 600 python tools/ab.py c1500 3:0 3:8 3:24 3:25 4:24 6:24 6:25
step pmc_a 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex rx_kernel -d gpurun_out/pmc_a -o run --output-format csv -- python bench.py --only c1500 --steps 2 --warmup 1 --no-cpu --no-check --no-membench
step pmc_b 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex rx_kernel -d gpurun_out/pmc_b -o run --output-format csv -- python bench.py --only c1500 --steps 2 --warmup 1 --no-cpu --no-check --no-membench
step pmc_c 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-include-regex rx_kernel -d gpurun_out/pmc_c -o run --output-format csv -- python bench.py --only c1500 --steps 2 --warmup 1 --no-cpu --no-check --no-membench
cat gpurun_out/ab_*.log | grep '^{'
