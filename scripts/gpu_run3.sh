#!/bin/bash
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step gputests 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu
step bench 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 10
step c64_plain 300 env PPTK_RX_TUNE=0 python bench.py --only c64 --steps 20 --no-cpu --no-check
step c1500_plain 300 env PPTK_RX_TUNE=0 python bench.py --only c1500 --steps 20 --no-cpu --no-check
step pmc_c64_a 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex rx_kernel -d gpurun_out/pmc_c64_a -o run --output-format csv -- python bench.py --only c64 --steps 2 --warmup 1 --no-cpu --no-check
step pmc_c64_b 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --kernel-include-regex rx_kernel -d gpurun_out/pmc_c64_b -o run --output-format csv -- python bench.py --only c64 --steps 2 --warmup 1 --no-cpu --no-check
step pmc_c64_f 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d gpurun_out/pmc_c64_f -o run --output-format csv -- python bench.py --only c64 --steps 2 --warmup 1 --no-cpu --no-check
step pmc_c64_w 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rx_kernel -d gpurun_out/pmc_c64_w -o run --output-format csv -- python bench.py --only c64 --steps 2 --warmup 1 --no-cpu --no-check
cat gpurun_out/steps.log
