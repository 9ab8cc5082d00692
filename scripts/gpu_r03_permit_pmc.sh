#!/bin/bash
# SQ counters of the rate limiter's resolve pass in the denying regime.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/permit_pmc
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/permit_pmc/trace -o run -- python3 tools/permit_probe.py > gpurun_out/permit_pmc/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex permit_resolve --output-format csv -d gpurun_out/permit_pmc/sq -o run -- python3 tools/permit_probe.py > gpurun_out/permit_pmc/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS --kernel-include-regex permit_resolve --output-format csv -d gpurun_out/permit_pmc/wait -o run -- python3 tools/permit_probe.py > gpurun_out/permit_pmc/wait.log 2>&1 || exit 1
echo done
