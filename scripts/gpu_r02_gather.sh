#!/bin/bash
# The collective beside the rx grid on one GPU: a one-rank RCCL all-gather
# with a separate send buffer (RCCL copies 128 MiB per batch), kernel trace
# (does the RCCL kernel run concurrently with the persistent rx grid?) and
# FETCH/WRITE passes (its HBM bytes).
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r02v
mkdir -p $O
step ag_copy_stats 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python tools/opbench.py allgather_copy --steps 10
step ag_copy_fetch 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python tools/opbench.py allgather_copy --steps 5
step ag_copy_write 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python tools/opbench.py allgather_copy --steps 5
step ag_copy_plain 300 python tools/opbench.py allgather_copy --steps 20
cat gpurun_out/steps.log
