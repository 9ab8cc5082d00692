#!/bin/bash
# Round 6: RCCL's own account of the channel cap (one-rank communicators).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
step cap 300 python -u tools/comm_cap_probe.py $O || exit $?
