#!/bin/bash
# Round 6: CMIX record-store policy on the oversubscribed grid: NT stores
# (product) vs plain vs write-through (sc1), T16S6 and T16S7L.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06ac
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=7
step cmix_stores 400 python -u tools/ab.py cmix 3:32 3:0 3:64 6:32 6:0 6:64 || exit $?
