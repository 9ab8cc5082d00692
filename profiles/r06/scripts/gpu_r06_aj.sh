#!/bin/bash
# Round 6: every 1536-byte-class shape on CMIX on the oversubscribed grid
# (and T32S4L, T16S6D1, outside the autotune's candidates), one process.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06aj
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=7
step cmix_shapes 500 python -u tools/ab.py cmix 3:-1 4:-1 6:-1 7:-1 8:-1 9:-1 13:-1 || exit $?
