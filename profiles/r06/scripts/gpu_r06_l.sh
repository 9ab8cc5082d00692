#!/bin/bash
# Round 6: the C64 lane kernel with coalesced tile loads (1 KB contiguous per
# load instruction, chunks handed to their frames' lanes through LDS) against
# the per-lane loads, one process, placed buffers; NT stores, +/- NT loads,
# 64- and 32-byte records.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
export AB_LIBS=coal=tools/ab_r06/libpptkrx_coal.so AB_PLACE=1 AB_ROUNDS=9 AB_SOL=1
step coal_c64 400 python -u tools/ab.py c64 12:32 coal:12:32 12:33 coal:12:33 12:32:c coal:12:32:c coal:12:33:c || exit $?
