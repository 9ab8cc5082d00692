#!/bin/bash
# Round 6: the final tree against the tree of the second closing run
# (final2: before the tile-range rework), one process, placed buffers:
# CMIX T16S6 / T16S7L / M6, IMIX M6, C64.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06ae
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=9 AB_LIBS=f2=tools/ab_r06/libpptkrx_final2.so
step cmix 400 python -u tools/ab.py cmix 3:-1 f2:3:-1 6:-1 f2:6:-1 13:-1 f2:13:-1 || exit $?
step imix 300 python -u tools/ab.py imix 13:-1 f2:13:-1 || exit $?
step c64 300 python -u tools/ab.py c64 12:-1 f2:12:-1 || exit $?
