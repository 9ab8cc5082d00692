#!/bin/bash
# Round 6: CMIX shapes on the oversubscribed grid against the persistent
# grid (the previous build), incl. the mixed call (batch order by plan).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=7 AB_LIBS=old=tools/ab_r06/libpptkrx_r06coal.so
step cmix_shapes 400 python -u tools/ab.py cmix 6:-1 old:6:-1 3:-1 old:3:-1 4:-1 old:4:-1 -1:-1:m old:-1:-1:m || exit $?
