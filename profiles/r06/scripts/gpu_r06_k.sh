#!/bin/bash
# Round 6: C64 on the lane kernel (L4) taken apart: product flags, the
# diagnostic build with the per-frame work skipped (tune bit 16), the record
# stores skipped (bit 8), both; compact records; the speed of light.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
export AB_LIBS=diag=tools/ab_r06/libpptkrx_diag.so AB_PLACE=1 AB_ROUNDS=7 AB_SOL=1
step decomp_c64 400 python -u tools/ab.py c64 12:-1 12:32 diag:12:32 diag:12:48 diag:12:40 diag:12:56 12:32:c || exit $?
