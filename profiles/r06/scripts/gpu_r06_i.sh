#!/bin/bash
# Round 6: CMIX (and C1500) taken apart on the round-6 kernel, T16S6 forced,
# placed buffers, one process: product flags; the diagnostic build with the
# record stores skipped (tune bit 8), the per-frame phase skipped (bit 16),
# both; and 32-byte records.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
export AB_LIBS=diag=tools/ab_r06/libpptkrx_diag.so AB_PLACE=1 AB_ROUNDS=7 AB_SOL=1
for cfg in cmix c1500; do
  step decomp_$cfg 400 python -u tools/ab.py $cfg 3:32 diag:3:32 diag:3:40 diag:3:48 diag:3:56 3:32:c || exit $?
done
