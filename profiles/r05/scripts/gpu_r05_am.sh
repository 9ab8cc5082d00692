#!/bin/bash
# Round 5: as r05al with the second stream (the stand-in's) masked to the K
# CUs the batches leave out ("side"): neither kernel can take the other's
# CUs at the batch boundary.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05am
mkdir -p $O
export PPTK_RX_LIB=tools/ab_libs/exp.so
for cfg in 16:side 32:side 64:side; do
  k=${cfg%%:*}
  PPTK_RX_RESERVE_CUS=$k step m_${cfg/:/_} 300 python -u tools/c8g_emul.py 20 --standin $((k/2)),$k,$((k*2)) --mask $cfg || exit $?
done
grep -h '^{' $O/m*.log
