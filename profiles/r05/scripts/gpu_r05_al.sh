#!/bin/bash
# Round 5: CU-masked batches beside the RCCL stand-in, with the stand-in's
# block start times traced.  Mask bit i names CU i // 8 of XCC i % 8, and CU
# c of an XCC sits in SE c % 4 (tools/cumask_map.py, r05ak), so "top K"
# leaves K / 8 CUs free in every XCC, spread over its SEs.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05al
mkdir -p $O
export PPTK_RX_LIB=tools/ab_libs/exp.so
step m0 300 python -u tools/c8g_emul.py 20 --standin 32 || exit $?
for cfg in 32:top 64:top; do
  k=${cfg%%:*}
  PPTK_RX_RESERVE_CUS=$k step m_${cfg/:/_} 300 python -u tools/c8g_emul.py 20 --standin 16,32,$k --mask $cfg || exit $?
done
grep -h '^{' $O/m*.log
