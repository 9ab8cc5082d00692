#!/bin/bash
# Round 5: the batches on a CU-masked stream (hipExtStreamCreateWithCUMask)
# that leaves K CUs to the collective, with the grid sized for the rest
# (experiment build, PPTK_RX_RESERVE_CUS=K), beside the RCCL stand-in on K
# blocks (tools/libstandin.so, 1.7 ms per batch).  Mask patterns: the top K
# bits, or every (256/K)-th bit.  One process per setting (the knob is read
# once); the first is the experiment build unmasked.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05aj
mkdir -p $O
export PPTK_RX_LIB=tools/ab_libs/exp.so
step m0 300 python -u tools/c8g_emul.py 20 --standin 16,32 || exit $?
for cfg in 16:spread 16:top 32:spread 32:top 64:spread; do
  k=${cfg%%:*}
  PPTK_RX_RESERVE_CUS=$k step m_${cfg/:/_} 300 python -u tools/c8g_emul.py 20 --standin $k --mask $cfg || exit $?
done
grep -h '^{' $O/m*.log
