#!/bin/bash
# Round 5: the split's size for C8G: the copying RCCL stand-in (7 x 128 MiB
# landed per batch, paced to 1.7 ms, one block per split CU) beside C1500
# with 32 and with 64 CUs split off; one process each.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05aw
mkdir -p $O
step split32 300 python -u tools/c8g_emul.py 20 --standin 32 --copy --split 32 || exit $?
step split64 300 python -u tools/c8g_emul.py 20 --standin 64 --copy --split 64 || exit $?
grep -h '^{' $O/split32.log $O/split64.log
