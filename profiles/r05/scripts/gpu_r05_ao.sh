#!/bin/bash
# Round 5: C8G's one-GPU emulation with the collective's CU footprint: the
# RCCL stand-in copies the 7 x 128 MiB landing bytes into the gather buffer
# paced to 1.7 ms (tools/c8g_emul.py --copy), without and with the product's
# 32-CU split; and the round-2 emulation (a device copy on the second
# stream) without and with the split.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05ao
mkdir -p $O
step copy_nosplit 300 python -u tools/c8g_emul.py 20 || exit $?
step copy_split32 300 python -u tools/c8g_emul.py 20 --split 32 || exit $?
step standin_copy_nosplit 300 python -u tools/c8g_emul.py 20 --standin 32 --copy || exit $?
step standin_copy_split32 300 python -u tools/c8g_emul.py 20 --standin 16,32 --copy --split 32 || exit $?
grep -h '^{' $O/*.log | cut -c1-1500
