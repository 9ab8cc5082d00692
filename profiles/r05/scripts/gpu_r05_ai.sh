#!/bin/bash
# Round 5: does the collective's kernel get room beside the persistent rx
# grid?  tools/libstandin.so stands in for RCCL's all-gather kernel with its
# gfx950 footprint (a block needs a whole CU) and spins 1.7 ms per batch on
# 16 / 64 / 256 blocks, ordered as bench.py orders the gather (C1500,
# placed buffers).  Then the experiment build with PPTK_RX_RESERVE_CUS=64
# (the rx grid sized for 192 CUs).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05ai
mkdir -p $O
step standin 300 python -u tools/c8g_emul.py 20 --standin 16,32,64,128,256 || exit $?
PPTK_RX_LIB=tools/ab_libs/exp.so PPTK_RX_RESERVE_CUS=64 step standin_res64 300 python -u tools/c8g_emul.py 20 --standin 16,32,64 || exit $?
grep -h '^{' $O/standin.log $O/standin_res64.log
