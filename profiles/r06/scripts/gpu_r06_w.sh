#!/bin/bash
# Round 6: tile order on the oversubscribed grid -- strided (product) vs
# blocked (each wave its tiles consecutively, PPTK_RX_TUNE_BLOCKED) for CMIX
# shapes and C64.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
export AB_PLACE=1 AB_ROUNDS=7
step cmix_blocked 400 python -u tools/ab.py cmix 3:32 3:288 6:32 6:288 || exit $?
step c64_blocked 300 python -u tools/ab.py c64 12:33 12:289 12:33:c 12:289:c || exit $?
