#!/bin/bash
# Round 5: C8G's HBM side emulated on one GPU again, on the tree with the
# global write phases (tools/c8g_emul.py; as gpu_r05_g.sh).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05ad
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/c8g_emul.py 20 > gpurun_out/r05ad/c8g_emul.json 2> gpurun_out/r05ad/c8g_emul.log
rc=$?; echo "c8g_emul rc=$rc"; head -c 2500 gpurun_out/r05ad/c8g_emul.json
exit $rc
