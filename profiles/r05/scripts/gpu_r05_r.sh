#!/bin/bash
# Round 5: lanes past a frame's end load nothing (A/B builds
# -DPPTK_RX_PRED_LOADS=1: the last line temporal, =2: all non-temporal)
# against the unconditional clamped loads; placed buffers, one process.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05r
export TMPDIR=/tmp
L=p1=tools/ab_libs/pred1.so,p2=tools/ab_libs/pred2.so
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L timeout -k 10 300 python -u tools/ab.py c1500 6:-1 p1:6:-1 p2:6:-1 > gpurun_out/r05r/ab_c1500.json 2> gpurun_out/r05r/ab_c1500.log
rc=$?; echo "ab c1500 rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/r05r/ab_c1500.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L timeout -k 10 300 python -u tools/ab.py cmix 3:-1 p2:3:-1 > gpurun_out/r05r/ab_cmix.json 2> gpurun_out/r05r/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/r05r/ab_cmix.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
