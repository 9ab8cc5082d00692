#!/bin/bash
# Round 5: write-phase stash of two tiles for the two-workgroup shapes
# (T16S6, T32S3; period 1.25 tile) against one tile (d1.so, period 0.75)
# and no phases (prev.so); placed buffers, one process per config; then the
# GPU parity suite on this tree.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05ab
mkdir -p $O
L=prev=tools/ab_libs/prev.so,d1=tools/ab_libs/d1.so
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L step ab_c1500 400 python -u tools/ab.py c1500 prev:3:-1 d1:3:-1 3:-1 prev:4:-1 d1:4:-1 4:-1 prev:6:-1 6:-1 || exit $?
grep '^{' $O/ab_c1500.log > $O/ab_c1500.json
python3 -c "
import json; d=json.load(open('$O/ab_c1500.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L step ab_cmix 300 python -u tools/ab.py cmix prev:3:-1 d1:3:-1 3:-1 prev:6:-1 6:-1 || exit $?
grep '^{' $O/ab_cmix.log > $O/ab_cmix.json
python3 -c "
import json; d=json.load(open('$O/ab_cmix.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
step gputests 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu || exit $?
grep -E "passed|failed" $O/gputests.log | tail -1
