#!/bin/bash
# Round 5: write phases in M6 (136-byte image pitch, one tile held) against
# M6 without them (nom6.so) and against no phases at all (prev.so): IMIX and
# CMIX with M6 forced, placed buffers, one process per config; then the GPU
# parity suite on this tree.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05ac
mkdir -p $O
L=prev=tools/ab_libs/prev.so,nom6=tools/ab_libs/nom6.so
for cfg in imix cmix; do
  AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L step ab_$cfg 300 python -u tools/ab.py $cfg prev:13:-1 nom6:13:-1 13:-1 nom6:3:-1 || exit $?
  grep '^{' $O/ab_$cfg.log > $O/ab_$cfg.json
  python3 -c "
import json; d=json.load(open('$O/ab_$cfg.json')); print('$cfg', {k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
done
step gputests 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu || exit $?
grep -E "passed|failed" $O/gputests.log | tail -1
