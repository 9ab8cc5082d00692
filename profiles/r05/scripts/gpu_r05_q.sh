#!/bin/bash
# Round 5: the team-round load pattern (tools/team_probe.py) on C1500 frames
# (descriptor form c1500g) and CMIX: lanes past a frame's end re-reading its
# last chunk, predicated off by a branch, or given an out-of-range offset of
# a raw buffer load (no request, no branch); plain vs non-temporal.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05q
export TMPDIR=/tmp
for cfg in c1500g cmix; do
  timeout -k 10 300 python -u tools/team_probe.py $cfg --out gpurun_out/r05q/team_$cfg.json > gpurun_out/r05q/team_$cfg.log 2>&1
  rc=$?; echo "team $cfg rc=$rc"; cat gpurun_out/r05q/team_$cfg.json
  [ $rc -eq 0 ] || exit $rc
done
