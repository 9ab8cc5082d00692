#!/bin/bash
# Round 5: the rx kernel's team-round load pattern on CMIX with nothing
# computed (tools/team_probe.py): plain vs non-temporal loads, lanes past a
# frame's end re-reading its last chunk vs predicated off, beside the SOL.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05p
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/team_probe.py cmix --out gpurun_out/r05p/team_cmix.json > gpurun_out/r05p/team_cmix.log 2>&1
rc=$?; echo "team cmix rc=$rc"; cat gpurun_out/r05p/team_cmix.json
exit $rc
