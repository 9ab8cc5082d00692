#!/bin/bash
# Round 4: rate-limiter tests incl. the hash-class overflow fallback; then
# profiles/r04/scripts/gpu_r04_ac.sh (C1500 tail-temporal loads A/B).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ab
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_permit.py > gpurun_out/r04ab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|overflow" gpurun_out/r04ab/tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/scripts/gpu_r04_ac.sh
