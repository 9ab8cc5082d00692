#!/bin/bash
# Round 3: GPU suite, smoke and the default bench line (untraced).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/gputests.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench.json
exit $rc
