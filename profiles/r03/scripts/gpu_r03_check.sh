#!/bin/bash
# Round 3 (re-entry): GPU suite and the default bench line on the rebuilt tree.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/gputests.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; cat gpurun_out/smoke.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench.json
exit $rc
