#!/bin/bash
# Round 3: GPU suite, the default bench line (untraced), the record-burst
# placement probe.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gputests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/gputests.log | tail -2
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/place_probe.py --bursts --batches 3 --matrix 6 --reps 3 > gpurun_out/bursts.json 2> gpurun_out/bursts.log
rc=$?; echo "bursts rc=$rc"; cat gpurun_out/bursts.json
exit $rc
