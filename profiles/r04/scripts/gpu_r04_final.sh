#!/bin/bash
# Round 4 final tree: full GPU suite, then profiles/r04/scripts/gpu_r04_prof.sh (smoke,
# traced default bench, per-config FETCH/WRITE passes), then the untraced
# default bench line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/steps.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/gputests.log | tail -2
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/scripts/gpu_r04_prof.sh || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/bench.json
exit $rc
