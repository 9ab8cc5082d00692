#!/bin/bash
# Round 3: rate limiter parity, then its per-kernel trace (three regimes).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/permit
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_permit.py -m gpu > gpurun_out/permit/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/permit/tests.log | tail -2
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/permit/prof -o run -- python3 tools/opbench.py permit --steps 10 --warmup 2 > gpurun_out/permit/opbench.json 2> gpurun_out/permit/opbench.log
rc=$?; echo "prof rc=$rc"
exit $rc
