#!/bin/bash
# Round 4: library-owned placed rings (pptk_rx_ring_alloc): their GPU tests,
# then the default bench line (whose C1500 rings now come from the library).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "ring_alloc or place" > gpurun_out/ring_tests.log 2>&1
rc=$?; echo "ring tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/ring_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/bench_ring.json 2> gpurun_out/bench_ring.log
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_ring.json
exit $rc
