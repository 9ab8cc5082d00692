#!/bin/bash
# Round 4: interleaved autotune -- the tests that exercise it, then the
# default bench twice on one box (which shape it picks for C1500, the time).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ai
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "autotune or variant or mixed" > gpurun_out/r04ai/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r04ai/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 900 python -u bench.py --no-live-pmc > gpurun_out/r04ai/bench_$k.json 2> gpurun_out/r04ai/bench_$k.log
  rc=$?; echo "bench $k rc=$rc"; python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/r04ai/bench_$k.json') if x.startswith('{')][-1])
r=d['roofline']; print(r['kernel_variant'], r['kernel_ms'], r['frac'], r.get('mix_sol_frac'), {k:(v.get('kernel_variant'), v['kernel_ms']) for k,v in d['secondary'].items()})"
  [ $rc -eq 0 ] || exit $rc
done
