#!/bin/bash
# Round 5, first box: GPU suite (rate-limiter abort/ordering tests, hooks
# library), in-process A/B of the flow-hash store modes on C1500, the rate
# limiter's timings after the deferred token commit.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/r05a/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r05a/gputests.log | tail -2
[ $rc -eq 0 ] || exit $rc
AB_PLACE=1 AB_ROUNDS=6 AB_LIBS=h0=tools/ab_libs/hash0.so,h1=tools/ab_libs/hash1.so timeout -k 10 300 python -u tools/ab.py c1500 -1:-1 -1:-1:h h0:-1:-1:h h1:-1:-1:h > gpurun_out/r05a/ab_hash_c1500.json 2> gpurun_out/r05a/ab_hash_c1500.log
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r05a/ab_hash_c1500.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench
dev = torch.device('cuda', 0)
print(json.dumps(bench.permit_bench(1 << 24, dev, 1, 0, 20, 5)))
" > gpurun_out/r05a/permit.json 2> gpurun_out/r05a/permit.log
rc=$?; echo "permit rc=$rc"; cut -c 1-1500 gpurun_out/r05a/permit.json
exit $rc
