#!/bin/bash
# (the path-independent lane flush was measured and removed from the source: DESIGN.md section 10)
# Round 3: C64 lane kernel with a path-independent record flush (no store is
# ever skipped, so the stores are not drained at each tile) against the
# previous flush (abl/libpptkrx_old.so); parity tests of the lane kernel first.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "lane or forced_variant or compact or fixed_stride" > gpurun_out/lf_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/lf_tests.log
[ $rc -eq 0 ] || exit $rc
export AB_LIBS=old=abl/libpptkrx_old.so AB_PLACE=1
timeout -k 10 300 python -u tools/ab.py c64 12:-1 old:12:-1 12:-1:c old:12:-1:c > gpurun_out/lf_ab.json 2> gpurun_out/lf_ab.log
rc=$?; echo "c64 rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/lf_ab.json')); print({k:v for k,v in d.items() if isinstance(v,dict) and 'ms' in v})"
exit $rc
