#!/bin/bash
# Round 4: fused rate limiter v20 (register class counts) vs v19.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04aa
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_permit.py > gpurun_out/r04aa/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r04aa/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/permit_run.py --stamps > gpurun_out/r04aa/stamps.json 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/r04aa/stamps.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/permit_run.py keys,keys_denying --ab --lib=v19=tools/ab_libs/libpptkrx_v19.so > gpurun_out/r04aa/permit_ab.json 2> gpurun_out/r04aa/permit_ab.log
rc=$?; echo "permit ab rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/r04aa/permit_ab.json'):
    d=json.loads(l)
    for k,v in d.items(): print(k, v['keys']['ms_per_batch'], v['keys_denying']['ms_per_batch'])"
[ $rc -eq 0 ] || exit $rc
