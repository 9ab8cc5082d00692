#!/bin/bash
# Round 4: fused rate limiter v9 (speculative verdicts after the table loads)
# vs v8 (before them, libpptkrx_early.so); CMIX record-store policies.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04n
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_permit.py > gpurun_out/r04n/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r04n/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/permit_run.py --stamps > gpurun_out/r04n/stamps.json 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/r04n/stamps.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/permit_run.py keys,keys_denying --ab --lib=early=tools/ab_libs/libpptkrx_early.so > gpurun_out/r04n/permit_ab.json 2> gpurun_out/r04n/permit_ab.log
rc=$?; echo "permit ab rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/r04n/permit_ab.json'):
    d=json.loads(l)
    for k,v in d.items(): print(k, v['keys']['ms_per_batch'], v['keys_denying']['ms_per_batch'])"
[ $rc -eq 0 ] || exit $rc
L=diag=tools/ab_libs/libpptkrx_diag.so
AB_PLACE=1 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py cmix 3:32 diag:3:32 diag:3:0 diag:3:64 diag:3:288 diag:3:256 > gpurun_out/r04n/ab_cmix_stores.json 2> gpurun_out/r04n/ab_cmix_stores.log
rc=$?; echo "ab cmix rc=$rc"; cut -c1-2000 gpurun_out/r04n/ab_cmix_stores.json
[ $rc -eq 0 ] || exit $rc
