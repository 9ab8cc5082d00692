#!/bin/bash
# Round 4: fused rate limiter: candidates counted by fine class in their own sweep, pass count a
# power of two (no class-count sweep), vs p4 = the committed v24.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ao
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_permit.py > gpurun_out/r04ao/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r04ao/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/permit_run.py --stamps > gpurun_out/r04ao/stamps.json 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/r04ao/stamps.json
[ $rc -eq 0 ] || exit $rc
A=tools/ab_libs/libpptkrx_code_
timeout -k 10 500 python -u tools/permit_run.py keys,keys_denying --ab --lib=p4=tools/ab_libs/libpptkrx_p4.so --lib=prod=pptk_amd/libpptkrx.so --lib=p4b=tools/ab_libs/libpptkrx_p4.so --lib=prodb=pptk_amd/libpptkrx.so > gpurun_out/r04ao/permit_ab.json 2> gpurun_out/r04ao/permit_ab.log
rc=$?; echo "permit ab rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/r04ao/permit_ab.json'):
    d=json.loads(l)
    for k,v in d.items(): print(k, v['keys']['ms_per_batch'], v['keys_denying']['ms_per_batch'], v['keys_denying']['verdicts'])"
[ $rc -eq 0 ] || exit $rc
