#!/bin/bash
# Round 4: where the denying case's extra phase-2 time goes (diagnostic
# builds: no boundary walk / no need stores; timing only, verdicts wrong).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04v
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/permit_run.py keys,keys_denying --lib=nowalk=tools/ab_libs/libpptkrx_nowalk.so --lib=noneed=tools/ab_libs/libpptkrx_noneed.so > gpurun_out/r04v/permit_ab.json 2> gpurun_out/r04v/permit_ab.log
rc=$?; echo "permit ab rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/r04v/permit_ab.json'):
    d=json.loads(l)
    for k,v in d.items(): print(k, v['keys']['ms_per_batch'], v['keys_denying']['ms_per_batch'])"
[ $rc -eq 0 ] || exit $rc
