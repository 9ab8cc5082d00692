#!/bin/bash
# Round 4: C1500 shapes with the temporal last line (in-process A/B, placed
# pair, 9 rounds): T32S3, T16S7L, T32S4L, T32S3D7, T16S6.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ah
export TMPDIR=/tmp
AB_ROUNDS=9 AB_PLACE=1 AB_SOL=1 timeout -k 10 500 python -u tools/ab.py c1500 4:33 6:33 7:33 8:33 3:33 > gpurun_out/r04ah/ab_c1500.json 2> gpurun_out/r04ah/ab_c1500.log
rc=$?; echo "ab rc=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/r04ah/ab_c1500.json').read().splitlines()[-1]); print(d.get('sol_ms'), {k:v['ms'] for k,v in d.items() if ':' in k})"
exit $rc
