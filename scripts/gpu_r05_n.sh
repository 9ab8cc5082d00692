#!/bin/bash
# Round 5: CMIX's speed of light per shape (plain vs non-temporal loads,
# loads in flight, blocks per CU) beside the kernel with plain and with
# non-temporal loads, placed buffers, one process.  Is the gap to SOL the
# load policy the mixes must use?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05n
export TMPDIR=/tmp
AB_PLACE=1 AB_SOL=1 RWMIX_SOL_SHAPES=1 AB_ROUNDS=3 timeout -k 10 300 python -u tools/ab.py cmix 3:32 3:33 > gpurun_out/r05n/ab_cmix.json 2> gpurun_out/r05n/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/r05n/ab_cmix.json')); print(d['sol_ms'], d['sol_desc']); print({k: v['ms'] for k, v in d.items() if ':' in k})"
