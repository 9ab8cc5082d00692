#!/bin/bash
# Round 5: the work queue with one counter per block % nq group instead of
# one counter (which capped claims at ~50-70 M/s, r05aq): nq = 8 (256 B
# apart), 8 (4 KB apart), 32 (256 B apart), against the committed library
# and this tree's static product; records compared.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05ar
mkdir -p $O
L=head=tools/ab_libs/head.so,wq8=tools/ab_libs/wq8.so,wq8k=tools/ab_libs/wq8k.so,wq32=tools/ab_libs/wq32.so
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L step ab_c1500 500 python -u tools/ab.py c1500 head:6:-1 6:-1 wq8:6:-1 wq8k:6:-1 wq32:6:-1 || exit $?
grep '^{' $O/ab_c1500.log > $O/ab_c1500.json
python3 -c "
import json; d=json.load(open('$O/ab_c1500.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L step ab_cmix 400 python -u tools/ab.py cmix head:3:-1 3:-1 wq8:3:-1 wq8k:3:-1 wq32:3:-1 || exit $?
grep '^{' $O/ab_cmix.log > $O/ab_cmix.json
python3 -c "
import json; d=json.load(open('$O/ab_cmix.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
