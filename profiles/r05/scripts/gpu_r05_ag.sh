#!/bin/bash
# Round 5: the write-phase check after every round instead of between round
# groups (A/B build -DPPTK_RX_PHASE_CHECK_ROUND: finer alignment for the
# shapes with D = 3, whose groups are four rounds); placed buffers, in
# process, two configs.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05ag
mkdir -p $O
L=pcr=tools/ab_libs/pcr.so
AB_PLACE=1 AB_ROUNDS=6 AB_LIBS=$L step ab_c1500 400 python -u tools/ab.py c1500 6:-1 pcr:6:-1 4:-1 pcr:4:-1 3:-1 pcr:3:-1 || exit $?
grep '^{' $O/ab_c1500.log > $O/ab_c1500.json
python3 -c "
import json; d=json.load(open('$O/ab_c1500.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
AB_PLACE=1 AB_ROUNDS=6 AB_LIBS=$L step ab_cmix 300 python -u tools/ab.py cmix 3:-1 pcr:3:-1 6:-1 pcr:6:-1 || exit $?
grep '^{' $O/ab_cmix.log > $O/ab_cmix.json
python3 -c "
import json; d=json.load(open('$O/ab_cmix.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
