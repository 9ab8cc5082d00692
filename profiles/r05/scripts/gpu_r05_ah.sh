#!/bin/bash
# Round 5: the dense flow-hash run held in the write-phase stash with the
# records (A/B build phh140: -DPPTK_RX_PHASE_HASH, which needs the 140-byte
# image pitch to fit three workgroups per CU) against the product; img140 =
# the pitch alone.  With (:h) and without the hash output; placed buffers.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05ah
mkdir -p $O
L=img140=tools/ab_libs/img140.so,phh140=tools/ab_libs/phh140.so
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L step ab_c1500 500 python -u tools/ab.py c1500 6:-1 img140:6:-1 6:-1:h img140:6:-1:h phh140:6:-1:h || exit $?
grep '^{' $O/ab_c1500.log > $O/ab_c1500.json
python3 -c "
import json; d=json.load(open('$O/ab_c1500.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L step ab_cmix 400 python -u tools/ab.py cmix 3:-1 img140:3:-1 13:-1 img140:13:-1 3:-1:h phh140:3:-1:h || exit $?
grep '^{' $O/ab_cmix.log > $O/ab_cmix.json
python3 -c "
import json; d=json.load(open('$O/ab_cmix.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
