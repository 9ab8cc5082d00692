#!/bin/bash
# Round 5: XCD-aware tile order (A/B build: the blocks one XCD runs take
# consecutive tiles), with non-temporal and with plain record / hash stores;
# placed buffers, one process, shapes forced (C1500 T16S7L, CMIX T16S6).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05k
export TMPDIR=/tmp
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=xcd=tools/ab_libs/xcd.so timeout -k 10 400 python -u tools/ab.py c1500 6:-1 xcd:6:-1 6:1 xcd:6:1 6:-1:h xcd:6:-1:h 6:1:h xcd:6:1:h > gpurun_out/r05k/ab_c1500.json 2> gpurun_out/r05k/ab_c1500.log
rc=$?; echo "ab c1500 rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/r05k/ab_c1500.json')); print({k: v['ms'] for k, v in d.items() if ':' in k}, all(v['same_records'] for k, v in d.items() if ':' in k))"
[ $rc -eq 0 ] || exit $rc
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=xcd=tools/ab_libs/xcd.so timeout -k 10 300 python -u tools/ab.py cmix 3:-1 xcd:3:-1 3:0 xcd:3:0 > gpurun_out/r05k/ab_cmix.json 2> gpurun_out/r05k/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/r05k/ab_cmix.json')); print({k: v['ms'] for k, v in d.items() if ':' in k}, all(v['same_records'] for k, v in d.items() if ':' in k))"
exit $rc
