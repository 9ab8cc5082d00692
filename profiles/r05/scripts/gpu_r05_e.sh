#!/bin/bash
# Round 5: the dense-hash write cost, two A/B builds against the product
# (in one process, placed buffers, T16S6 forced everywhere): the staged hash
# run with temporal stores (hasht), and two consecutive tiles per wave with
# one 8 KB record run and one 1 KB hash run per pair (pairs).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05e
export TMPDIR=/tmp
AB_PLACE=1 AB_ROUNDS=6 AB_LIBS=hasht=tools/ab_libs/hasht.so,pairs=tools/ab_libs/pairs.so timeout -k 10 300 python -u tools/ab.py c1500 3:-1 3:-1:h hasht:3:-1:h pairs:3:-1 pairs:3:-1:h > gpurun_out/r05e/ab_c1500.json 2> gpurun_out/r05e/ab_c1500.log
rc=$?; echo "ab c1500 rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/r05e/ab_c1500.json')); print({k: v for k, v in d.items() if ':' in k})"
[ $rc -eq 0 ] || exit $rc
AB_PLACE=1 AB_ROUNDS=6 AB_LIBS=pairs=tools/ab_libs/pairs.so timeout -k 10 300 python -u tools/ab.py cmix 3:-1 pairs:3:-1 > gpurun_out/r05e/ab_cmix.json 2> gpurun_out/r05e/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/r05e/ab_cmix.json')); print({k: v for k, v in d.items() if ':' in k})"
exit $rc
