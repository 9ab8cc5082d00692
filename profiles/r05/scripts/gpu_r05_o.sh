#!/bin/bash
# Round 5: CMIX with non-temporal frame loads on the line-aligned shapes
# (T16S7L, T32S4L: chunk grid on 128-byte lines, where the window's last
# line is loaded temporally) against T16S6, plain and non-temporal loads;
# placed buffers, one process.  (The SOL kernel reads CMIX 9 % faster with
# non-temporal loads: profiles/r05/n/.)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05o
export TMPDIR=/tmp
AB_PLACE=1 AB_ROUNDS=4 timeout -k 10 300 python -u tools/ab.py cmix 3:32 3:33 6:32 6:33 7:32 7:33 > gpurun_out/r05o/ab_cmix.json 2> gpurun_out/r05o/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/r05o/ab_cmix.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
