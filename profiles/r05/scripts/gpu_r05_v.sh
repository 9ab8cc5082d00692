#!/bin/bash
# Round 5: global write phases in the rx kernel (A/B builds
# -DPPTK_RX_PHASE_TICKS=2000 / 4000: each tile's record run held in an LDS
# stash until the chip-wide clock enters a new 20 / 40 us period), placed
# buffers, one process; C1500 on T16S7L and T32S3, CMIX on T16S6.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05v
export TMPDIR=/tmp
L=ph2=tools/ab_libs/phase2000.so,ph4=tools/ab_libs/phase4000.so
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py c1500 6:-1 ph2:6:-1 ph4:6:-1 4:-1 ph2:4:-1 ph4:4:-1 > gpurun_out/r05v/ab_c1500.json 2> gpurun_out/r05v/ab_c1500.log
rc=$?; echo "ab c1500 rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/r05v/ab_c1500.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L timeout -k 10 300 python -u tools/ab.py cmix 3:-1 ph2:3:-1 ph4:3:-1 > gpurun_out/r05v/ab_cmix.json 2> gpurun_out/r05v/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/r05v/ab_cmix.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
