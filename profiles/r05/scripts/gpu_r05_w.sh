#!/bin/bash
# Round 5: global write phases, the period swept (A/B builds
# -DPPTK_RX_PHASE_TICKS=1000..8000, 10-80 us), placed buffers, one process
# per config: C1500 on T16S7L, CMIX on T16S6.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05w
export TMPDIR=/tmp
L=""; for p in 1000 1500 2000 3000 4000 5000 6000 8000; do L="$L,p$p=tools/ab_libs/phase$p.so"; done; L=${L#,}
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L timeout -k 10 500 python -u tools/ab.py c1500 6:-1 p3000:6:-1 p4000:6:-1 p5000:6:-1 p6000:6:-1 p8000:6:-1 > gpurun_out/r05w/ab_c1500.json 2> gpurun_out/r05w/ab_c1500.log
rc=$?; echo "ab c1500 rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/r05w/ab_c1500.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py cmix 3:-1 p1000:3:-1 p1500:3:-1 p2000:3:-1 p3000:3:-1 > gpurun_out/r05w/ab_cmix.json 2> gpurun_out/r05w/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/r05w/ab_cmix.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
