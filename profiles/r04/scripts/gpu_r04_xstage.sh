#!/bin/bash
# Round 4: XCD-staged 256 KB record flush probe (tools/place_probe.py --xstage)
# on slow and fast (frames, records) pairs, plus a quick bench sanity line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/place_probe.py --xstage --batches 3 --matrix 2 --reps 3 > gpurun_out/xstage.json 2> gpurun_out/xstage.log
rc=$?; echo "xstage rc=$rc"; cat gpurun_out/xstage.json
exit $rc
