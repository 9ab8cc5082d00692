#!/bin/bash
# Round 6: the default bench line on this tree (its own same-run PMC passes
# give roofline.traffic).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
step bench 1000 python -u bench.py --detail $O/bench_detail.json || exit $?
grep '^{' $O/bench.log | tail -1 > $O/bench.json
