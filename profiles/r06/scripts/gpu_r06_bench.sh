#!/bin/bash
# Round 6: the default bench line alone (after a bench.py change).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/${R06_OUT:-r06bench}
mkdir -p $O
step bench 1000 python -u bench.py --detail $O/bench_detail.json || exit $?
grep '^{' $O/bench.log | tail -1 > $O/bench.json
