#!/bin/bash
# Round 6 closing tree: the -m gpu suite and smoke() as the driver runs them,
# then the default bench line (its own same-run PMC passes give
# roofline.traffic).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/${R06_OUT:-r06final}
mkdir -p $O
step gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 1000 python -u bench.py --detail $O/bench_detail.json || exit $?
grep '^{' $O/bench.log | tail -1 > $O/bench.json
