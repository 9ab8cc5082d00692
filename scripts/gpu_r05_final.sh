#!/bin/bash
# Round 5 closing tree, first box: the whole GPU suite, smoke, then the
# default bench line (untraced; its own same-run PMC passes give
# roofline.traffic), full result in $O/bench_detail.json.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05final
mkdir -p $O
step gputests 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu || exit $?
grep -E "passed|failed" $O/gputests.log | tail -1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 900 python -u bench.py --detail $O/bench_detail.json || exit $?
grep '^{' $O/bench.log | tail -1 > $O/bench.json
tail -c 600 $O/bench.json
