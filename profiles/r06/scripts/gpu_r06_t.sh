#!/bin/bash
# Round 6: the tree with coalesced lane tiles and oversubscribed grids --
# the whole -m gpu suite, smoke(), and the default bench line.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
step suite 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ || exit $?
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 900 python -u bench.py --detail $O/bench_detail.json || exit $?
