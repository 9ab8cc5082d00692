#!/bin/bash
# Round 6: the whole -m gpu suite and smoke() on the final commit.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06final4
mkdir -p $O
step gputests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu || exit $?
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
