#!/bin/bash
# Round 6: ring chunks in one read-only descriptor pass (per-chunk ring
# check): the host-path tests, then the default bench line.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step host 600 $PT -m gpu tests/test_gpu_parity.py -k "host_batch or ring" tests/test_examples.py || exit $?
step bench 1000 python -u bench.py --detail $O/bench_detail.json || exit $?
grep '^{' $O/bench.log | tail -1 > $O/bench.json
