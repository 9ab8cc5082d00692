#!/bin/bash
# Round 5: the split example hung now and then after its run, in the
# cleanup, after destroying the stream its gathers ran on: in the device-wide
# waits of the frees, or in the communicator teardown.  Now main destroys
# the split streams (events first) after the contexts.
# The unsplit and split example tests, three times, each pass required.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05at
mkdir -p $O
for i in 1 2 3; do
  step examples_$i 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_examples.py -k "allgather_bit_exact or split_overlap" || exit $?
  tail -1 $O/examples_$i.log
done
