#!/bin/bash
# Round 6, first box: the multi-GPU C-ABI ownership / channel cap, the
# fail-closed rate limiter with its agreed commit decision, compact records
# host to host; then the whole -m gpu suite.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step new 600 $PT tests/test_gpu_comm.py tests/test_gpu_permit.py tests/test_examples.py \
  "tests/test_gpu_parity.py::test_host_batch_compact_records" \
  "tests/test_gpu_parity.py::test_stream_split" -s || exit $?
step all 900 $PT -m gpu tests || exit $?
