#!/bin/bash
# Round 6, first box: the new tests first (multi-GPU ownership / channel cap,
# fail-closed rate limiter, compact host records, the in-round tail
# correction's parity), then the whole -m gpu suite.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step new 600 $PT tests/test_gpu_comm.py tests/test_gpu_permit.py \
  "tests/test_gpu_parity.py::test_host_batch_compact_records" \
  "tests/test_gpu_parity.py::test_stream_split" \
  "tests/test_gpu_parity.py::test_mixed_shape_kernel_vs_oracle" -s || exit $?
step all 1000 $PT -m gpu tests || exit $?
