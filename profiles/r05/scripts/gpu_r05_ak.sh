#!/bin/bash
# Round 5: the CU named by each CU-mask bit (tools/cumask_map.py).
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05ak
mkdir -p $O
step cumask_map 120 python -u tools/cumask_map.py || exit $?
grep -h '^{' $O/cumask_map.log
