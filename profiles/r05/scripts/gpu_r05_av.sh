#!/bin/bash
# Round 5: a fifth wave per workgroup as the only writer (tools/epoch_probe.hip
# MODE 5/6, EPOCH_SWEEP=writer): the streaming waves hand each tile's run
# over through LDS, so their wait counters hold loads only; against the run
# stored by its own wave at tile end and the global write phases (MODE 0/1),
# bare C1500 tiles on the library's rings, 2 and 3 workgroups per CU.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05av
mkdir -p $O
EPOCH_SWEEP=writer step writer 400 python -u tools/epoch_probe.py --rounds 4 --out $O/writer.json || exit $?
cat $O/writer.json
