#!/bin/bash
# Record-write burst sizes against frame/record placement (tools/place_probe.py --bursts).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/place_probe.py --bursts --batches 3 --matrix 2 --reps 3 > gpurun_out/bursts4.json 2> gpurun_out/bursts4.log
rc=$?; echo "bursts rc=$rc"; cat gpurun_out/bursts4.json
exit $rc
