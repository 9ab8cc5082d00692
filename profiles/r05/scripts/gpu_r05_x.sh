#!/bin/bash
# Round 5: global write phases in the product (period from the launch's
# geometry): the GPU parity suite, then in-process A/B against the library
# without them (tools/ab_libs/prev.so) on every config, autotuned shapes,
# placed buffers.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
step gputests 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu || exit $?
grep -E "passed|failed" $O/gputests.log | tail -1
for cfg in c1500 cmix c64 imix jmix; do
  extra=""; [ $cfg = c1500 ] && extra="prev:6:-1 6:-1 prev:4:-1 4:-1"
  AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=prev=tools/ab_libs/prev.so step ab_$cfg 300 python -u tools/ab.py $cfg prev:-1:-1 -1:-1 prev:-1:-1:c -1:-1:c $extra || exit $?
  grep '^{' $O/ab_$cfg.log > $O/ab_$cfg.json
  python3 -c "
import json; d=json.load(open('$O/ab_$cfg.json')); print('$cfg', {k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
done
