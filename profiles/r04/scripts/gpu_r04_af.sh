#!/bin/bash
# Round 4: repeat of the per-round tail A/B (more rounds), CMIX and JMIX.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04af
export TMPDIR=/tmp
L=tpr=tools/ab_libs/libpptkrx_tpr.so
for cfg in cmix:3:32 jmix:5:32; do
  c=${cfg%%:*}; s=${cfg#*:}
  AB_ROUNDS=9 AB_PLACE=1 AB_LIBS=$L timeout -k 10 500 python -u tools/ab.py $c $s tpr:$s > gpurun_out/r04af/ab_$c.json 2> gpurun_out/r04af/ab_$c.log
  rc=$?; echo "ab $c rc=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/r04af/ab_$c.json').read().splitlines()[-1]); print({k:v for k,v in d.items() if ':' in k})"
  [ $rc -eq 0 ] || exit $rc
done
