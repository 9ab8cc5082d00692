#!/bin/bash
# Round 4: with the temporal last line, are non-temporal loads now a win for
# the offset-described mixes?  CMIX / IMIX / JMIX, NT stores vs NT loads+stores.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ag
export TMPDIR=/tmp
for cfg in cmix:3 jmix:5; do
  c=${cfg%%:*}; v=${cfg#*:}
  AB_PLACE=1 timeout -k 10 400 python -u tools/ab.py $c $v:32 $v:33 > gpurun_out/r04ag/ab_$c.json 2> gpurun_out/r04ag/ab_$c.log
  rc=$?; echo "ab $c rc=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/r04ag/ab_$c.json').read().splitlines()[-1]); print({k:v for k,v in d.items() if ':' in k})"
  [ $rc -eq 0 ] || exit $rc
done
