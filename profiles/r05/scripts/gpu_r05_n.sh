#!/bin/bash
# Round 5: CMIX's speed of light per shape (plain vs non-temporal loads,
# loads in flight, blocks per CU) beside the kernel with plain and with
# non-temporal loads, placed buffers, one process.  Is the gap to SOL the
# load policy the mixes must use?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05n
export TMPDIR=/tmp
AB_PLACE=1 AB_SOL=1 RWMIX_SOL_SHAPES=1 AB_ROUNDS=3 timeout -k 10 300 python -u tools/ab.py cmix 3:32 3:33 > gpurun_out/r05n/ab_cmix.json 2> gpurun_out/r05n/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/r05n/ab_cmix.json')); print(d['sol_ms'], d['sol_desc']); print({k: v['ms'] for k, v in d.items() if ':' in k})"
# HBM reads per launch, plain vs non-temporal loads (T16S6 forced)
for tune in 32 33; do
  PPTK_RX_VARIANT=3 PPTK_RX_TUNE=$tune timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d gpurun_out/r05n/fetch_$tune -o run --output-format csv -- python3 bench.py --only cmix --steps 3 --warmup 1 --no-cpu --no-check --no-membench --no-rec32 --no-place --settle 0.3 --no-live-pmc --no-e2e > gpurun_out/r05n/fetch_$tune.log 2>&1
  rc=$?; echo "fetch tune $tune rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import sys; sys.path.insert(0, '.')
from tools.pmc_summary import counter
for t in (32, 33):
    v, d, name = counter(f'gpurun_out/r05n/fetch_{t}', 'FETCH_SIZE')
    print(t, name[:70], 'FETCH_SIZE x2 GB', round(2 * v[-1] * 1024 / 1e9, 3), 'ms', round(d[-1], 4))
PY
