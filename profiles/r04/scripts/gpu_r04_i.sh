#!/bin/bash
# Round 4: tail chunk through LDS (CMIX over-fetch) + fused rate limiter v5
# (nonce barriers, no memset, per-workgroup stamps).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04i
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_permit.py tests/test_gpu_parity.py > gpurun_out/r04i/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r04i/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/permit_run.py --stamps > gpurun_out/r04i/stamps.json 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/r04i/stamps.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/permit_run.py keys,keys_denying --ab > gpurun_out/r04i/permit_ab.json 2> gpurun_out/r04i/permit_ab.log
rc=$?; echo "permit ab rc=$rc"; python3 -c "
import json
for l in open('gpurun_out/r04i/permit_ab.json'):
    d=json.loads(l)
    for k,v in d.items(): print(k, v['keys']['ms_per_batch'], v['keys_denying']['ms_per_batch'])"
[ $rc -eq 0 ] || exit $rc
L=old=tools/ab_libs/libpptkrx_diag.so
AB_PLACE=1 AB_SOL=1 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py cmix 3:32 old:3:32 -1:-1 > gpurun_out/r04i/ab_cmix.json 2> gpurun_out/r04i/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"; cut -c1-1800 gpurun_out/r04i/ab_cmix.json
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=1 AB_REPS=2 AB_LIBS=$L timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d gpurun_out/r04i/tcc_cmix -o run -- python3 tools/ab.py cmix 3:32 old:3:32 > gpurun_out/r04i/tcc_cmix.log 2>&1
rc=$?; echo "tcc cmix rc=$rc"
[ $rc -eq 0 ] || exit $rc
for run in keys keys_denying; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r04i/pmc_${run}_$c -o run -- python3 tools/permit_run.py $run > gpurun_out/r04i/pmc_${run}_$c.log 2>&1
    rc=$?; echo "pmc $run $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
