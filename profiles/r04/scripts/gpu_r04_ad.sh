#!/bin/bash
# Round 4: the temporal last line as the product default: parity suite on
# the rx kernels, the A/B against the previous kernel (diag build = round-4
# code before the change), RDREQ, and a default bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ad
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tx.py > gpurun_out/r04ad/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r04ad/tests.log | tail -4
[ $rc -eq 0 ] || exit $rc
L=old=tools/ab_libs/libpptkrx_diag.so
AB_PLACE=1 AB_SOL=1 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py c1500 4:33 old:4:33 4:32 > gpurun_out/r04ad/ab_c1500.json 2> gpurun_out/r04ad/ab_c1500.log
rc=$?; echo "ab c1500 rc=$rc"; cut -c1-1600 gpurun_out/r04ad/ab_c1500.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r04ad/bench.json 2> gpurun_out/r04ad/bench.log
rc=$?; echo "bench rc=$rc"; python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/r04ad/bench.json') if x.startswith('{')][-1])
r=d['roofline']; print('c1500', r['kernel_ms'], r['frac'], r.get('mix_sol_frac'), r.get('traffic'))"
exit $rc
