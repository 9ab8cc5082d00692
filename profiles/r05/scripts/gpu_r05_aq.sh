#!/bin/bash
# Round 5: the work queue (tiles past each wave's first five claimed from a
# chip-wide counter, RxKArgs::ticket; build wq = -DPPTK_RX_WORK_QUEUE=1)
# against fixed strided tiles: the committed library (head), this tree's
# product (the same kernel with ticket null) and wq; records compared.  Then
# the GPU parity tests on the wq library.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r05aq
mkdir -p $O
L=head=tools/ab_libs/head.so,wq=tools/ab_libs/wq.so
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L step ab_c1500 500 python -u tools/ab.py c1500 head:6:-1 6:-1 wq:6:-1 head:4:-1 wq:4:-1 || exit $?
grep '^{' $O/ab_c1500.log > $O/ab_c1500.json
python3 -c "
import json; d=json.load(open('$O/ab_c1500.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
AB_PLACE=1 AB_ROUNDS=5 AB_LIBS=$L step ab_cmix 400 python -u tools/ab.py cmix head:3:-1 3:-1 wq:3:-1 head:6:-1 wq:6:-1 || exit $?
grep '^{' $O/ab_cmix.log > $O/ab_cmix.json
python3 -c "
import json; d=json.load(open('$O/ab_cmix.json')); print({k: (v['ms'], v['same_records']) for k, v in d.items() if ':' in k})"
PPTK_RX_LIB=tools/ab_libs/wq.so step tests_wq 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py || exit $?
tail -3 $O/tests_wq.log
