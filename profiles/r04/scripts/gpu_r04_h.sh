#!/bin/bash
# Round 4: does processing adjacent frames in one round (PPTK_RX_ADJ build)
# remove the boundary-line re-fetches (TCC_EA0_RDREQ above the SOL kernel's)?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04h
export TMPDIR=/tmp
L=adj=tools/ab_libs/libpptkrx_adj.so
AB_PLACE=1 AB_SOL=1 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py cmix 3:32 adj:3:32 3:33 adj:3:33 > gpurun_out/r04h/ab_cmix.json 2> gpurun_out/r04h/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"; cut -c1-1500 gpurun_out/r04h/ab_cmix.json
[ $rc -eq 0 ] || exit $rc
AB_PLACE=1 AB_SOL=1 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py c1500 4:33 adj:4:33 4:32 adj:4:32 > gpurun_out/r04h/ab_c1500.json 2> gpurun_out/r04h/ab_c1500.log
rc=$?; echo "ab c1500 rc=$rc"; cut -c1-1500 gpurun_out/r04h/ab_c1500.json
[ $rc -eq 0 ] || exit $rc
for cfg in cmix:3:32:3:33 c1500:4:33:4:32; do
  IFS=: read c v f1 v2 f2 <<< "$cfg"
  AB_ROUNDS=1 AB_REPS=2 AB_LIBS=$L timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d gpurun_out/r04h/tcc_$c -o run -- python3 tools/ab.py $c $v:$f1 adj:$v:$f1 $v2:$f2 adj:$v2:$f2 > gpurun_out/r04h/tcc_$c.log 2>&1
  rc=$?; echo "tcc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
