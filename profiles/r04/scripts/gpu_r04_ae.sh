#!/bin/bash
# Round 4: CMIX with each frame's tail chunk loaded right after the round
# that streamed it (libpptkrx_tpr.so) vs the product: time and L2 reads.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ae
export TMPDIR=/tmp
L=tpr=tools/ab_libs/libpptkrx_tpr.so
AB_PLACE=1 AB_SOL=1 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py cmix 3:32 tpr:3:32 > gpurun_out/r04ae/ab_cmix.json 2> gpurun_out/r04ae/ab_cmix.log
rc=$?; echo "ab cmix rc=$rc"; cut -c1-1600 gpurun_out/r04ae/ab_cmix.json
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=1 AB_REPS=2 AB_LIBS=$L timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d gpurun_out/r04ae/tcc_cmix -o run -- python3 tools/ab.py cmix 3:32 tpr:3:32 > gpurun_out/r04ae/tcc_cmix.log 2>&1
rc=$?; echo "tcc rc=$rc"
exit $rc
