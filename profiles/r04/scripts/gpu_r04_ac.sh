#!/bin/bash
# Round 4: C1500 with the window's last 8 chunks loaded temporally (the
# boundary line kept in L2 for the next frame) vs the product kernel:
# time (placed pair, in-process A/B) and L2 read requests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ac
export TMPDIR=/tmp
L=tailt=tools/ab_libs/libpptkrx_tailt.so
AB_PLACE=1 AB_SOL=1 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py c1500 4:33 tailt:4:33 > gpurun_out/r04ac/ab_c1500.json 2> gpurun_out/r04ac/ab_c1500.log
rc=$?; echo "ab c1500 rc=$rc"; cut -c1-1500 gpurun_out/r04ac/ab_c1500.json
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=1 AB_REPS=2 AB_LIBS=$L timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d gpurun_out/r04ac/tcc_c1500 -o run -- python3 tools/ab.py c1500 4:33 tailt:4:33 > gpurun_out/r04ac/tcc_c1500.log 2>&1
rc=$?; echo "tcc rc=$rc"
exit $rc
