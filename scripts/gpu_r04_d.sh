#!/bin/bash
# Round 4 (VERDICT ask 2): where CMIX's time over its speed of light goes.
# In-process A/B: the product T16S6 launch, the same kernel from a
# -DPPTK_RX_DIAG build with the record stores (tune 8), the per-frame phase
# (16) or both (24) skipped, and the searched SOL of the launch's traffic;
# then FETCH_SIZE of the rx launch, the streaming-only launch and the SOL
# kernels (calibration of the 1.08x "over-fetch").
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04d
export TMPDIR=/tmp
L=diag=tools/ab_libs/libpptkrx_diag.so
AB_SOL=1 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py cmix 3:0 diag:3:0 diag:3:8 diag:3:16 diag:3:24 > gpurun_out/r04d/decomp_cmix.json 2> gpurun_out/r04d/decomp_cmix.log
rc=$?; echo "decomp cmix rc=$rc"; cut -c1-900 gpurun_out/r04d/decomp_cmix.json
[ $rc -eq 0 ] || exit $rc
AB_SOL=1 AB_LIBS=$L timeout -k 10 400 python -u tools/ab.py c1500 4:1 diag:4:1 diag:4:9 diag:4:17 diag:4:25 > gpurun_out/r04d/decomp_c1500.json 2> gpurun_out/r04d/decomp_c1500.log
rc=$?; echo "decomp c1500 rc=$rc"; cut -c1-900 gpurun_out/r04d/decomp_c1500.json
[ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  AB_SOL=1 AB_ROUNDS=1 AB_REPS=2 AB_LIBS=$L timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r04d/pmc_cmix_$c -o run -- python3 tools/ab.py cmix 3:0 diag:3:24 > gpurun_out/r04d/pmc_cmix_$c.log 2>&1
  rc=$?; echo "pmc cmix $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/r04d/list_avail.txt 2>&1
echo "list-avail rc=$?"
