#!/bin/bash
# Round 4 (VERDICT ask 2), second pass: the CMIX / C1500 decomposition with
# the product's default memory policy (NT record stores; C1500 also NT
# loads) on placed buffers, and the read/write request mix at the L2's
# memory side (request sizes, DRAM vs Infinity-Cache reads, write stalls)
# for the rx launch, the streaming-only launch and the SOL kernels.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04f
export TMPDIR=/tmp
L=diag=tools/ab_libs/libpptkrx_diag.so
AB_PLACE=1 AB_SOL=1 AB_LIBS=$L timeout -k 10 500 python -u tools/ab.py cmix 3:32 diag:3:32 diag:3:40 diag:3:48 diag:3:56 > gpurun_out/r04f/decomp_cmix.json 2> gpurun_out/r04f/decomp_cmix.log
rc=$?; echo "decomp cmix rc=$rc"; cut -c1-1200 gpurun_out/r04f/decomp_cmix.json
[ $rc -eq 0 ] || exit $rc
AB_PLACE=1 AB_SOL=1 AB_LIBS=$L timeout -k 10 500 python -u tools/ab.py c1500 4:33 diag:4:33 diag:4:41 diag:4:49 diag:4:57 > gpurun_out/r04f/decomp_c1500.json 2> gpurun_out/r04f/decomp_c1500.log
rc=$?; echo "decomp c1500 rc=$rc"; cut -c1-1200 gpurun_out/r04f/decomp_c1500.json
[ $rc -eq 0 ] || exit $rc
PA="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
PB="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum"
PC="TCC_EA0_WRREQ_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_BUBBLE_sum"
for cfg in cmix:3:32 c1500:4:33; do
  c=${cfg%%:*}; s=${cfg#*:}; v=${s%%:*}
  for p in A B C; do
    eval C=\$P$p
    AB_SOL=1 AB_ROUNDS=1 AB_REPS=2 AB_LIBS=$L timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/r04f/tcc_${c}_$p -o run -- python3 tools/ab.py $c $s diag:$v:$(( ${s##*:} + 24 )) > gpurun_out/r04f/tcc_${c}_$p.log 2>&1
    rc=$?; echo "tcc $c $p rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
