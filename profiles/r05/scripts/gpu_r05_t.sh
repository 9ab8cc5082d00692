#!/bin/bash
# Round 5: host-to-host C64 and C1500, records written by the kernel over
# PCIe (product) vs written to device memory and copied back by DMA
# (experiment build, PPTK_RX_RECS_DMA=1), record array registered (C64) or
# not; separate processes, same box, alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05t
export TMPDIR=/tmp
for r in 1 2; do
  for v in prod dma; do
    if [ $v = dma ]; then export E2E_LIB=tools/ab_libs/exp.so PPTK_RX_RECS_DMA=1; else unset E2E_LIB PPTK_RX_RECS_DMA; fi
    E2E_CFGS=c64 E2E_REG_OUT=1 timeout -k 10 200 python -u tools/e2e.py 4194304 65536 > gpurun_out/r05t/c64_reg_${v}_$r.json 2> gpurun_out/r05t/c64_reg_${v}_$r.log
    rc=$?; echo "c64 reg $v $r rc=$rc"; cat gpurun_out/r05t/c64_reg_${v}_$r.json
    [ $rc -eq 0 ] || exit $rc
    E2E_CFGS=c64,c1500 timeout -k 10 200 python -u tools/e2e.py 1048576 65536 > gpurun_out/r05t/copied_${v}_$r.json 2> gpurun_out/r05t/copied_${v}_$r.log
    rc=$?; echo "copied $v $r rc=$rc"; cat gpurun_out/r05t/copied_${v}_$r.json
    [ $rc -eq 0 ] || exit $rc
  done
done
