#!/bin/bash
# Round 5: host to host with the records copied back by DMA on a second
# stream per slot (experiment build, PPTK_RX_RECS_DMA=2: the copy-back of
# chunk k overlaps the frame copy of chunk k + 1) against the product
# (records stored by the kernel over PCIe); separate processes, alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05ae
export TMPDIR=/tmp
for r in 1 2; do
  for v in prod dma2; do
    if [ $v = dma2 ]; then export E2E_LIB=tools/ab_libs/exp.so PPTK_RX_RECS_DMA=2; else unset E2E_LIB PPTK_RX_RECS_DMA; fi
    E2E_CFGS=c64 E2E_REG_OUT=1 timeout -k 10 200 python -u tools/e2e.py 4194304 65536 > gpurun_out/r05ae/c64_reg_${v}_$r.json 2> gpurun_out/r05ae/c64_reg_${v}_$r.log
    rc=$?; echo "c64 reg $v $r rc=$rc"; cat gpurun_out/r05ae/c64_reg_${v}_$r.json
    [ $rc -eq 0 ] || exit $rc
    E2E_CFGS=c64,c1500 timeout -k 10 200 python -u tools/e2e.py 1048576 65536 > gpurun_out/r05ae/copied_${v}_$r.json 2> gpurun_out/r05ae/copied_${v}_$r.log
    rc=$?; echo "copied $v $r rc=$rc"; cat gpurun_out/r05ae/copied_${v}_$r.json
    [ $rc -eq 0 ] || exit $rc
  done
done
