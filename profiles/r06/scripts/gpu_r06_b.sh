#!/bin/bash
# Round 6: the in-round tail correction (no second read of each frame's last
# chunk): parity, then in-process A/B against the round-5 kernel, the PMC
# read bytes of CMIX, and a write-phase period sweep on CMIX.
cd $GRAFT_REPO_ROOT
source scripts/gpu_steps.sh
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step permit 300 $PT -s "tests/test_gpu_permit.py::test_permit_fused_commit_decision_is_agreed" \
  "tests/test_gpu_permit.py::test_permit_fused_abort_leaves_tokens_and_reports" || exit $?
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
export AB_LIBS=r05=tools/ab_r06/libpptkrx_r05.so AB_PLACE=1 AB_ROUNDS=7
for cfg in cmix c1500 imix jmix c64; do
  step ab_$cfg 300 python -u tools/ab.py $cfg -1:-1 r05:-1:-1 || exit $?
done
unset AB_LIBS AB_PLACE
export AB_ROUNDS=2 AB_REPS=3
step pmc_cmix_new 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d $O/pmc_new \
  -o run --output-format csv -- python3 tools/ab.py cmix -1:-1 || exit $?
export AB_LIBS=r05=tools/ab_r06/libpptkrx_r05.so
step pmc_cmix_r05 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rx_kernel -d $O/pmc_r05 \
  -o run --output-format csv -- python3 tools/ab.py cmix r05:-1:-1 || exit $?
# write-phase period sweep on CMIX (experiment build: PPTK_RX_PHASE_TICKS
# forces the period, 100 MHz ticks; the product's estimate beside it)
export AB_LIBS=exp=tools/ab_r06/libpptkrx_exp.so AB_PLACE=1 AB_ROUNDS=5 AB_REPS=5
for t in 0 1000 1360 1700 2000 2500 3200; do
  PPTK_RX_PHASE_TICKS=$t step sweep_cmix_$t 240 python -u tools/ab.py cmix -1:-1 exp:-1:-1 || exit $?
done
# last (a hang here ends the call): the round-5 teardown order replayed with
# the HIP runtime's API log, then the library's order
gcc -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tools/split_hang_repro.c -Lpptk_amd \
  -lpptkrx -Wl,-rpath,$PWD/pptk_amd -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -o $O/repro || exit 1
AMD_LOG_LEVEL=3 step repro_old 60 $O/repro old 4 || exit $?
AMD_LOG_LEVEL=3 step repro_new 60 $O/repro new 4 || exit $?
