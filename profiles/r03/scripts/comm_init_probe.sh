cd $GRAFT_REPO_ROOT
export PPTK_RX_COMM_TRACE=1
run() {  # name, env..., mode
  name=$1; shift
  env "$@" timeout -k 5 40 python -u scripts/comm_init_probe.py $mode > gpurun_out/py_$name.log 2>&1
  echo "== $name rc=$?"; grep -v "alt_rsmi\|^$" gpurun_out/py_$name.log | grep -v "NCCL INFO\|version\|Hostname" | tail -12
}
mode=two run two PPTK_RX_LIB=$PWD/dbgexp/libpptkrx.so
mode=torch_two run torch_two PPTK_RX_LIB=$PWD/dbgexp/libpptkrx.so
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_comm.py tests/test_examples.py tests/test_gpu_tx.py -m gpu > gpurun_out/comm.log 2>&1; echo "pytest rc=$?"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/comm.log | tail -50
