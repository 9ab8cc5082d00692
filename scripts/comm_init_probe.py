"""Debug: communicator creation variants (scripts/comm_init_probe.sh; needs an experiment build, make abvariant NAME=exp DEFS=-DPPTK_RX_EXPERIMENTS, copied to dbgexp/)."""
import sys, threading, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
mode = sys.argv[1]
if "torch" in mode:
    import torch
    torch.zeros(1, device="cuda:0"); torch.cuda.synchronize()
from pptk_amd.rx import RxContext, comm_uid
ctx = RxContext(0, bytes(range(1, 17)), comm_timeout_ms=3000)
t0 = time.monotonic()
try:
    ctx.comm_create(1, 0, comm_uid()); ctx.comm_destroy()
    print("one-rank ok", round(time.monotonic() - t0, 2), flush=True)
except OSError as e:
    print("one-rank err", e, flush=True)
if "two" in mode:
    t0 = time.monotonic()
    try:
        ctx.comm_create(2, 0, comm_uid())
        print("two-rank ok?!", flush=True)
    except OSError as e:
        print("two-rank", -e.errno, round(time.monotonic() - t0, 2), flush=True)
print("end", flush=True)
