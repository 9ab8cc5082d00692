"""PROBE: what RCCL's INFO log says about the channel count of a one-rank
communicator created through the library, on a split context (maxCTAs =
coll_cus), unsplit, and unsplit under NCCL_MAX_NCHANNELS / NCCL_MAX_CTAS.
Writes each child's full log to <outdir>/<case>.log and prints the lines that
name channels or CTAs.

    python tools/comm_cap_probe.py outdir"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = """
import sys; sys.path.insert(0, %r)
import torch; torch.cuda.init()
from pptk_amd.rx import RxContext, comm_uid
ctx = RxContext(0, bytes(range(1, 17)))
if %d: ctx.stream_split(%d)
ctx.comm_create(1, 0, comm_uid())
h = torch.zeros(1 << 20, dtype=torch.int64, device="cuda")
ctx.allgather_hash(h, 1 << 20, h)
torch.cuda.synchronize()
ctx.close()
print("child ok")
"""


def run(name, split, extra, outdir):
    env = dict(os.environ, NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="ALL")
    for k in ("NCCL_MAX_NCHANNELS", "NCCL_MAX_CTAS"):
        env.pop(k, None)
    env.update(extra)
    out = subprocess.run([sys.executable, "-c", CHILD % (ROOT, split, split)],
                         capture_output=True, text=True, timeout=180, env=env)
    log = out.stdout + out.stderr
    with open(os.path.join(outdir, name + ".log"), "w") as f:
        f.write(log)
    lines = [ln for ln in log.splitlines()
             if re.search(r"[Cc]hannel|CTA|[Cc]tas\b|nc=|maxC", ln)]
    print(f"== {name}: rc {out.returncode}, {len(lines)} lines")
    for ln in lines[:40]:
        print("   ", ln[-200:])


def main():
    outdir = sys.argv[1]
    os.makedirs(outdir, exist_ok=True)
    run("split32", 32, {}, outdir)
    run("unsplit", 0, {}, outdir)
    run("env_nchannels32", 0, {"NCCL_MAX_NCHANNELS": "32"}, outdir)
    run("env_ctas32", 0, {"NCCL_MAX_CTAS": "32"}, outdir)


if __name__ == "__main__":
    main()
