"""BENCH TOOLING: in-process A/B of tx-side (pptk_tx_cksum_device) settings
on one batch.  python tools/ab_tx.py c1500 3:32 3:33 3:544 ...
(variant:flags; flag 512 = diagnostics, no checksum writes; a setting
lib:variant:flags uses the library build AB_LIBS names lib, e.g.
AB_LIBS=old=build/ab_old/libpptkrx.so ... -1:-1 old:-1:-1)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    cfg = sys.argv[1]
    def parse(a):
        p = a.split(":")
        return (p[0], int(p[1]), int(p[2])) if len(p) == 3 else ("", int(p[0]), int(p[1]))
    settings = [parse(a) for a in sys.argv[2:]]
    libs = {"": None}
    for kv in filter(None, os.environ.get("AB_LIBS", "").split(",")):
        k, v = kv.split("=", 1)
        libs[k] = os.path.join(ROOT, v)
    n = int(os.environ.get("AB_FRAMES", 16 * 1024 * 1024))
    dev = torch.device("cuda", 0)
    b = make_batch(cfg, n, dev)
    kw = (dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]) if "off" in b
          else dict(stride=b["stride"], fixed_len=b["fixed_len"]))
    ctxs = {k: RxContext(0, bytes(range(1, 17)), lib_path=v) for k, v in libs.items()}
    times = {s: [] for s in settings}
    for _ in range(5):
        for s in settings:
            ctx = ctxs[s[0]]
            ctx.set_tuning(s[1], s[2])
            ctx.tx_cksum_device(b["frames"], n, **kw)
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ctx.tx_cksum_device(b["frames"], n, **kw)
                e1.record()
                torch.cuda.synchronize()
                times[s].append(e0.elapsed_time(e1))
    out = {"cfg": cfg, "frames": n}
    for s, t in times.items():
        ms = float(np.median(t))
        out[":".join(str(x) for x in s if x != "")] = {"ms": round(ms, 4), "gbs": round(b["bytes"] / ms / 1e6, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
