"""BENCH TOOLING: in-process A/B of pptk_tx_rewrite_device across library
builds on one batch (source/destination/port rewrite of every frame, no TTL
change, so repeated launches stay steady).

    AB_LIBS=old=build/ab_old/libpptkrx.so python tools/ab_rewrite.py c64 "" old

Every build must leave identical bytes (checked on a fresh copy first)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pptk_amd.records import REWRITE_DTYPE
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    cfg = sys.argv[1]
    names = sys.argv[2:] or [""]
    libs = {"": None}
    for kv in filter(None, os.environ.get("AB_LIBS", "").split(",")):
        k, v = kv.split("=", 1)
        libs[k] = os.path.join(ROOT, v)
    n = int(os.environ.get("AB_FRAMES", 16 * 1024 * 1024))
    dev = torch.device("cuda", 0)
    b = make_batch(cfg, n, dev)
    kw = (dict(off=b["off"], lens=b["lens"]) if "off" in b
          else dict(stride=b["stride"], fixed_len=b["fixed_len"]))
    rw = np.zeros(1, REWRITE_DTYPE)
    rw["ops"], rw["src"], rw["dst"], rw["sport"], rw["dport"] = 0x1E, 0xC0A80A01, 0x0A000002, 4242, 443
    rw_t = torch.from_numpy(rw.view(np.uint8).copy()).to(dev)
    ctxs = {k: RxContext(0, bytes(range(1, 17)), lib_path=libs[k]) for k in names}
    orig = b["frames"].clone()
    ref = None
    same = {}
    for k in names:
        b["frames"].copy_(orig)
        ctxs[k].tx_rewrite_device(b["frames"], n, rw_t, **kw)
        torch.cuda.synchronize()
        if ref is None:
            ref = b["frames"].clone()
        same[k] = bool(torch.equal(ref, b["frames"]))
    del orig, ref
    times = {k: [] for k in names}
    for _ in range(5):
        for k in names:
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ctxs[k].tx_rewrite_device(b["frames"], n, rw_t, **kw)
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1))
    out = {"cfg": cfg, "frames": n}
    for k, t in times.items():
        ms = float(np.median(t))
        out[k or "new"] = {"ms": round(ms, 4), "mpkts": round(n / ms / 1e3, 1),
                           "same_bytes": same[k]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
