"""BENCH TOOLING: in-process A/B of library builds on bench.py's
rate-limiter workload (16 M C64 records, 2^16 buckets).

    AB_LIBS=old=build/ab_old/libpptkrx.so python tools/ab_permit.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pptk_amd.rx import RxContext
    from tools.synth import make_batch
    dev = torch.device("cuda", 0)
    n, hs = 16 * 1024 * 1024, 1 << 16
    libs = {"": None}
    for kv in filter(None, os.environ.get("AB_LIBS", "").split(",")):
        k, v = kv.split("=", 1)
        libs[k] = os.path.join(ROOT, v)
    b = make_batch("c64", n, dev)
    ctxs = {k: RxContext(0, bench.KEY, 24, 0, hs, lib_path=p) for k, p in libs.items()}
    recs = ctxs[""].batch_device(b["frames"], n, stride=b["stride"], fixed_len=b["fixed_len"])
    del b
    out, ref = {}, None
    times = {k: [] for k in libs}
    for _ in range(4):
        for k, ctx in ctxs.items():
            tok = torch.full((hs,), 200, dtype=torch.int32, device=dev)   # buckets run dry
            verdict = torch.empty(n, dtype=torch.uint8, device=dev)
            scratch = torch.empty(ctx._L.pptk_rx_permit_scratch_bytes(n, hs), dtype=torch.uint8,
                                  device=dev)
            ctx.permit_device(recs, 4, tok, verdict=verdict, scratch=scratch)
            torch.cuda.synchronize()
            v = verdict.cpu().numpy()
            if ref is None:
                ref = v
            assert np.array_equal(v, ref), k
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ctx.permit_device(recs, 4, tok, verdict=verdict, scratch=scratch)
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1))
    for k, t in times.items():
        out[k or "current"] = round(float(np.median(t)), 4)
    out["denied_first_batch"] = int((ref == 0).sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
