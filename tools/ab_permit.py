"""BENCH TOOLING: in-process A/B of library builds on bench.py's
rate-limiter workload (16 M C64 records, 2^16 buckets).

    AB_LIBS=old=build/ab_old/libpptkrx.so python tools/ab_permit.py
    AB_KEYS=1 ...: from the dense keys (pptk_rx_permit_keys_device), as
                   bench.py's keys (AB_TOKENS=1048576) / keys_denying (128)
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
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n, hs = 16 * 1024 * 1024, 1 << 16
    libs = {"": None}
    for kv in filter(None, os.environ.get("AB_LIBS", "").split(",")):
        k, v = kv.split("=", 1)
        libs[k] = os.path.join(ROOT, v)
    b = make_batch("c64", n, dev)
    ctxs = {k: RxContext(0, bench.KEY, 24, 0, hs, lib_path=p) for k, p in libs.items()}
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    recs = ctxs[""].batch_device(b["frames"], n, stride=b["stride"], fixed_len=b["fixed_len"],
                                 key_out=keys)
    del b
    use_keys = bool(os.environ.get("AB_KEYS"))
    ntok = int(os.environ.get("AB_TOKENS", 200))

    def call(ctx, tok, verdict, scratch):
        if use_keys:
            ctx.permit_keys_device(keys, 4, tok, verdict=verdict, scratch=scratch)
        else:
            ctx.permit_device(recs, 4, tok, verdict=verdict, scratch=scratch)
    out, ref = {}, None
    times = {k: [] for k in libs}
    for _ in range(int(os.environ.get("AB_ROUNDS", 4))):
        for k, ctx in ctxs.items():
            tok = torch.full((hs,), ntok, dtype=torch.int32, device=dev)   # (200: buckets run dry)
            verdict = torch.empty(n, dtype=torch.uint8, device=dev)
            scratch = torch.empty(ctx._L.pptk_rx_permit_scratch_bytes(n, hs), dtype=torch.uint8,
                                  device=dev)
            call(ctx, tok, verdict, scratch)
            torch.cuda.synchronize()
            v = verdict.cpu().numpy()
            if ref is None:
                ref = v
            assert np.array_equal(v, ref), k
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if ntok < 1 << 16:
                    tok.fill_(ntok)          # (keys_denying: refilled before each batch)
                e0.record()
                call(ctx, tok, verdict, scratch)
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1))
    for k, t in times.items():
        out[k or "current"] = round(float(np.median(t)), 4)
    out["denied_first_batch"] = int((ref == 0).sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
