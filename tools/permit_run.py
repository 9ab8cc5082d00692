"""BENCH TOOLING: run bench.py's rate-limiter workload once (for rocprofv3
wrapping): python tools/permit_run.py [runs] [--ab]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stamps():
    """The fused rate limiter's phase timestamps (workgroup 0, 100 MHz
    clock, PermitFused::sync[8..15]) on 16 M dense keys, 2^16 buckets, as
    bench's keys / keys_denying runs: microseconds from the kernel's start."""
    import numpy as np
    import torch
    from pptk_amd.rx import RxContext
    dev = torch.device("cuda", 0)
    n, hs = 16 * 1024 * 1024, 1 << 16
    ctx = RxContext(0, bytes(range(1, 17)), 24, 0, hs)
    keys = torch.randint(0, hs, (n,), dtype=torch.int32, device=dev)
    scratch = torch.zeros(ctx._L.pptk_rx_permit_scratch_bytes(n, hs), dtype=torch.uint8, device=dev)
    out = {}
    for name, t in (("keys", 1 << 20), ("keys_denying", 128)):
        rows = []
        for _ in range(8):
            tok = torch.full((hs,), t, dtype=torch.int32, device=dev)
            ctx.permit_keys_device(keys, 4, tok, scratch=scratch)
            torch.cuda.synchronize()
            w = scratch[:64].view(torch.int32).cpu().numpy().view(np.uint32)
            st = w[8:16].astype(np.int64)
            rows.append([round(float(x - st[0]) / 100.0, 2) for x in st])
        out[name] = {"phase_stamps_us": rows[len(rows) // 2],
                     "labels": ["start", "row written", "barrier 1", "phase 2", "barrier 2",
                                "code staged", "resolved", "verdicts"]}
    print(json.dumps(out), flush=True)


def main():
    import torch
    import bench
    if "--stamps" in sys.argv:
        return stamps()
    dev = torch.device("cuda", 0)
    runs = tuple(sys.argv[1].split(",")) if len(sys.argv) > 1 else ("records", "keys",
                                                                     "keys_denying")
    ab = "--ab" in sys.argv
    print(json.dumps({"fused": bench.permit_bench(16 * 1024 * 1024, dev, 1, 0, 20, 3, runs=runs)}),
          flush=True)
    if ab:   # the four-launch path on the same workload
        print(json.dumps({"passes": bench.permit_bench(16 * 1024 * 1024, dev, 1, 0, 20, 3, runs=runs,
                                                       tune=0x400)}), flush=True)


if __name__ == "__main__":
    main()
