"""BENCH TOOLING: latency of pptk_rx_batch for small LDP-sized batches (the
rx loop hands out 32 - 4096 frames per ldp_in_nextpkts call): median
microseconds per call and the frame rate, staged and zero-copy ring; and
the same batches through pptk_rx_batch_submit / _complete E2E_DEPTH deep
(default 2; `pipe_*`: microseconds per batch in a steady loop of
back-to-back submissions, what an rx loop that overlaps batches gets).

    python tools/e2e_small.py [cfg]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pptk_amd.records import REC_DTYPE, diff_records
    from pptk_amd.rx import RxContext, ldp_packets
    from harness.synth import make_batch
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c64"
    dev = torch.device("cuda", 0)
    sizes = [int(x) for x in os.environ.get("E2E_SIZES", "32,256,1024,4096").split(",")]
    nmax = max(sizes)
    b = make_batch(cfg, nmax, dev)
    stride = b["stride"]
    ring = b["frames"][: nmax * stride + 64].cpu().numpy()
    want = RxContext(0, bytes(range(1, 17))).batch_device(
        b["frames"], nmax, stride=stride, fixed_len=b["fixed_len"]).cpu().numpy()
    # E2E_OUT=fresh: a new record array per call (the earlier measurement);
    # reuse (default): one array reused; reg: reused and registered, so the
    # records land in it directly
    out_mode = os.environ.get("E2E_OUT", "reuse")
    out = {"cfg": cfg, "out": out_mode,
           "gather_threads": int(os.environ.get("E2E_GATHER_THREADS", "1"))}
    depth = int(os.environ.get("E2E_DEPTH", "2"))
    out["depth"] = depth
    both = np.zeros(depth * nmax, dtype=REC_DTYPE)     # a record array per batch in flight
    outbuf = both[:nmax]
    for mode in ("staged", "ring"):
        ctx = RxContext(0, bytes(range(1, 17)), max_batch=nmax, max_frame=1518,
                        gather_threads=int(os.environ.get("E2E_GATHER_THREADS", "1")),
                        lib_path=os.environ.get("E2E_LIB"))    # A/B: another build
        if mode == "ring":
            ctx.register_ring(ring)
        if out_mode == "reg":
            ctx.register_ring(both)
        for n in sizes:
            pkts = ldp_packets(ring, np.arange(n, dtype=np.uint64) * stride,
                               np.full(n, b["fixed_len"], np.uint16))
            o = None if out_mode == "fresh" else outbuf[:n]
            got = ctx.batch_host(pkts, out=o)
            assert not diff_records(got, want[:n]), (mode, n)
            ts = []
            for _ in range(300 if n <= 4096 else 60):
                t0 = time.perf_counter()
                ctx.batch_host(pkts, out=o)
                ts.append(time.perf_counter() - t0)
            us = float(np.median(ts)) * 1e6
            out[f"{mode}_{n}"] = {"us_per_call": round(us, 1), "mpkts": round(n / us, 2)}
            if hasattr(ctx._L, "pptk_rx_batch_submit"):
                outs = [both[j * nmax:j * nmax + n] for j in range(depth)]
                reps = 300 if n <= 4096 else 60
                runs = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    for k in range(reps):
                        if ctx.pending_host() == depth:
                            ctx.complete_host()
                        ctx.submit_host(pkts, outs[k % depth])
                    while ctx.pending_host():
                        ctx.complete_host()
                    runs.append((time.perf_counter() - t0) / reps)
                for o_ in outs:
                    assert not diff_records(o_.copy(), want[:n]), ("pipe", mode, n)
                us = float(np.median(runs)) * 1e6
                out[f"pipe_{mode}_{n}"] = {"us_per_batch": round(us, 1),
                                           "mpkts": round(n / us, 2)}
        if mode == "ring":
            ctx.unregister_ring(ring)
        if out_mode == "reg":
            ctx.unregister_ring(both)
        ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
