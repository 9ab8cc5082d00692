"""BENCH TOOLING: the HBM side of C8G (8 x MI355X, 128 M x 1500 B, RCCL
all-gather of the flow hashes; BASELINE.json configs[4]) emulated on one
GPU.  Per batch, rank 0 of 8 writes its 16 M hashes into its slice of the
double-buffered gather buffer and the all-gather lands the other seven
ranks' 7 x 128 MiB there while the next batch streams its frames.  Here the
landing is a device copy of those bytes on a second stream, ordered exactly
as bench.py orders the real collective (after the batch that produced the
slice, overlapping the next one; batch k waits for the gather of k - 2).
What this cannot show is xGMI: RCCL's receive of 896 MiB per rank per batch
at ~0.5 TB/s takes ~1.7 ms, inside the ~4 ms batch.

Runs on the library's rings (pptk_rx_ring_alloc) with the gather buffers
from pptk_rx_gather_alloc (nranks 8, rank 0: its probe includes the
landing copies), and for comparison on a plain allocation of the same size.

    python tools/c8g_emul.py [steps]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(ctx, b, recs, n, kw, bufs, steps, land, dev):
    """ms per step: batches with their hashes into bufs[k % 2][0:n] and, when
    `land`, the other ranks' bytes copied into bufs[k % 2][n:] beside the
    next batch; bufs None: no hashes, no gather."""
    import torch
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    kdone = [torch.cuda.Event() for _ in range(2)]
    gdone = [torch.cuda.Event() for _ in range(2)]
    src = torch.zeros(7 * n, dtype=torch.int64, device=dev) if land else None

    def step(k):
        if bufs is None:
            ctx.batch_device(b["frames"], n, recs=recs, **kw)
            return
        out = bufs[k & 1]
        main.wait_event(gdone[k & 1])
        ctx.batch_device(b["frames"], n, recs=recs, hash_out=out[:n], **kw)
        kdone[k & 1].record(main)
        side.wait_event(kdone[k & 1])
        if land:
            with torch.cuda.stream(side):
                out[n:8 * n].copy_(src)
        gdone[k & 1].record(side)

    for k in range(40):            # settle (clocks)
        step(k)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    import torch
    import bench
    from pptk_amd.rx import RxContext
    from tools.synth import make_batch
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    n = bench.N_PER_GPU
    ctx = RxContext(0, bench.KEY)
    b = make_batch("c1500", n, dev)
    kw = dict(stride=b["stride"], fixed_len=b["fixed_len"])
    recs, rep = bench.ring_buffers(ctx, b, n, dev, False)
    time.sleep(max(0.0, rep["_freed_at"] + rep["freed_bytes"] / bench.SCRUB_BYTES_PER_S
                   - time.perf_counter()))
    ctx.autotune(b["frames"], n, recs=recs, reps=5, **kw)
    g = ctx.gather_alloc(b["frames"], n, n, 8, 0, recs=recs, **kw)
    placed = [g.out[0], g.out[1]]
    plain = [torch.zeros(8 * n, dtype=torch.int64, device=dev) for _ in range(2)]
    freed, _ = bench.release(dev)
    time.sleep(2.0 + g.report["freed_bytes"] / bench.SCRUB_BYTES_PER_S)
    res = {k: [] for k in ("none", "hashes_placed", "c8g_placed", "c8g_plain")}
    for _ in range(3):             # interleaved rounds
        res["none"].append(run(ctx, b, recs, n, kw, None, steps, False, dev))
        res["hashes_placed"].append(run(ctx, b, recs, n, kw, placed, steps, False, dev))
        res["c8g_placed"].append(run(ctx, b, recs, n, kw, placed, steps, True, dev))
        res["c8g_plain"].append(run(ctx, b, recs, n, kw, plain, steps, True, dev))
    ms = {k: round(float(np.median(v)), 4) for k, v in res.items()}
    out = {"frames_per_rank": n, "steps": steps, "ms_per_step": ms,
           "loss_vs_none": {k: round(1 - ms["none"] / v, 4) for k, v in ms.items() if k != "none"},
           "landing_bytes_per_batch": 7 * n * 8, "gather_probe": g.report,
           "ring": {k: rep[k] for k in ("chosen_frames", "chosen_recs", "chosen_ms",
                                        "plain_alloc_ms")}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
