"""BENCH TOOLING: what the dense flow-hash writes (the multi-GPU all-gather's
send slice, pptk_rx_dev_batch.d_hash) cost beside the C1500 frame stream, and
what decides it.  On the library's rings (pptk_rx_ring_alloc, as bench.py),
after the scrub: the batch without hashes, and with its hashes into the
library-placed gather buffer (pptk_rx_gather_alloc) and into several fresh
buffers allocated 4 GB apart -- interleaved rounds, median kernel ms.  Then
the same on a second ring allocation (another frame/record placement) and
on a third placed with the hash stream in its probe (PPTK_RX_RING_PROBE_HASH).

    python tools/hash_probe.py [rounds]
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
    import bench
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    dev = torch.device("cuda", 0)
    n = bench.N_PER_GPU
    ctx = RxContext(0, bench.KEY)
    out = {"frames": n}
    for ring_k in range(3):
        b = make_batch("c1500", n, dev)
        kw = dict(stride=b["stride"], fixed_len=b["fixed_len"])
        # rings 0 and 1: placed for the records alone (two allocations);
        # ring 2: placed with the hash stream in the probe
        recs, rep = bench.ring_buffers(ctx, b, n, dev, False, probe_hash=ring_k == 2)
        time.sleep(max(0.0, rep["_freed_at"] + rep["freed_bytes"] / bench.SCRUB_BYTES_PER_S
                       - time.perf_counter()))
        ctx.autotune(b["frames"], n, recs=recs, reps=5, **kw)
        g = ctx.gather_alloc(b["frames"], n, n, 1, 0, recs=recs, **kw)
        hold, bufs = [], {"gather": g.out[0][:n]}
        for k in range(4):
            hold.append(torch.empty(4 << 30, dtype=torch.uint8, device=dev))
            bufs[f"fresh{k}"] = torch.empty(n, dtype=torch.int64, device=dev)
        del hold
        bench.release(dev)
        time.sleep(1.5)
        names = ["none"] + list(bufs)
        times = {k: [] for k in names}
        for _ in range(rounds):
            for k in names:
                h = None if k == "none" else bufs[k]
                for rep_i in range(6):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    ctx.batch_device(b["frames"], n, recs=recs, hash_out=h, **kw)
                    e1.record()
                    torch.cuda.synchronize()
                    if rep_i:
                        times[k].append(e0.elapsed_time(e1))
        out[f"ring{ring_k}"] = {
            "ring": {k: rep[k] for k in ("chosen_frames", "chosen_recs", "chosen_ms",
                                         "plain_alloc_ms")},
            "gather_probe": g.report,
            "ms": {k: round(float(np.median(v)), 4) for k, v in times.items()}}
        print(json.dumps(out[f"ring{ring_k}"]["ms"]), file=sys.stderr, flush=True)
        del b, recs, g, bufs
        bench.release(dev)
        time.sleep(2.0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
