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
    python tools/c8g_emul.py [steps] --standin B1,B2,..

--standin: instead of the copy, tools/libstandin.so's kernel with RCCL's
gfx950 footprint (512 threads, 37 664 B LDS, 248 VGPRs per block: a block
needs a whole CU) spinning STANDIN_US (default 1700) microseconds on B
blocks -- whether the persistent rx grid lets the collective's kernel run
beside the batch at all, or only between batches.  Run it under the
experiment build with PPTK_RX_RESERVE_CUS=k to leave k CUs free.
--mask K:top|spread|side: the batches run on a stream created with a CU mask
(hipExtStreamCreateWithCUMask) that leaves K CUs out -- the top K mask bits
or every (256/K)-th -- so the stand-in's blocks find whole CUs free; run it
under the experiment build with PPTK_RX_RESERVE_CUS=K (grid for the rest).
"side": as "top", and the second stream's mask holds just those K CUs.
--split K: the same through the library (pptk_rx_stream_split), product
build.  --copy: the stand-in also copies the 7 x 128 MiB landing bytes into
the gather buffer, paced to STANDIN_US (the collective's HBM side and its CU
footprint together).
Mask bit i names CU i // 8 of XCC i % 8, and CU c of an XCC sits in SE
c % 4 (tools/cumask_map.py): the top K bits are K / 8 CUs of every XCC,
spread over its SEs.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def SIDE(dev):
    import torch
    return torch.cuda.Stream(dev)


def masked_stream(dev, bits):
    """A torch stream over a HIP stream whose CU mask holds `bits`."""
    import ctypes
    import torch
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
    for i in bits:
        words[i // 32] |= 1 << (i % 32)
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.init()
    h = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), len(words), words) == 0
    return torch.cuda.ExternalStream(h.value, device=dev), [hex(w) for w in words]


def run(ctx, b, recs, n, kw, bufs, steps, land, dev):
    """ms per step: batches with their hashes into bufs[k % 2][0:n] and, when
    `land`, the other ranks' bytes copied into bufs[k % 2][n:] beside the
    next batch; bufs None: no hashes, no gather."""
    import torch
    main = torch.cuda.current_stream(dev)
    side = SIDE(dev)
    kdone = [torch.cuda.Event() for _ in range(2)]
    gdone = [torch.cuda.Event() for _ in range(2)]
    src = torch.zeros(7 * n, dtype=torch.int64, device=dev) if land is True else None

    def step(k):
        if bufs is None:
            ctx.batch_device(b["frames"], n, recs=recs, **kw)
            return
        out = bufs[k & 1]
        main.wait_event(gdone[k & 1])
        ctx.batch_device(b["frames"], n, recs=recs, hash_out=out[:n], **kw)
        kdone[k & 1].record(main)
        side.wait_event(kdone[k & 1])
        if land is True:
            with torch.cuda.stream(side):
                out[n:8 * n].copy_(src)
        elif land:
            land(side, out)
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
    global SIDE
    import torch
    import bench
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    n = bench.N_PER_GPU
    mask = None
    if "--mask" in sys.argv:
        k, pat = sys.argv[sys.argv.index("--mask") + 1].split(":")
        k = int(k)
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        out = (set(range(ncu - k, ncu)) if pat in ("top", "side") else
               {j for j in range(ncu) if j % (ncu // k) == ncu // k - 1})
        stream, words = masked_stream(dev, [i for i in range(ncu) if i not in out])
        torch.cuda.set_stream(stream)
        if pat == "side":
            # the second stream (the collective's) holds the complement
            SIDE = lambda d: masked_stream(d, sorted(out))[0]   # noqa: E731
        mask = {"excluded": k, "pattern": pat, "words": words}
    ctx = RxContext(0, bench.KEY)
    if "--split" in sys.argv:
        # the product's split (pptk_rx_stream_split): batches and the
        # second stream on disjoint CUs, the grid sized for the batches'
        k = int(sys.argv[sys.argv.index("--split") + 1])
        rx_s, coll_s = ctx.stream_split(k)
        torch.cuda.set_stream(rx_s)
        SIDE = lambda d: coll_s   # noqa: E731
        mask = {"split": k}
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
    if "--standin" in sys.argv:
        import ctypes
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libstandin.so"))
        lib.standin_run.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p]
        sink = torch.zeros(512, dtype=torch.int32, device=dev)
        ticks = int(os.environ.get("STANDIN_US", "1700")) * 100   # 100 MHz
        blocks = [int(x) for x in sys.argv[sys.argv.index("--standin") + 1].split(",")]

        trace = torch.zeros(3 * 256, dtype=torch.int64, device=dev)

        lib.standin_copy.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        copy = "--copy" in sys.argv
        src = torch.zeros(7 * n, dtype=torch.int64, device=dev) if copy else None

        def standin(nb):
            def land(side, out=None):
                if copy:
                    # the landing bytes, copied by the stand-in at xGMI pace
                    dst = out if out is not None else src
                    assert lib.standin_copy(nb, ticks, src.data_ptr(), dst[n:8 * n].data_ptr()
                                            if out is not None else dst.data_ptr(),
                                            7 * n * 8, side.cuda_stream) == 0
                    return
                assert lib.standin_run(nb, ticks, sink.data_ptr(), trace.data_ptr(),
                                       side.cuda_stream) == 0
            return land

        def starts(nb):
            # the last step's stand-in blocks: start spread (us) and where
            # the late ones (> 100 us after the first) ran
            t = trace[:3 * nb].view(nb, 3).cpu().tolist()
            t0 = min(r[0] for r in t)
            late = [(r[1], (r[2] >> 13) & 7) for r in t if r[0] - t0 > 10000]
            return {"spread_us": (max(r[0] for r in t) - t0) / 100, "late": len(late),
                    "late_xcc_se": sorted(set(late))[:16]}

        # the stand-in alone: its own duration on an idle chip
        side = torch.cuda.Stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(side)
        for _ in range(10):
            standin(max(blocks))(side)
        e1.record(side)
        torch.cuda.synchronize(dev)
        alone = e0.elapsed_time(e1) / 10
        res = {k: [] for k in ["none", "hashes_placed"] + [f"standin_{nb}" for nb in blocks]}
        st = {}
        for _ in range(3):
            res["none"].append(run(ctx, b, recs, n, kw, None, steps, False, dev))
            res["hashes_placed"].append(run(ctx, b, recs, n, kw, placed, steps, False, dev))
            for nb in blocks:
                res[f"standin_{nb}"].append(run(ctx, b, recs, n, kw, placed, steps,
                                                standin(nb), dev))
                if not copy:
                    st[nb] = starts(nb)
        ms = {k: round(float(np.median(v)), 4) for k, v in res.items()}
        print(json.dumps({"frames_per_rank": n, "steps": steps, "ms_per_step": ms,
                          "standin_alone_ms": round(alone, 4), "standin_starts": st, "standin_us": ticks // 100,
                          "reserve_cus": os.environ.get("PPTK_RX_RESERVE_CUS"),
                          "lib": os.environ.get("PPTK_RX_LIB"), "mask": mask,
                          "variant": ctx.last_variant() if hasattr(ctx, "last_variant")
                          else None}))
        return
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
