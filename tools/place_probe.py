"""BENCH TOOLING: does the C1500 launch time depend on WHERE the record
buffer sits in HBM relative to the frame buffer?

    python tools/place_probe.py [--step-mb 16] [--count 32] [--reps 4]

One frame batch; one record pool of 1 GiB + count * step MB; the same
C1500 launch timed with its records at pool + k * step MB for k in
0..count-1, interleaved over `reps` rounds (medians).  One JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def matrix(args):
    import torch
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    hold = []
    bs = [make_batch("c1500", n, dev)]
    for k in range(1, args.batches):
        if args.spacer_gb:
            hold.append(torch.empty(int(args.spacer_gb * (1 << 30)), dtype=torch.uint8,
                                    device=dev))
        bs.append(make_batch("c1500", n, dev, first=k * n))
    rs = []
    for _ in range(args.matrix):
        if args.spacer_gb:
            hold.append(torch.empty(int(args.spacer_gb * (1 << 30)), dtype=torch.uint8,
                                    device=dev))
        rs.append(torch.zeros((n, 64), dtype=torch.uint8, device=dev))
    torch.cuda.synchronize()
    t = {}
    for rep in range(args.reps + 1):
        for bi, b in enumerate(bs):
            for ri, r in enumerate(rs):
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                ctx.batch_device(b["frames"], n, stride=1500, fixed_len=1500, recs=r)
                z.record()
                torch.cuda.synchronize()
                if rep:
                    t.setdefault((bi, ri), []).append(a.elapsed_time(z))
    m = [[round(sorted(t[(bi, ri)])[len(t[(bi, ri)]) // 2], 3) for ri in range(len(rs))]
         for bi in range(len(bs))]
    print(json.dumps({"rx_ms": m, "frames": [hex(b["frames"].data_ptr()) for b in bs],
                      "recs": [hex(r.data_ptr()) for r in rs]}), flush=True)


def policies(args):
    """The slow (allocated right after the frames) and a fast record buffer,
    each under every result-preserving store/load policy (PPTK_RX_TUNE_*
    bits via pptk_rx_set_tuning) and the rwmix speed-of-light kernel's
    store modes."""
    import torch
    from pptk_amd.rx import RxContext
    from harness.rwmix import mix_ms
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    b = make_batch("c1500", n, dev)
    rs = [torch.zeros((n, 64), dtype=torch.uint8, device=dev) for _ in range(6)]
    torch.cuda.synchronize()
    pols = {"nt_ld+nt_st": 0x21, "nt_ld+wb_st": 0x1, "nt_ld+sc1_st": 0x41, "wb_ld+nt_st": 0x20,
            "nt_ld+nt_st+blocked": 0x121, "nt_ld+lane_st": 0x23}
    t = {}
    for rep in range(args.reps + 1):
        for ri in (0, 1, 5):
            for name, fl in pols.items():
                ctx.set_tuning(-1, fl)
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                ctx.batch_device(b["frames"], n, stride=1500, fixed_len=1500, recs=rs[ri])
                z.record()
                torch.cuda.synchronize()
                if rep:
                    t.setdefault(f"r{ri}/{name}", []).append(a.elapsed_time(z))
    out = {k: round(sorted(v)[len(v) // 2], 3) for k, v in t.items()}
    for ri in (0, 1, 5):
        for nt in (0, 1, 3, 9):
            out[f"r{ri}/rwmix_nt{nt}"] = round(mix_ms(b["frames"], 96000, n // 64, rs[ri], 4096,
                                                      nt=nt), 3)
    print(json.dumps(out), flush=True)


def orders(args):
    """Allocation-order experiment: a record buffer allocated BEFORE the
    frame batch, six after it, and one arena holding both (frames copied
    into its first 24 GB, records right after) -- which placements are
    slow, and is any allocation strategy reliably fast?"""
    import torch
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    rb = torch.zeros((n, 64), dtype=torch.uint8, device=dev)
    b = make_batch("c1500", n, dev)
    ra = [torch.zeros((n, 64), dtype=torch.uint8, device=dev) for _ in range(6)]
    fb = n * 1500
    arena = torch.empty(fb + 64 + n * 64 + (2 << 20), dtype=torch.uint8, device=dev)
    arena[:fb + 64].copy_(b["frames"][:fb + 64])
    off = (fb + 64 + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    arec = arena[off:off + n * 64].view(n, 64)
    torch.cuda.synchronize()
    cases = {"before": (b["frames"], rb), "arena": (arena, arec)}
    cases.update({f"after{k}": (b["frames"], r) for k, r in enumerate(ra)})
    cases["arena_frames+before"] = (arena, rb)
    t = {}
    for rep in range(args.reps + 1):
        for name, (fr, r) in cases.items():
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ctx.batch_device(fr, n, stride=1500, fixed_len=1500, recs=r)
            z.record()
            torch.cuda.synchronize()
            if rep:
                t.setdefault(name, []).append(a.elapsed_time(z))
    print(json.dumps({k: round(sorted(v)[len(v) // 2], 3) for k, v in t.items()}), flush=True)


def flags(args):
    """Record buffers from hipExtMallocWithFlags with each allocation flag
    (default, fine-grained, uncached, contiguous), several of each, the same
    C1500 launch into each: does an allocation kind avoid the slow class?"""
    import ctypes
    import torch
    from pptk_amd.rx import RxContext, RxDevBatch
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    b = make_batch("c1500", n, dev)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                          ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    kinds = {"default": 0, "finegrained": 1, "uncached": 3, "contiguous": 4}
    bufs = []
    for rep in range(3):
        for name, fl in kinds.items():
            p = ctypes.c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(p), n * 64, fl)
            bufs.append((f"{name}{rep}", p if rc == 0 else None, rc))
    s = torch.cuda.current_stream(dev)
    t = {}
    for rnd in range(args.reps + 1):
        for name, p, rc in bufs:
            if p is None:
                continue
            bb = RxDevBatch(b["frames"].data_ptr(), None, None, None, 1500, 1500, 1500, n,
                            p.value, None, None, None)
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            r = ctx._L.pptk_rx_batch_device(ctx._ctx, ctypes.byref(bb),
                                             ctypes.c_void_p(s.cuda_stream))
            z.record()
            torch.cuda.synchronize()
            if r == 0 and rnd:
                t.setdefault(name, []).append(a.elapsed_time(z))
    out = {k: round(sorted(v)[len(v) // 2], 3) for k, v in t.items()}
    out["alloc_errors"] = {name: rc for name, p, rc in bufs if p is None}
    for _, p, _ in bufs:
        if p is not None:
            hip.hipFree(p)
    print(json.dumps(out), flush=True)


def keep(args):
    """Does a placed pair stay fast?  Frames + 8 record candidates behind 4 GB
    spacers, each timed; then the best is re-timed (a) with everything still
    allocated, (b) after the other candidates and the spacers are freed
    (empty_cache), (c) over a sustained run of 300 launches."""
    import torch
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    b = make_batch("c1500", n, dev)
    hold, rs = [], []
    for _ in range(8):
        hold.append(torch.empty(4 << 30, dtype=torch.uint8, device=dev))
        rs.append(torch.empty((n, 64), dtype=torch.uint8, device=dev))

    def t(r, k=5):
        ts = []
        for _ in range(k + 1):
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ctx.batch_device(b["frames"], n, stride=1500, fixed_len=1500, recs=r)
            z.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(z))
        return round(sorted(ts[1:])[k // 2], 3)
    cand = [t(r) for r in rs]
    bi = min(range(8), key=lambda i: cand[i])
    wi = max(range(8), key=lambda i: cand[i])
    out = {"candidates": cand, "best": bi, "best_again": t(rs[bi]), "worst_again": t(rs[wi])}
    best, worst = rs[bi], rs[wi]
    del hold, rs
    torch.cuda.empty_cache()
    out["best_after_free"] = t(best)
    out["worst_after_free"] = t(worst)
    sus = []
    for k in range(300):
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ctx.batch_device(b["frames"], n, stride=1500, fixed_len=1500, recs=best)
        z.record()
        if k % 50 == 49:
            torch.cuda.synchronize()
            sus.append(round(a.elapsed_time(z), 3))
    torch.cuda.synchronize()
    out["best_sustained_every50"] = sus
    print(json.dumps(out), flush=True)


def benchpath(args):
    """bench.placed_buffers as bench.py calls it, then a sustained run on
    the chosen pair: is the probe's time what the sustained run gets?"""
    import torch
    import bench
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    b = make_batch("c1500", n, dev)
    kw = dict(stride=1500, fixed_len=1500)
    out = {}
    for mode in ("pairs", "records"):
        recs, rep = bench.placed_buffers(ctx, b, n, dev, False, kw, frames=mode == "pairs")
        sus = []
        for k in range(200):
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ctx.batch_device(b["frames"], n, recs=recs, **kw)
            z.record()
            if k % 40 == 39:
                torch.cuda.synchronize()
                sus.append(round(a.elapsed_time(z), 3))
        torch.cuda.synchronize()
        out[mode] = {"chosen": rep["chosen"], "probe_ms": rep["chosen_ms"],
                     "as_allocated": rep["as_allocated_ms"], "sustained": sus}
        del recs
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


def txplace(args):
    """Does the tx kernel (checksums set in place: the writes land in the
    frame buffer itself) depend on where the frame buffer sits?  The same
    C1500 batch copied into `--batches` buffers allocated behind 8 GB
    spacers; tx timed on each, interleaved rounds, median per buffer."""
    import torch
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    b = make_batch("c1500", n, dev)
    kw = dict(stride=1500, fixed_len=1500)
    hold, fr = [], [b["frames"]]
    for _ in range(max(1, args.batches) - 1):
        hold.append(torch.empty(8 << 30, dtype=torch.uint8, device=dev))
        t = torch.empty_like(b["frames"])
        t.copy_(b["frames"])
        fr.append(t)
    del hold
    torch.cuda.synchronize()
    time.sleep(4.0)                     # the scrub of the freed spacers
    ms = [[] for _ in fr]
    for _ in range(5):
        for i, f in enumerate(fr):
            for k in range(4):
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                ctx.tx_cksum_device(f, n, **kw)
                z.record()
                torch.cuda.synchronize()
                if k:
                    ms[i].append(a.elapsed_time(z))
    print(json.dumps({"tx_ms_per_frame_buffer": [round(sorted(v)[len(v) // 2], 4) for v in ms]}),
          flush=True)


def txside(args):
    """Two-pass tx on placed frames: does the side array's placement matter
    like a record buffer's?  The side array as the context allocates it,
    the placed record buffer, and six fresh buffers 4 GB apart; tx timed on
    each (interleaved rounds, median)."""
    import torch
    import bench
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    b = make_batch("c1500", n, dev)
    kw = dict(stride=1500, fixed_len=1500)
    recs, rep = bench.placed_buffers(ctx, b, n, dev, False, kw)
    hold, cands = [], []
    for _ in range(6):
        hold.append(torch.empty(4 << 30, dtype=torch.uint8, device=dev))
        cands.append(torch.empty(n * 8, dtype=torch.uint8, device=dev))
    del hold
    torch.cuda.synchronize()
    time.sleep(max(4.0, rep.get("freed_bytes", 0) / 20e9 + 2.0))
    sides = [None, recs] + cands
    ms = [[] for _ in sides]
    for _ in range(4):
        for i, sd in enumerate(sides):
            ctx.tx_set_side_buffer(sd)
            for k in range(4):
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                ctx.tx_cksum_device(b["frames"], n, **kw)
                z.record()
                torch.cuda.synchronize()
                if k:
                    ms[i].append(a.elapsed_time(z))
    med = [round(sorted(v)[len(v) // 2], 4) for v in ms]
    print(json.dumps({"placement_chosen_ms": rep["chosen_ms"], "tx_ms_own_side": med[0],
                      "tx_ms_side_in_records": med[1], "tx_ms_side_candidates": med[2:]}),
          flush=True)


def bursts(args):
    """Does a longer record-write burst rescue a slow (frames, records)
    pair?  Frame batches (each behind a spacer) x record buffers (each behind
    a spacer), as bench.placed_buffers allocates them; per pair the rx launch
    and the trivial read/write kernel (tools/rwmix.hip rw_kernel, non-
    temporal) moving the same bytes with the records written in bursts of
    4 KB per 96 KB tile (the rx kernel's flush), 16 KB per 4 tiles and 64 KB
    per 16 tiles.  One JSON line: per pair the medians."""
    import ctypes
    import torch
    from pptk_amd.rx import RxContext
    from harness.rwmix import _lib, sol_ms
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    L = _lib()
    hold, bs, rs = [], [], []
    for k in range(args.batches):
        if k:
            hold.append(torch.empty(8 << 30, dtype=torch.uint8, device=dev))
        bs.append(make_batch("c1500", n, dev, first=k * n))
    for _ in range(args.matrix or 4):
        hold.append(torch.empty(4 << 30, dtype=torch.uint8, device=dev))
        rs.append(torch.zeros((n, 64), dtype=torch.uint8, device=dev))
    sink = torch.zeros(64, dtype=torch.int32, device=dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    s = torch.cuda.current_stream(dev)
    modes = [("rx", 0, 0), ("mix4k", 96000, 4096), ("mix16k", 4 * 96000, 16384),
             ("mix32k", 8 * 96000, 32768), ("mix64k", 16 * 96000, 65536),
             ("mix128k", 32 * 96000, 131072), ("mix256k", 64 * 96000, 262144),
             ("defer4", 96000, 4096), ("defer16", 96000, 4096),
             ("stage1", 96000, 4096), ("stage2", 96000, 4096), ("stage4", 96000, 4096),
             ("stage2s", 96000, 4096), ("sol", 96000, 4096)]
    t, sol_how = {}, {}
    torch.cuda.synchronize()
    for rep in range(args.reps + 1):
        for bi, b in enumerate(bs):
            for ri, r in enumerate(rs):
                for name, rb, wb in modes:
                    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    if name == "rx":
                        ctx.batch_device(b["frames"], n, stride=1500, fixed_len=1500, recs=r)
                    elif name == "sol":
                        if rep == 1:
                            ms, how = sol_ms(b["frames"], n, r, 4096, rb=96000, reps=2)
                            t[(bi, ri, name)] = [ms]
                            sol_how[f"{bi},{ri}"] = how
                        continue
                    elif name.startswith("stage"):
                        # stageN: 36 KB of header-image LDS as in the rx kernel;
                        # stage2s: the same burst with no pad (occupancy bound by
                        # the staging alone)
                        if L.rwstage_run(b["frames"].data_ptr(), r.data_ptr(), n * 1500 // rb,
                                         rb, wb, int(name[5]), 0 if name.endswith("s") else 36864,
                                         ncu * 2, sink.data_ptr(),
                                         ctypes.c_void_p(s.cuda_stream)):
                            continue
                    elif name.startswith("defer"):
                        L.rwdefer_run(b["frames"].data_ptr(), r.data_ptr(), n * 1500 // rb, rb,
                                      wb, int(name[5:]), ncu * 2, sink.data_ptr(),
                                      ctypes.c_void_p(s.cuda_stream))
                    else:
                        L.rwmix_run(b["frames"].data_ptr(), r.data_ptr(), n * 1500 // rb, rb, wb, 1,
                                    ncu * 2, sink.data_ptr(), ctypes.c_void_p(s.cuda_stream))
                    z.record()
                    torch.cuda.synchronize()
                    if rep:
                        t.setdefault((bi, ri, name), []).append(a.elapsed_time(z))
    out = {}
    for (bi, ri, name), v in sorted(t.items()):
        out.setdefault(f"{bi},{ri}", {})[name] = round(sorted(v)[len(v) // 2], 3)
    print(json.dumps({"pairs": out, "sol_setting": sol_how}), flush=True)


def xstage(args):
    """Round-4 probe: records staged per XCD group and flushed as 256 KB
    runs (tools/rwmix.hip rw_xstage_kernel) against the rx kernel and the
    4 KB / 256 KB burst kernels, on every (frames, records) pair as
    `bursts` allocates them.  One JSON line: per pair the medians, plus the
    blockIdx -> XCC census of the probe's grid."""
    import ctypes
    import torch
    from pptk_amd.rx import RxContext
    from harness.rwmix import _lib
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    L = _lib()
    vp = ctypes.c_void_p
    L.rwxstage_run.argtypes = [vp, vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32,
                               ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, vp, vp]
    L.rwxstage_run.restype = ctypes.c_int
    L.xcc_census.argtypes = [vp, ctypes.c_int, vp]
    L.rwblk_run.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                            ctypes.c_int, ctypes.c_int, vp, vp]
    hold, bs, rs = [], [], []
    for k in range(args.batches):
        if k:
            hold.append(torch.empty(8 << 30, dtype=torch.uint8, device=dev))
        bs.append(make_batch("c1500", n, dev, first=k * n))
    for _ in range(args.matrix or 2):
        hold.append(torch.empty(4 << 30, dtype=torch.uint8, device=dev))
        rs.append(torch.zeros((n, 64), dtype=torch.uint8, device=dev))
    sink = torch.zeros(64, dtype=torch.int32, device=dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    s = torch.cuda.current_stream(dev)
    ntiles = n * 1500 // 96000
    stg = torch.empty(8 * 32 * 64 * 4096, dtype=torch.uint8, device=dev)
    cnt = torch.zeros((ntiles + 63) // 64 + 64, dtype=torch.int32, device=dev)
    gen = torch.zeros(8 * 32, dtype=torch.int32, device=dev)
    census = torch.zeros(ncu * 2, dtype=torch.int32, device=dev)
    L.xcc_census(census.data_ptr(), ncu * 2, vp(s.cuda_stream))
    torch.cuda.synchronize()
    cen = census.tolist()
    groups_ok = all(cen[b] == cen[b % 8] for b in range(len(cen)))
    modes = [("rx", 0, 0), ("mix4k", 96000, 4096), ("mix256k", 64 * 96000, 262144),
             ("xorder", 0, 0), ("xst4nosync", 4, 5), ("xst8nosync", 8, 5),
             ("xst16nosync", 16, 5), ("xst8nosync_nt", 8, 7)]
    t = {}
    for rep in range(args.reps + 1):
        for bi, b in enumerate(bs):
            for ri, r in enumerate(rs):
                for name, p1, p2 in modes:
                    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    if name == "rx":
                        ctx.batch_device(b["frames"], n, stride=1500, fixed_len=1500, recs=r)
                    elif name.startswith("blk"):
                        L.rwblk_run(b["frames"].data_ptr(), r.data_ptr(), ntiles, 96000, 4096, p1,
                                    ncu * 2, sink.data_ptr(), vp(s.cuda_stream))
                    elif name.startswith("mix"):
                        L.rwmix_run(b["frames"].data_ptr(), r.data_ptr(), n * 1500 // p1, p1, p2, 1,
                                    ncu * 2, sink.data_ptr(), vp(s.cuda_stream))
                    else:
                        ns, mode = (8, 0) if name == "xorder" else (p1, p2)
                        rc = L.rwxstage_run(b["frames"].data_ptr(), r.data_ptr(), stg.data_ptr(),
                                            cnt.data_ptr(), gen.data_ptr(), ntiles, 96000, 4096,
                                            ns, mode, ncu * 2, sink.data_ptr(), vp(s.cuda_stream))
                        assert rc == 0, rc
                    z.record()
                    torch.cuda.synchronize()
                    if rep:
                        t.setdefault((bi, ri, name), []).append(a.elapsed_time(z))
        print(json.dumps({"rep": rep}), file=sys.stderr, flush=True)
    out = {}
    for (bi, ri, name), v in sorted(t.items()):
        out.setdefault(f"{bi},{ri}", {})[name] = round(sorted(v)[len(v) // 2], 3)
    print(json.dumps({"pairs": out, "census_groups_share_xcc": groups_ok,
                      "census_first16": cen[:16]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--step-mb", type=float, default=16)
    ap.add_argument("--count", type=int, default=32)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--n", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--matrix", type=int, default=0,
                    help="instead: 2 frame batches x this many separate 1 GiB record buffers")
    ap.add_argument("--policies", action="store_true")
    ap.add_argument("--orders", action="store_true")
    ap.add_argument("--flags", action="store_true")
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--benchpath", action="store_true")
    ap.add_argument("--txplace", action="store_true")
    ap.add_argument("--txside", action="store_true")
    ap.add_argument("--bursts", action="store_true")
    ap.add_argument("--xstage", action="store_true")
    ap.add_argument("--batches", type=int, default=2)
    ap.add_argument("--spacer-gb", type=float, default=0.0,
                    help="matrix: allocate this many GB before every batch after the first "
                         "and before every record buffer")
    args = ap.parse_args()
    if args.bursts:
        return bursts(args)
    if args.xstage:
        return xstage(args)
    if args.matrix:
        return matrix(args)
    if args.policies:
        return policies(args)
    if args.orders:
        return orders(args)
    if args.flags:
        return flags(args)
    if args.keep:
        return keep(args)
    if args.benchpath:
        return benchpath(args)
    if args.txplace:
        return txplace(args)
    if args.txside:
        return txside(args)
    import torch
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = args.n
    ctx = RxContext(0, bytes(range(1, 17)))
    b = make_batch("c1500", n, dev)
    step = int(args.step_mb * (1 << 20)) // 64 * 64
    pool = torch.zeros(n * 64 + step * args.count + 64, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t = {}
    for rep in range(args.reps + 1):
        for k in range(args.count):
            r = pool[k * step: k * step + n * 64].view(n, 64)
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ctx.batch_device(b["frames"], n, stride=1500, fixed_len=1500, recs=r)
            z.record()
            torch.cuda.synchronize()
            if rep:
                t.setdefault(k, []).append(a.elapsed_time(z))
    med = [round(sorted(v)[len(v) // 2], 3) for _, v in sorted(t.items())]
    print(json.dumps({"step_bytes": step, "rx_ms": med, "frames": hex(b["frames"].data_ptr()),
                      "pool": hex(pool.data_ptr())}), flush=True)


if __name__ == "__main__":
    main()
