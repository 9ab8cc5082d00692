#!/usr/bin/env python3
"""bench.py -- device-resident throughput of the MI355X rx transform.

One "step" = one launch of the rx transform (checksum verify + header
parse + SipHash flow hash, pptk_rx_batch_device) over one batch of
synthetic frames already resident in HBM.  Primary workload: C1500
(16 M x 1500 B IPv4/TCP per GPU, BASELINE.json configs[2], on which the
70 %-of-HBM target is stated); C64 (configs[1]) and CMIX (configs[3]) are
reported in "secondary".  With N > 1 GPUs every rank processes its own
16 M-frame shard (weak scaling) and the per-frame flow hashes of each batch
are all-gathered over RCCL, overlapped with the next batch's kernel.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement".
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpkts/s device-resident (cksum+parse+SipHash), 64B & 1500B; % HBM roofline"
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md)
KEY = bytes(range(1, 17))
N_PER_GPU = 16 * 1024 * 1024
SETTLE_S = 1.5                  # seconds of untimed launches before warmup
# N > 1: CUs left to the all-gather beside the batches (pptk_rx_stream_split;
# the forced one-rank line splits only when PPTK_BENCH_COLL_CUS is set):
# RCCL's kernel needs whole CUs and the persistent grid fills them all, so
# without a split the gather runs between batches, not beside them (DESIGN
# section 8: +1.6-1.8 ms per batch with a 1.7 ms stand-in, +0.09 ms split)
COLL_CUS = int(os.environ.get("PPTK_BENCH_COLL_CUS", "32"))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


_ROCTX = []


def roctx_range(name):
    """A ROCTx range around a timed region when PPTK_BENCH_ROCTX=1, so that a
    `rocprofv3 --kernel-trace --marker-trace --kernel-rename --stats` run
    reports the timed launches under the range's name, apart from the
    placement probes, autotune trials and warm-up launches of the same
    kernel (profiles/ READMEs: the summary's average is then exactly the
    timed steps').  A no-op otherwise."""
    import contextlib
    if os.environ.get("PPTK_BENCH_ROCTX") != "1":
        return contextlib.nullcontext()
    if not _ROCTX:
        import ctypes
        L = None
        for nm in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"):
            try:
                L = ctypes.CDLL(nm)
                break
            except OSError:
                continue
        if L is not None:
            L.roctxRangePushA.argtypes = [ctypes.c_char_p]
            L.roctxRangePushA.restype = ctypes.c_int
            L.roctxRangePop.restype = ctypes.c_int
        _ROCTX.append(L)
    L = _ROCTX[0]
    if L is None:
        return contextlib.nullcontext()

    @contextlib.contextmanager
    def rng():
        L.roctxRangePushA(name.encode())
        try:
            yield
        finally:
            L.roctxRangePop()
    return rng()


def dist_on(ws):
    """A process group exists: N > 1, or PPTK_BENCH_FORCE_DIST=1 (a one-rank
    RCCL communicator, to exercise the all-gather path on a one-GPU box)."""
    return ws > 1 or os.environ.get("PPTK_BENCH_FORCE_DIST") == "1"


def launch_ranks(argv, ngpus):
    """`python bench.py --gpus N` (N > 1) outside a launcher: start N rank
    processes through torch.distributed.run (127.0.0.1 rendezvous) before
    anything here touches a GPU, and exit with their status.  Under a
    launcher (LOCAL_RANK set) this is a no-op."""
    if ngpus <= 1 or "LOCAL_RANK" in os.environ:
        return
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ngpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + argv
    log(f"launching {ngpus} ranks: {' '.join(cmd[1:])}")
    raise SystemExit(subprocess.call(cmd))


def join_all(ctx, ws, rank, join_fn=None):
    """Join `ctx` to the job's RCCL communicator on every rank or on none.  A
    rank whose creation fails (no RCCL, a peer that never joins: -ETIMEDOUT
    after opts.comm_timeout_ms) tells the others over the gloo group; every
    rank that did join then aborts and drops its communicator, and the run
    goes on without the collective: the line carries allgather.error (and
    fails validate_line, so the process still exits non-zero) beside the
    sharded rates every rank measured.  Returns None or the error."""
    if join_fn is None:
        from pptk_amd.shard import join as join_fn
    err = None
    try:
        join_fn(ctx, ws, rank)
    except Exception as e:   # (RuntimeError from the C-ABI's -errno, or a missing librccl)
        err = f"[rank {rank}] {type(e).__name__}: {e}"[:300]
    if ws > 1:
        import torch
        import torch.distributed as dist
        failed = torch.tensor([0 if err is None else 1], dtype=torch.int32)
        dist.all_reduce(failed)
        if int(failed.item()) and err is None:
            err = f"{int(failed.item())} of {ws} ranks could not join the RCCL communicator"
            for drop in (ctx.comm_abort, ctx.comm_destroy):
                try:
                    drop()
                except Exception:   # (already gone: nothing to drop)
                    pass
    return err


def dist_setup(ngpus):
    """One process per GPU.  The host control plane (barriers, max over
    ranks, the communicator uid) is a gloo group; the data-path collective
    is RCCL inside libpptkrx.so (pptk_rx_allgather_hash)."""
    import torch
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != ngpus and "LOCAL_RANK" in os.environ:
        log(f"[rank {rank}] --gpus {ngpus} but WORLD_SIZE {ws}: using {ws}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist_on(ws):
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(ws))
        dist.init_process_group("gloo")
    return ws, rank, dev


# (ctx, stream) pairs that carry all-gathers: barrier() waits for them with
# pptk_rx_comm_sync (bounded, RCCL errors surfaced) before the device-wide
# synchronize, so a rank whose peer died exits with an error instead of
# hanging in hipDeviceSynchronize (include/pptk_rx.h "Failure containment")
GATHER_STREAMS = []
COMM_SYNC_TIMEOUT_MS = 120000


def barrier(ws, dev):
    import torch
    for ctx, s in GATHER_STREAMS:
        rc = ctx.comm_sync(s, COMM_SYNC_TIMEOUT_MS)
        if rc != 0:
            raise RuntimeError(f"all-gather stream failed: pptk_rx_comm_sync {rc} "
                               "(-110 timeout: a peer stopped; -5 RCCL error; -125 aborted)")
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    if dist_on(ws):
        import torch.distributed as dist
        dist.barrier()


def _reduce(x, ws, op):
    if not dist_on(ws):
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)      # gloo: host tensors
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(x, ws, dev=None):
    import torch.distributed as dist
    return _reduce(x, ws, dist.ReduceOp.MAX)


def sum_over_ranks(x, ws, dev=None):
    import torch.distributed as dist
    return _reduce(x, ws, dist.ReduceOp.SUM)


def per_rank(x, ws):
    """Every rank's value of x (gloo all_gather_object), rank order."""
    if not dist_on(ws):
        return [x]
    import torch.distributed as dist
    out = [None] * ws
    dist.all_gather_object(out, x)
    return out


def gather_bw(per, ws, seconds):
    """All-gather bandwidths (RCCL convention): algorithmic = bytes received
    per rank / time, bus = algorithmic * (ws - 1) / ws."""
    alg = per * ws * 8 / seconds / 1e9
    return round(alg, 1), round(alg * (ws - 1) / ws, 1)


PLACE_FRAMES = 4          # frame-buffer candidates (a fresh synthetic batch)
PLACE_RECORDS = 8         # record-buffer candidates
# Freed device memory is scrubbed by the driver in the background (SOCCLK
# at 1.2 GHz while it runs, `tools/clock_probe.py --free-gb`): ~1 s after
# freeing 16 GB, ~2 s after 64 GB, ~4 s after 128 GB, and the rx launches
# beside it run up to 9 % slower.  The settle after a placement probe lasts
# until the scrub of what the probe freed is over, at this (conservative)
# rate.
SCRUB_BYTES_PER_S = 20e9


_SCRUB_UNTIL = [0.0]   # when the scrub of everything freed so far should be over


def note_freed(nbytes, at):
    _SCRUB_UNTIL[0] = max(_SCRUB_UNTIL[0], at + nbytes / SCRUB_BYTES_PER_S)


def wait_scrub(cap_s=20.0):
    """Sleep until the driver's scrub of what this process freed is over
    (at SCRUB_BYTES_PER_S, at most cap_s); returns the seconds slept."""
    left = min(cap_s, _SCRUB_UNTIL[0] - time.perf_counter())
    if left > 0:
        time.sleep(left)
    return round(max(0.0, left), 2)


def release(dev):
    """Return the caching allocator's free blocks to the driver; returns
    (bytes released, when), the input of the scrub wait."""
    import torch
    torch.cuda.synchronize(dev)
    before = torch.cuda.memory_reserved(dev)
    torch.cuda.empty_cache()
    freed, at = max(0, before - torch.cuda.memory_reserved(dev)), time.perf_counter()
    note_freed(freed, at)
    return freed, at


def _spaced(dev, count, nbytes, spacer, hold):
    """count buffers of nbytes, each allocated after a spacer of `spacer`
    bytes (kept in `hold`) so that they land apart in HBM."""
    import torch
    out = []
    for _ in range(count):
        if spacer:
            hold.append(torch.empty(spacer, dtype=torch.uint8, device=dev))
        out.append(torch.empty(nbytes, dtype=torch.uint8, device=dev))
    return out


def placed_buffers(ctx, b, n, dev, compact, kw, frames=True, nf=PLACE_FRAMES,
                   nr=PLACE_RECORDS, autotune=True):
    """Place the batch's buffers (pptk_rx_place_buffers): what the memory
    charges for the record writes beside the frame reads depends on where
    the frame buffer and the record buffer sit physically (the same launch:
    4.15-4.3 ms or 4.5-5.1 ms).  Frame candidates (with
    frames=True: the batch as generated plus nf - 1 copies, each allocated
    behind a spacer so that they land apart) times record candidates (nr,
    behind spacers too); the batch timed on every pair, the fastest pair
    kept -- b["frames"] is replaced by the chosen copy.  Untimed, once per
    batch, as a long-lived rx ring would be set up.  Returns (recs, report)."""
    import torch
    rb = 32 if compact else 64
    fbytes = b["frames"].numel()
    spacer_r = min(4 << 30, max(256 << 20, 4 * n * rb))
    spacer_f = min(8 << 30, max(1 << 30, fbytes // 2))
    free, _ = torch.cuda.mem_get_info(dev)
    if not frames:
        nf = 1
    while nf > 1 and (nf - 1) * (fbytes + spacer_f) + nr * (n * rb + spacer_r) > 0.6 * free:
        nf -= 1
    while nr > 1 and (nf - 1) * (fbytes + spacer_f) + nr * (n * rb + spacer_r) > 0.6 * free:
        nr -= 1
    hold = []
    fc = [b["frames"]]
    for t in _spaced(dev, nf - 1, fbytes, spacer_f, hold):
        t.copy_(b["frames"])
        fc.append(t)
    rc = [t.view(n, rb) for t in _spaced(dev, nr, n * rb, spacer_r, hold)]
    if autotune:
        # the probe times the shape later batches will run (pptk_rx_autotune
        # on the as-allocated pair; run_config tunes again on the chosen one)
        ctx.autotune(fc[0], n, recs=rc[0], compact=compact, reps=9, **kw)
    fi, ri, ms = ctx.place_buffers(fc, n, rc, compact=compact, **kw)
    b["frames"] = fc[fi]
    recs = rc[ri]
    report = {"frame_candidates": nf, "record_candidates": nr, "chosen": [fi, ri],
              "chosen_ms": ms[fi * nr + ri], "as_allocated_ms": ms[0],
              "pair_ms": [ms[k * nr:(k + 1) * nr] for k in range(nf)]}
    del fc, rc, hold
    report["freed_bytes"], report["_freed_at"] = release(dev)
    return recs, report


def ring_buffers(ctx, b, n, dev, compact, probe_hash=False):
    """The product's default device rings (pptk_rx_ring_alloc): the library
    allocates frame and record candidates spread apart in HBM, probes every
    pair with a synthetic batch of the ring's geometry and keeps the fastest
    (DESIGN.md section 7 "Placement"); the batch is then written into the
    frame ring, as an rx queue fills its ring.  b["frames"] is replaced by
    the ring's frame buffer.  Returns (recs, report)."""
    fbytes = b["frames"].numel() - 64
    probe = b.get("fixed_len") or 1500
    ring = ctx.ring_alloc(fbytes, n, 32 if compact else 64, probe_len=min(1536, max(64, probe)),
                          probe_hash=probe_hash)
    ring.frames.copy_(b["frames"])
    b["frames"] = ring.frames
    report = dict(ring.report)
    report["alloc"] = "pptk_rx_ring_alloc"
    report["plain_alloc_ms"] = report.pop("first_ms")
    # the probe is the batch's own launch only for fixed-stride batches of
    # the probe's frame length (C1500, C64); for offset-described mixes it is
    # a C1500-stride probe over the same bytes (placement, not a CMIX time)
    report["probe_is_batch"] = "off" not in b and report["probe_frames"] == n
    freed, at = release(dev)          # the batch as generated, now copied into the ring
    report["freed_bytes"] += freed
    report["_freed_at"] = at
    note_freed(report["freed_bytes"], at)
    return ring.recs, report


def placed_gather(ctx, b, recs, kw, n_total, ws, rank, dev):
    """The two gather buffers, placed by the library (pptk_rx_gather_alloc,
    include/pptk_rx.h): the all-gather lands (ws - 1) shards of hashes in
    this GPU's HBM while the next batch streams its frames, and the kernel
    writes its own hashes into its slice; what those writes cost depends on
    where the buffer sits, as for the records.  The
    library probes candidate regions with this batch and a device copy of
    the bytes the gather would land beside each launch, and keeps the
    fastest -- the same call a C application makes (examples/rx_multigpu.c).
    Rank-local (no collective).  Returns ([GatherBuffer, GatherBuffer],
    report)."""
    from pptk_amd.shard import GatherBuffer, shard_range
    first, count, per = shard_range(n_total, ws, rank)
    g = ctx.gather_alloc(b["frames"], count, per, ws, rank, recs=recs, **kw)
    gbs = [GatherBuffer(n_total, ws, rank, dev, out=g.out[k]) for k in range(2)]
    rep = dict(g.report)
    rep["_freed_at"] = time.perf_counter()
    note_freed(rep.get("freed_bytes", 0), rep["_freed_at"])
    return gbs, rep


def run_config(cfg, n, ctx, dev, ws, rank, steps, warmup, gbs, check, settle=SETTLE_S,
               compact=False, batch=None, autotune=True, first=None, place=True, recs=None,
               n_gather_total=None, coll_stream=None):
    """Generate this rank's shard of config `cfg` (n frames from global frame
    `first`, default rank * n) or reuse `batch`, time `steps` launches.
    gbs: two shard.GatherBuffer (double-buffered all-gather of the flow
    hashes after every launch, on a second stream: `coll_stream`, or a new
    one) or None.  compact: 32-byte records (struct pptk_rx_rec32)."""
    import torch
    from harness.synth import make_batch
    first = rank * n if first is None else first
    b = batch if batch is not None else make_batch(cfg, n, dev, first=first)
    torch.cuda.synchronize(dev)
    if "off" in b:
        # mixed sizes: per-frame offset/length arrays, frames in batch order
        # (the binned order is measured separately: DESIGN.md)
        kw = dict(off=b["off"], lens=b["lens"], max_len=b["max_len"])
    else:
        kw = dict(stride=b["stride"], fixed_len=b["fixed_len"])
    placement = None
    if recs is not None:
        pass                      # the caller's (already placed) record buffer
    elif place:
        # where the frame and record buffers sit changes what the memory
        # charges for the record writes by up to 25 %:
        # pick a well-placed pair, untimed, as a long-lived rx ring would be
        # set up once (a reused batch keeps its frames: records only)
        if batch is None:
            # (with a gather the batches also write the dense hashes: the
            # ring probe writes them too, PPTK_RX_RING_PROBE_HASH)
            recs, placement = ring_buffers(ctx, b, n, dev, compact, probe_hash=bool(gbs))
        else:
            recs, placement = placed_buffers(ctx, b, n, dev, compact, kw, frames=False,
                                             autotune=autotune)
    else:
        recs = torch.empty((n, 32 if compact else 64), dtype=torch.uint8, device=dev)
    gplace = None
    if isinstance(gbs, str):          # "place": the gather buffers, placed
        # (after the scrub of what the ring placement freed: beside it every
        # candidate runs slow alike and the probe cannot tell them apart)
        if placement and "_freed_at" in placement:
            wait = placement["_freed_at"] + placement["freed_bytes"] / SCRUB_BYTES_PER_S \
                - time.perf_counter()
            if wait > 0:
                time.sleep(wait)
        gbs, gplace = placed_gather(ctx, b, recs, kw, n_gather_total, ws, rank, dev)
    if autotune:
        # pick this GPU's fastest interchangeable kernel shape for the batch
        # (pptk_rx_autotune: results identical, untimed, before the settle)
        ctx.autotune(b["frames"], n, recs=recs, compact=compact, reps=9, **kw)

    main = torch.cuda.current_stream(dev)
    gs = (coll_stream or torch.cuda.Stream(dev)) if gbs else None
    del GATHER_STREAMS[:]
    if gbs:
        GATHER_STREAMS.extend([(ctx, main), (ctx, gs)])
    kdone = [torch.cuda.Event() for _ in range(2)]
    gdone = [torch.cuda.Event() for _ in range(2)]

    def step(k, collective=True):
        # the dense flow-hash array only feeds the all-gather (N > 1); at
        # N = 1 the records (which carry flow_hash) are the whole output.
        # The kernel writes this rank's hashes into its slice of gather
        # buffer k % 2 (after the gather of step k - 2 has read it), then
        # the in-place all-gather runs on the second stream, overlapping
        # the next launch.
        gb = gbs[k & 1] if gbs else None
        if gb is not None:
            main.wait_event(gdone[k & 1])
        ctx.batch_device(b["frames"], n, recs=recs, compact=compact,
                         hash_out=None if gb is None else gb.local[:n], **kw)
        if gb is not None and collective:
            kdone[k & 1].record(main)
            gs.wait_event(kdone[k & 1])
            gb.gather(ctx, stream=gs)
            gdone[k & 1].record(gs)

    # settle: clocks ramp up over the first few hundred ms of sustained
    # load (the kernel trace shows the first launches 4-5 % slower, and a
    # cold first process up to 20 %); run until `settle` seconds have passed
    # before the W warmup steps, so the K timed steps see steady state.  The
    # settle launches issue no collective: their number depends on each
    # rank's clock, and ranks must issue the same sequence of all-gathers.
    # After a placement probe the settle also outlasts the driver's scrub of
    # the candidates it freed (SCRUB_BYTES_PER_S).
    t_settle = time.perf_counter()
    settle_end = t_settle + settle
    for rep in (placement, gplace):
        if rep and "_freed_at" in rep:
            scrub_end = rep.pop("_freed_at") + rep["freed_bytes"] / SCRUB_BYTES_PER_S
            settle_end = max(settle_end, scrub_end)
            rep["scrub_wait_s"] = round(max(0.0, scrub_end - t_settle), 2)
    k = 0
    while time.perf_counter() < settle_end:
        step(k, collective=False)
        k += 1
        if k % 16 == 0:
            torch.cuda.synchronize(dev)
    if gbs:
        # one untimed collective whatever the warmup count, so that RCCL's
        # lazy channel setup never lands in the timed steps
        gbs[0].gather(ctx, stream=main)
    for k in range(warmup):
        step(k)
    barrier(ws, dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    t0 = time.perf_counter()
    with roctx_range(f"timed_{cfg}{'_rec32' if compact else ''}"):
        for k in range(steps):
            ev[k][0].record(main)
            step(k)
            ev[k][1].record(main)
        barrier(ws, dev)
    wall = time.perf_counter() - t0
    wall = max_over_ranks(wall, ws, dev)
    # kernel-only duration: the rx launch is the only work between the
    # events when there is no gather; with a gather the event pair also
    # spans the wait for the gather of step k - 2
    kms = [a.elapsed_time(z) for a, z in ev]
    kernel_ms = float(np.median(kms))
    from pptk_amd.rx import VARIANTS
    variant = VARIANTS[ctx._L.pptk_rx_last_variant(ctx._ctx)]
    n_all = gbs[0].n_total if gbs else n * ws
    res = {
        "n": n, "bytes": b["bytes"], "rec_bytes": n * (32 if compact else 64), "wall_s": wall,
        "ms_per_step": wall / steps * 1e3, "kernel_ms": kernel_ms,
        "mpkts": n_all * steps / wall / 1e6, "variant": variant, "placement": placement,
        "gather_placement": gplace, "_gbs": gbs,
    }
    # size-independent parity on the full batch: every frame parsed, and the
    # checksum verdicts equal what the generator planted
    if check:
        from pptk_amd.records import F_IP_OK, F_L4_OK, F_PARSED
        fcol = 10 if compact else 27                                  # flags @20 / @54
        r = recs.view(torch.int16)[:, fcol].to(torch.int32) & 0xFFFF
        exp = b["expect"].to(torch.int32)
        ok_parsed = bool(((r & F_PARSED) != 0).all().item())
        ip_ok = ((r & F_IP_OK) != 0).to(torch.int32)
        l4_ok = ((r & F_L4_OK) != 0).to(torch.int32)
        ok_ip = bool((ip_ok == (exp & 1)).all().item())
        ok_l4 = bool((l4_ok == ((exp >> 1) & 1)).all().item())
        res["full_batch_check"] = {"parsed": ok_parsed, "ip_verdicts": ok_ip,
                                   "l4_verdicts": ok_l4,
                                   "corrupted": int((exp != 3).sum().item())}
        res["oracle_sample"] = oracle_sample(b, recs, n, dev, compact=compact)
    res["_batch"] = b
    res["_recs"] = recs
    return res


GATHER_CHECK_FRAMES = 4096    # per rank: regenerated and run through the CPU oracle


def gathered_check(prim, gbs, n, dev, k=GATHER_CHECK_FRAMES):
    """The all-gathered flow hashes: this rank's slice equals the flow_hash
    column of its own records (every frame), and the first k frames of
    every rank's shard, regenerated here from the same synthetic recipe and
    run through the CPU oracle, equal their gathered slots."""
    import torch
    from oracle.oracle import Oracle, make_opts
    from harness.synth import make_batch
    gb = gbs[0]
    got = gb.out.cpu().numpy().view(np.uint64)
    own = prim["_recs"].view(torch.int64)[:, 0] if prim["_recs"].shape[1] == 64 else None
    ok_own = own is not None and bool(torch.equal(own, gb.local[:n]))
    bad = 0
    cfg = prim["_batch"]["cfg"]
    for r in range(gb.world):
        lo = r * gb.per
        cnt = min(k, max(0, gb.n_total - lo))
        if cnt == 0:
            continue
        b = make_batch(cfg, cnt, dev, first=lo)
        host = b["frames"][: cnt * b["stride"]].cpu().numpy()
        want = Oracle().rx_batch(host, None, None, stride=b["stride"], fixed_len=b["fixed_len"],
                                 n=cnt, opts=make_opts(KEY))
        bad += int((want["flow_hash"] != got[lo:lo + cnt]).sum())
    sampled = sum(min(k, max(0, gb.n_total - r * gb.per)) for r in range(gb.world))
    return {"own_slice_equals_records": ok_own, "sampled_frames": sampled,
            "sampled_frames_per_rank": k, "sampled_mismatches": bad}


def validate_line(line):
    """The checks the multi-GPU line must pass before it is printed (the
    driver's 8-GPU run is not rehearsable here): the communicator spans every
    rank, the all-gather was measured, its gathered array was checked on at
    least GATHER_CHECK_FRAMES frames of every rank's shard with no mismatch,
    and every rank reported its kernel time.  Returns the list of problems
    (empty: the line is good); a one-GPU line without a gather passes."""
    bad = []
    ws = line.get("n_gpus")
    gat = line.get("allgather")
    if not isinstance(ws, int) or ws < 1:
        return ["n_gpus missing"]
    if ws > 1 and not gat:
        bad.append("N > 1 without an all-gather")
    if gat and gat.get("error"):
        bad.append(f"all-gather failed: {gat['error']}")
    elif gat:
        if line.get("config", {}).get("rccl_ranks") != ws:
            bad.append(f"config.rccl_ranks {line.get('config', {}).get('rccl_ranks')} != n_gpus {ws}")
        if gat.get("rccl_ranks") != ws:
            bad.append(f"allgather.rccl_ranks {gat.get('rccl_ranks')} != n_gpus {ws}")
        for key in ("ms", "algbw_gbs", "busbw_gbs", "overlap_loss"):
            if not isinstance(gat.get(key), (int, float)):
                bad.append(f"allgather.{key} missing")
        chk = gat.get("gathered_check")
        if not chk:
            bad.append("allgather.gathered_check missing")
        else:
            if chk.get("sampled_frames_per_rank", 0) < GATHER_CHECK_FRAMES:
                bad.append("gathered check samples fewer than "
                           f"{GATHER_CHECK_FRAMES} frames per rank")
            if chk.get("sampled_mismatches") != 0:
                bad.append(f"gathered check: {chk.get('sampled_mismatches')} mismatches")
            if chk.get("own_slice_equals_records") is not True:
                bad.append("own slice != records")
        if not isinstance(line.get("value_no_gather"), (int, float)):
            bad.append("value_no_gather missing")
    prk = line.get("per_rank_kernel_ms")
    if not isinstance(prk, list) or len(prk) != ws:
        bad.append("per_rank_kernel_ms does not list every rank")
    return bad


LINE_MAX_CHARS = 4000     # the stdout line must fit the driver's stored tail whole


def _cfg_entry(sec):
    """One config's entry of the compact line."""
    if not sec:
        return None
    r = sec.get("roofline") or {}
    e = {"mpkts": sec.get("value"), "kernel_ms": sec.get("kernel_ms"), "frac": r.get("frac"),
         "variant": sec.get("kernel_variant")}
    if r.get("traffic"):
        e["traffic"] = r["traffic"]
    if r.get("mix_sol_frac"):
        e["sol_frac"] = r["mix_sol_frac"]
    o = sec.get("oracle_sample")
    if o:
        e["oracle_mismatches"] = o.get("mismatches")
    fb = sec.get("full_batch_check")
    if fb:
        e["verdicts_ok"] = bool(fb.get("parsed") and fb.get("ip_verdicts") and fb.get("l4_verdicts"))
    return e


def compact_line(full, detail_path=None):
    """The printed JSON line: the contract keys, the primary roofline and
    CPU baseline, and one compact entry per BASELINE config (C1500, C64,
    CMIX with M6 beside it, IMIX, JMIX; compact-record runs), the end-to-end
    rates, the batch ops and, with N > 1, the all-gather -- every number the
    driver should keep, under LINE_MAX_CHARS so the stored stdout tail holds
    it whole.  Everything else (placement reports, box probes, workloads) is
    in the full result at `detail_path` and on stderr."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data")
    line = {k: full.get(k) for k in keep}
    c = full.get("config") or {}
    line["config"] = {k: c.get(k) for k in ("workload", "frames_per_gpu", "global_frames",
                                             "parallelism", "rccl_ranks")}
    r = full.get("roofline") or {}
    line["roofline"] = {k: r.get(k) for k in (
        "bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms", "kernel_variant",
        "algorithmic_bytes_per_launch", "frac_plain_alloc", "mix_sol_frac") if k in r}
    src = r.get("traffic_source") or ""
    line["roofline"]["traffic_source"] = "live rocprofv3 PMC" if src.startswith("live") else src
    cpu = full.get("cpu_baseline")
    line["cpu_baseline"] = None           # (rank 0 of a one-GPU run only)
    if cpu:
        line["cpu_baseline"] = {k: cpu.get(k) for k in ("value", "unit", "cores", "kind",
                                                        "single_thread_mpkts", "cpu_model")}
        line["cpu_baseline"]["sample"] = "1 M distinct C1500 frames, full path (reference functions)"
    cfgs = {}
    cfgs[(c.get("workload") or "c1500").split(":")[0].lower()] = _cfg_entry(
        {"value": full.get("value"), "kernel_ms": r.get("kernel_ms"),
         "kernel_variant": r.get("kernel_variant"), "roofline": r,
         "oracle_sample": (full.get("parity") or {}).get("oracle_sample"),
         "full_batch_check": (full.get("parity") or {}).get("full_batch")})
    if full.get("rec32"):
        cfgs["c1500_rec32"] = _cfg_entry(full["rec32"])
    for name, sec in (full.get("secondary") or {}).items():
        cfgs[name] = _cfg_entry(sec)
        if sec.get("rec32"):
            cfgs[name + "_rec32"] = _cfg_entry(sec["rec32"])
        if sec.get("m6"):
            cfgs[name]["m6_ms"] = sec["m6"]["kernel_ms"]
            cfgs[name]["m6_frac"] = sec["m6"]["frac"]
        if sec.get("binned"):
            cfgs[name]["mixed_call_ms"] = sec["binned"].get("ms_per_batch")
            cfgs[name]["binned"] = sec["binned"].get("binned_by_plan")
    line["configs"] = cfgs
    e2e = full.get("e2e")
    if e2e:
        line["e2e"] = ({k: ({kk: v.get(kk) for kk in ("mpkts", "path", "frame_gbs", "of_pcie")}
                            if isinstance(v, dict) else v)
                        for k, v in e2e.items() if k not in ("gather_threads", "numa", "scrub_wait_s")})
    ops = {}
    pm = full.get("permit") or {}
    for key, sub in (("permit_records_ms", pm), ("permit_keys_ms", pm.get("keys")),
                     ("permit_keys_denying_ms", pm.get("keys_denying"))):
        if sub and sub.get("ms_per_batch") is not None:
            ops[key] = sub["ms_per_batch"]
    for key, sub in (("tx_ms", full.get("tx")), ("rewrite_ms", full.get("rewrite")),
                     ("mss_clamp_ms", full.get("mss_clamp"))):
        if sub:
            ops[key] = sub.get("kernel_ms")
    if ops:
        line["ops"] = ops
    gat = full.get("allgather")
    if gat and gat.get("error"):
        line["allgather"] = {"error": gat["error"]}
    elif gat:
        g = {k: gat.get(k) for k in ("ms", "algbw_gbs", "busbw_gbs", "overlap_loss", "rccl_ranks",
                                      "bytes_per_rank", "coll_cus", "split",
                                      "max_ctas")}
        chk = gat.get("gathered_check") or {}
        g["gathered_check"] = {k: chk.get(k) for k in ("own_slice_equals_records",
                                                        "sampled_frames_per_rank",
                                                        "sampled_mismatches")}
        bp = gat.get("buffer_placement") or {}
        g["placement"] = {k: bp.get(k) for k in ("alloc", "candidates", "chosen", "chosen_ms", "candidate_ms",
                                                  "first_ms")}
        line["allgather"] = g
        line["value_no_gather"] = full.get("value_no_gather")
    line["per_rank_kernel_ms"] = full.get("per_rank_kernel_ms")
    if detail_path:
        line["detail"] = detail_path
    return line


def mix_sol(b, recs, n):
    """(ms, description) of the speed of light of an rx launch's traffic mix
    on this GPU (tools/rwmix.py sol_ms): the fastest of several trivial
    kernels reading the launch's frame bytes in its 64-frame tiles -- the
    fixed-stride tile, or for offset-described batches (CMIX: frames packed
    in batch order) each tile's actual span after its 10-byte descriptors --
    and writing the tile's records, nothing computed; None if the shapes do
    not fit.  A real ceiling only if the rx kernel never beats it
    (roofline.mix_sol_frac <= 1)."""
    from harness.rwmix import sol_ms
    ntiles = n // 64
    if ntiles == 0:
        return None
    wb = 64 * (recs.shape[1] if recs.dim() == 2 else 64)
    if "off" in b:
        ms, how = sol_ms(b["frames"], n, recs, wb, off=b["off"], lens=b["lens"])
        return round(ms, 4), (f"{ntiles} tiles, each its frames' span read after its "
                              f"descriptors + {wb} B written, {how}")
    rb = 64 * b["stride"]
    if rb % 16:
        return None
    ms, how = sol_ms(b["frames"], n, recs, wb, rb=rb)
    return round(ms, 4), f"{ntiles} tiles x {rb} B read + {wb} B written, {how}"


def binned_bench(ctx, b, n, dev, steps, warmup, recs=None):
    """The mixed-size call BASELINE.json's configs[3] names ("lanes binned
    by length"): pptk_rx_batch_device_mixed, timed per batch, whole call
    (into `recs`, the batch-order run's placed record buffer, when given),
    without d_perm (the processing order is not needed here; an untimed call
    with d_perm reports whether this batch was binned)."""
    import torch
    if recs is None:
        recs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    scratch = torch.empty(ctx._L.pptk_rx_bin_scratch_bytes(n), dtype=torch.uint8, device=dev)
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.batch_device_mixed(b["frames"], n, b["off"], b["lens"], max_len=b["max_len"], recs=recs,
                           perm=perm, scratch=scratch)
    p = perm[:min(n, 1 << 20)].cpu()
    binned = bool((p != torch.arange(p.numel(), dtype=p.dtype)).any().item())
    del perm
    kw = dict(max_len=b["max_len"], recs=recs, scratch=scratch)
    for _ in range(max(warmup, 3)):
        ctx.batch_device_mixed(b["frames"], n, b["off"], b["lens"], **kw)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for a, z in ev:
        a.record()
        ctx.batch_device_mixed(b["frames"], n, b["off"], b["lens"], **kw)
        z.record()
    torch.cuda.synchronize(dev)
    ms = float(np.median([a.elapsed_time(z) for a, z in ev]))
    ach = b["bytes"] / (ms * 1e-3) / 1e9
    return {"value": round(n / ms / 1e3, 1), "unit": "Mpkts/s", "ms_per_batch": round(ms, 4),
            "workload": f"{b['cfg'].upper()}, pptk_rx_batch_device_mixed (max_len hint "
                        f"{b['max_len']}): binned into length groups only when jumbo frames "
                        "(> 1521 B) mix with shorter ones, else batch order; records at the "
                        "frames' own indices",
            "binned_by_plan": binned,
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4)}}


def summary(r, n):
    """Per-config result: rate, kernel time, read roofline fraction (SURVEY
    8(d): frame bytes / kernel time / peak) and read+write fraction (frame
    bytes + record bytes), parity checks."""
    ks = r["kernel_ms"] * 1e-3
    ach = r["bytes"] / ks / 1e9
    rw = (r["bytes"] + r["rec_bytes"]) / ks / 1e9
    out = {"value": round(r["mpkts"], 1), "unit": "Mpkts/s",
            "kernel_ms": round(r["kernel_ms"], 4), "kernel_variant": r.get("variant"),
            "frames_per_gpu": n, "frame_bytes": r["bytes"], "record_bytes": r["rec_bytes"],
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                         "rw_achieved": round(rw, 1), "rw_frac": round(rw / HBM_PEAK_GBS, 4)},
            "full_batch_check": r.get("full_batch_check"),
            "oracle_sample": r.get("oracle_sample"),
            "record_placement": r.get("placement")}
    out["roofline"].update(as_allocated(r))
    return out


def as_allocated(r):
    """What a caller gets from the default allocation.  With the product's
    device rings (pptk_rx_ring_alloc, the default here) that is the timed
    run itself: "frac_as_allocated" = frac, and "frac_plain_alloc" is the
    same launch on a plain hipMalloc pair (the ring probe's candidate pair
    0: what a caller that allocates its own buffers and does not place them
    gets on this GPU).  With caller-placed buffers (records-only placement
    of a reused batch) "frac_as_allocated" is the probe's pair 0, as before."""
    p = r.get("placement") or {}
    frac = lambda ms: round(r["bytes"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if p.get("alloc") == "pptk_rx_ring_alloc":
        out = {"as_allocated": "pptk_rx_ring_alloc", "frac_as_allocated": frac(r["kernel_ms"]),
               "as_allocated_ms": round(r["kernel_ms"], 4)}
        if p.get("plain_alloc_ms") and p.get("probe_is_batch"):
            out["frac_plain_alloc"] = frac(p["plain_alloc_ms"])
            out["plain_alloc_ms"] = p["plain_alloc_ms"]
        return out
    ms = p.get("as_allocated_ms")
    if not ms:
        return {}
    return {"frac_as_allocated": frac(ms), "as_allocated_ms": ms}


def oracle_sample(b, recs, n, dev, k=4096, compact=False):
    """Bit-exact check of k random frames against the CPU oracle."""
    import torch
    from oracle.oracle import Oracle, make_opts
    from pptk_amd.records import REC32_DTYPE, REC_DTYPE, diff_records, to_rec32
    rng = np.random.default_rng(1234)
    idx = np.sort(rng.choice(n, size=min(k, n), replace=False))
    if "off" in b:
        off = b["off"].cpu().numpy()[idx].astype(np.uint64)
        lens = (b["lens"].cpu().numpy().view(np.uint16))[idx]
    else:
        off = idx.astype(np.uint64) * b["stride"]
        lens = np.full(len(idx), b["fixed_len"], dtype=np.uint16)
    frames = b["frames"]
    chunks, offs, pos = [], [], 0
    for o, l in zip(off, lens):
        chunks.append(frames[int(o):int(o) + int(l)].cpu().numpy())
        offs.append(pos)
        pos += int(l)
    buf = np.concatenate(chunks + [np.zeros(64, np.uint8)])
    want = Oracle().rx_batch(buf, np.array(offs, np.uint64), lens,
                             opts=make_opts(KEY), nthreads=8)
    got = recs[torch.from_numpy(idx).to(dev)].cpu().numpy()
    if compact:
        want = to_rec32(want)
    d = diff_records(got, want, dtype=REC32_DTYPE if compact else REC_DTYPE)
    return {"frames": int(len(idx)), "mismatches": 0 if not d else int(d.split()[0])}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_lib():
    from oracle.oracle import REF_SO, Oracle, Reference
    kind = "reference" if os.path.exists(REF_SO) else "port"
    lib = Reference() if kind == "reference" else Oracle()
    kw = {"with_bucket": False} if kind == "reference" else {}
    return kind, lib, kw


def _cpu_topology():
    """(threads to use, description): the physical cores this process may
    run on (its CPU affinity, one hardware thread per core, from the sysfs
    core ids), capped by its cgroup CPU quota (cpu.max) -- on the GPU box
    the job's share of the host, not the whole machine."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    cores = set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id") as f:
                core = f.read().strip()
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id") as f:
                pkg = f.read().strip()
            cores.add((pkg, core))
        except OSError:
            cores.add(("?", c))
    phys = max(1, len(cores))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    n = min(phys, quota) if quota else phys
    env = int(os.environ.get("PPTK_CPU_THREADS", "0") or 0)
    if env > 0:
        n = env
    desc = (f"{len(cpus)} CPUs in affinity = {phys} physical cores"
            + (f", cgroup quota {quota} CPUs" if quota else "") + f" -> {n} threads")
    return n, desc


def _cpu_rate(b, n, nth, seconds):
    """Mpkts/s of the CPU full path over the first n frames of batch b."""
    from oracle.oracle import make_opts
    kind, lib, kw = _cpu_lib()
    host = b["frames"][: n * b["stride"]].cpu().numpy()
    opts = make_opts(KEY)
    done, t0 = 0, time.perf_counter()
    while True:
        lib.rx_batch(host, None, None, stride=b["stride"], fixed_len=b["fixed_len"],
                     n=n, opts=opts, nthreads=nth, **kw)
        done += n
        el = time.perf_counter() - t0
        if el >= seconds:
            return done / el / 1e6, el


def cpu_baseline(b, seconds=10.0, sample=1 << 20):
    """PPTK's CPU path on this host's cores (BASELINE.json
    configs[0]) over 1,048,576 distinct C1500 frames (1500 B IPv4/TCP) of
    the same batch: the reference's own functions (oracle/_ref, built from
    /root/reference by oracle/Makefile and shipped to the box as a binary;
    kind "reference"), else the C restatement ("port").  Full path on every
    physical core the job may use (the value) and on one thread, plus
    ipcksumperf semantics (iphdr/ipcksumperf.c:21-29: ip_cksum_feed over
    one 1500 B buffer, one thread, Gbit/s)."""
    kind, lib, _ = _cpu_lib()
    n = min(sample, b["n"])
    threads, topo = _cpu_topology()
    mt, el_mt = _cpu_rate(b, n, threads, seconds)
    st, _ = _cpu_rate(b, n, 1, seconds / 2) if seconds >= 1 else (None, 0)
    one = b["frames"][: b["stride"]].cpu().numpy()
    iters, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < min(2.0, seconds / 4):
        lib.cksum_loop(one, 200000)
        iters += 200000
    gbps = iters * one.size * 8 / (time.perf_counter() - t0) / 1e9
    return {"value": round(mt, 3), "unit": "Mpkts/s", "cores": threads, "kind": kind,
            "sample": f"{n} distinct C1500 frames (1500 B IPv4/TCP) from the same batch, "
                      f"full path (IPv4 hdr cksum + TCP cksum + parse + 40 B SipHash), "
                      f"repeated for {el_mt:.1f} s on {threads} threads",
            "topology": topo,
            "single_thread_mpkts": None if st is None else round(st, 3),
            "ipcksumperf_gbps_1thread": round(gbps, 2),
            "cpu_model": _cpu_model()}


def cpu_baseline_small(b, seconds=4.0, sample=1 << 20):
    """The same CPU full path over a sample of the C64 batch."""
    kind, _, _ = _cpu_lib()
    n = min(sample, b["n"])
    threads, _ = _cpu_topology()
    mt, el = _cpu_rate(b, n, threads, seconds)
    st, _ = _cpu_rate(b, n, 1, seconds / 2)
    return {"value": round(mt, 3), "unit": "Mpkts/s", "cores": threads, "kind": kind,
            "sample": f"{n} distinct C64 frames (64 B IPv4/UDP), full path, "
                      f"repeated for {el:.1f} s on {threads} threads",
            "single_thread_mpkts": round(st, 3)}


def tx_bench(ctx, b, n, dev, steps, warmup):
    """Tx-side checksum setting over batch b in place:
    reads every frame, writes 4 bytes per frame."""
    import torch
    kw = (dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]) if "off" in b
          else dict(stride=b["stride"], fixed_len=b["fixed_len"]))
    for _ in range(warmup):
        ctx.tx_cksum_device(b["frames"], n, **kw)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for a, z in ev:
        a.record()
        ctx.tx_cksum_device(b["frames"], n, **kw)
        z.record()
    torch.cuda.synchronize(dev)
    ms = float(np.median([a.elapsed_time(z) for a, z in ev]))
    ach = b["bytes"] / (ms * 1e-3) / 1e9
    return {"value": round(n / ms / 1e3, 1), "unit": "Mpkts/s", "kernel_ms": round(ms, 4),
            "workload": f"{b['cfg'].upper()} frames, checksums set in place",
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4)}}


def rewrite_bench(ctx, n, dev, rank, steps, warmup):
    """Header rewrite with incremental checksum updates (SURVEY 8(f) row 4,
    pptk_tx_rewrite_device) of a C64 batch in place: TTL decrement + new
    source/destination + new ports on every frame (a NAT + forwarding step;
    each frame is read once, 14 bytes of it written)."""
    import torch
    from pptk_amd.records import REWRITE_DTYPE
    from harness.synth import make_batch
    b = make_batch("c64", n, dev, first=rank * n)
    rw = np.zeros(1, REWRITE_DTYPE)
    rw["ops"], rw["src"], rw["dst"], rw["sport"], rw["dport"] = 0x1F, 0xC0A80A01, 0x0A000002, 4242, 443
    rw_t = torch.from_numpy(rw.view(np.uint8).copy()).to(dev)
    assert warmup + steps < 64          # the synthetic TTL is 64: stays > 0
    kw = dict(stride=b["stride"], fixed_len=b["fixed_len"])
    for _ in range(warmup):
        ctx.tx_rewrite_device(b["frames"], n, rw_t, **kw)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for a, z in ev:
        a.record()
        ctx.tx_rewrite_device(b["frames"], n, rw_t, **kw)
        z.record()
    torch.cuda.synchronize(dev)
    ms = float(np.median([a.elapsed_time(z) for a, z in ev]))
    ach = b["bytes"] / (ms * 1e-3) / 1e9
    del b
    release(dev)
    return {"value": round(n / ms / 1e3, 1), "unit": "Mpkts/s", "kernel_ms": round(ms, 4),
            "workload": "C64 frames, TTL-1 + src/dst/ports rewritten in place, "
                        "checksums updated incrementally (RFC 1624)",
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4)}}


def mss_bench(ctx, n, dev, steps, warmup, stride=80):
    """TCP MSS clamping (pptk_tcp_mss_clamp_device) of n IPv4 SYNs in place,
    each carrying a typical SYN option list (MSS 1460, SACK-permitted,
    timestamps, NOP, window scale: 74-byte frames in 80-byte slots); every
    timed launch clamps to a lower value than the one before, so every frame
    is parsed, walked and written (4 bytes) in every launch."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import framegen
    rng = np.random.default_rng(0x355)
    opts = (b"\x02\x04\x05\xb4" + b"\x04\x02" + b"\x08\x0a" + bytes(8) + b"\x01"
            + b"\x03\x03\x07")
    f = framegen.frame_tcp_opts(rng, opts=opts, payload=b"")
    slot = np.zeros(stride, np.uint8)
    slot[:len(f)] = np.frombuffer(f, np.uint8)
    frames = torch.from_numpy(slot).to(dev).repeat(n)
    kw = dict(stride=stride, fixed_len=len(f))
    mss = 1460
    assert warmup + steps < 400
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    for _ in range(warmup):
        mss -= 1
        ctx.mss_clamp_device(frames, n, mss, syn_only=True, status=st, **kw)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for a, z in ev:
        mss -= 1
        a.record()
        ctx.mss_clamp_device(frames, n, mss, syn_only=True, status=st, **kw)
        z.record()
    torch.cuda.synchronize(dev)
    clamped = int((st == 7).sum().item())
    ms = float(np.median([a.elapsed_time(z) for a, z in ev]))
    ach = n * len(f) / (ms * 1e-3) / 1e9
    del frames, st
    release(dev)
    return {"value": round(n / ms / 1e3, 1), "unit": "Mpkts/s", "kernel_ms": round(ms, 4),
            "workload": f"{n} IPv4 SYNs ({len(f)} B, MSS/SACK-perm/TS/NOP/WS options) in "
                        f"{stride}-byte slots, MSS clamped in place with checksum update",
            "clamped_every_frame": clamped == n,
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4)}}


def permit_bench(n, dev, ws, rank, steps, warmup, hash_size=1 << 16,
                 runs=("records", "keys", "keys_denying"), tune=None, lib_path=None):
    """Batched ip_permitted over a C64 batch: buckets of
    the /24 source prefixes in 2^16 buckets, every IPv4 frame a subject, one
    token array carried across the timed batches.  Three runs:
      records       pptk_rx_permit_device on the 64-byte records;
      keys          pptk_rx_permit_keys_device on the dense 4-byte keys the
                    same rx launch wrote (pptk_rx_dev_batch.d_key);
      keys_denying  the same with tokens refilled to 128 per bucket before
                    every batch: ~half the frames denied, so the per-bucket
                    resolve pass runs in every histogram block.
    Roofline: the algorithmic bytes of a verdict are its 4-byte key read and
    1-byte verdict written (records: the 16-byte slice of the record the key
    is in -- a DRAM burst of 64 bytes is what the memory moves for it), plus
    the token array read and written; `traffic` is the committed PMC
    summary's HBM bytes for that run (tools/opbench.py permit_<run>).
    `runs` selects the runs (profiling: one run per PMC pass)."""
    import torch
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    b = make_batch("c64", n, dev, first=rank * n)
    ctx = RxContext(dev.index, KEY, 24, 0, hash_size, lib_path=lib_path)
    if tune is not None:          # (A/B: PPTK_RX_TUNE_PERMIT_PASSES = the four-launch path)
        ctx.set_tuning(-1, tune)
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    recs = ctx.batch_device(b["frames"], n, stride=b["stride"], fixed_len=b["fixed_len"],
                            key_out=keys)
    del b
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    scratch = torch.empty(ctx._L.pptk_rx_permit_scratch_bytes(n, hash_size), dtype=torch.uint8,
                          device=dev)

    def timed(call, refill=None):
        tok = torch.full((hash_size,), 1 << 20, dtype=torch.int32, device=dev)
        for _ in range(warmup):
            if refill:
                refill(tok)
            call(tok)
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        for a, z in ev:
            if refill:
                refill(tok)
            a.record()
            call(tok)
            z.record()
        torch.cuda.synchronize(dev)
        ms = float(np.median([a.elapsed_time(z) for a, z in ev]))
        v = verdict.cpu().numpy()
        return ms, {"permitted": int((v == 1).sum()), "denied": int((v == 0).sum()),
                    "not_subject": int((v == 2).sum())}

    def line(ms, per_frame_bytes, what, counts, run):
        alg = n * per_frame_bytes + 2 * 4 * hash_size
        ach = alg / (ms * 1e-3) / 1e9
        traffic, src = pmc_traffic("op_permit_" + run, n)
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": alg,
                "traffic": traffic}
        if src:
            roof["traffic_source"] = src
        return {"value": round(n / ms / 1e3, 1), "unit": "Mpkts/s", "ms_per_batch": round(ms, 4),
                "frames": n, "hash_size": hash_size, "workload": what, "verdicts": counts,
                "roofline": roof}

    out = {}
    if "records" in runs:
        ms, c = timed(lambda tok: ctx.permit_device(recs, 4, tok, verdict=verdict,
                                                    scratch=scratch))
        out = line(ms, 64 + 1, "C64 records (64 B each), IPv4 /24 buckets, all frames subject",
                   c, "records")
    if "keys" in runs:
        ms, c = timed(lambda tok: ctx.permit_keys_device(keys, 4, tok, verdict=verdict,
                                                         scratch=scratch))
        out["keys"] = line(ms, 4 + 1, "dense 4-byte keys of the same batch (d_key)", c, "keys")
    if "keys_denying" in runs:
        ms, c = timed(lambda tok: ctx.permit_keys_device(keys, 4, tok, verdict=verdict,
                                                         scratch=scratch),
                      refill=lambda tok: tok.fill_(128))
        out["keys_denying"] = line(ms, 4 + 1, "dense keys, 128 tokens per bucket before each "
                                   "batch (~half the frames denied: resolve pass in every block)",
                                   c, "keys_denying")
    del recs, keys, verdict, scratch
    release(dev)
    return out


def pcie_ceiling(dev, mb=96, reps=20):
    """The host-to-device copy ceiling the end-to-end path is bound by:
    pinned hipMemcpyAsync of mb MB, GB/s (tools/pcie_probe.py's h2d row)."""
    import torch
    h = torch.empty(mb << 20, dtype=torch.uint8).pin_memory()
    d = torch.empty(mb << 20, dtype=torch.uint8, device=dev)
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(dev)
    return round((mb << 20) * reps / (time.perf_counter() - t0) / 1e9, 2)


def gpu_numa(dev):
    """The GPU's NUMA node (sysfs, by PCI bus id) and the CPUs of that node
    this process may run on: {"node": N, "cpus": [...]}, or None when the
    box does not say."""
    import torch
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read().strip())
        if node < 0:
            return None
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = set()
            for part in f.read().strip().split(","):
                lo, _, hi = part.partition("-")
                cpus.update(range(int(lo), int(hi or lo) + 1))
        mine = sorted(cpus & os.sched_getaffinity(0))
        return {"node": node, "bdf": bdf, "cpus": mine} if mine else None
    except (OSError, AttributeError, ValueError):
        return None


def e2e_bench(dev, seconds=2.0, cfgs=(("c1500", "c1500", 1 << 20, False, False),
                                      ("c64", "c64", 1 << 22, True, False),
                                      ("c64_rec32", "c64", 1 << 22, True, True)),
              numa_local=True):
    """End to end, host to host (the north star's "rate
    including pinned hipMemcpyAsync to and from the GPU"): pptk_rx_batch on
    borrowed ldp_packet frames in host memory (reference rx loop
    ldp/ldprecv.c:60-70: frames in a netmap ring, ldp/ldpnetmap.c:163-185),
    records back in host memory, synchronous, chunks of 65 536 frames
    pipelined over four streams.  Two paths per config: "staged" (host
    threads gather the frames into pinned staging, DMA down) and "ring" (the
    frame area registered once with pptk_rx_register_ring: dense chunks go
    down as one DMA span, nothing gathered); with `reg` the record array is
    registered too (records written in place over PCIe, no copy back); with
    `compact` the records are the 32-byte struct pptk_rx_rec32
    (pptk_rx_batch32: half the bytes back over PCIe, what bounds C64).
    Every mode is checked bit-exact against a device-resident launch of the
    same frames before it is timed.  Reported: the faster path, Mpkt/s,
    frame GB/s and its fraction of this box's pinned H2D copy rate."""
    threads, _ = _cpu_topology()
    gt = max(1, min(16, threads))
    # An rx loop runs on the CPUs next to its NIC and GPU, and its ring lives
    # in their memory (netmap allocates it once, ldp/ldpnetmap.c:163-185).
    # numa_local: this process (so the library's gather threads, created per
    # context below, and the first touch of the ring and record arrays) on the
    # GPU's NUMA node for the measurement -- unpinned, the ring's pages land
    # wherever the main thread happens to run, and a ring on the far socket
    # made the C64 ring path swing between runs (716 vs 588 Mpkt/s with 32-byte
    # records, profiles/r06/e2e/).
    # After the device-resident configs the driver is still scrubbing the
    # tens of GB their placement probes and buffers freed; beside that scrub
    # the C64 paths measured 20-25 % slower (588 / 518 against 716 / 683
    # Mpkt/s ring / staged with 32-byte records, profiles/r06/e2e/), so the
    # measurement starts after it.
    scrub_s = wait_scrub()
    numa = gpu_numa(dev) if numa_local else None
    old_aff = os.sched_getaffinity(0)
    if numa:
        os.sched_setaffinity(0, numa["cpus"])
    try:
        out = {"pcie_h2d_gbs": pcie_ceiling(dev), "gather_threads": gt, "scrub_wait_s": scrub_s,
               "numa": None if not numa else {"node": numa["node"], "cpus": len(numa["cpus"])}}
        _e2e_configs(dev, seconds, cfgs, gt, out)
    finally:
        if numa:
            os.sched_setaffinity(0, old_aff)
    return out


def _e2e_configs(dev, seconds, cfgs, gt, out):
    import torch
    from pptk_amd.records import REC32_DTYPE, REC_DTYPE, diff_records
    from pptk_amd.rx import RxContext, ldp_packets
    from harness.synth import make_batch
    ceil = out["pcie_h2d_gbs"]
    for key, cfg, n, reg, compact in cfgs:
        b = make_batch(cfg, n, dev)
        stride, flen = b["stride"], b["fixed_len"]
        # the host "ring", first touched here (on the CPUs just chosen)
        ring = np.zeros(n * stride + 64, dtype=np.uint8)
        torch.from_numpy(ring).copy_(b["frames"][: n * stride + 64])
        ctx = RxContext(0, KEY, max_batch=65536, max_frame=1518, gather_threads=gt)
        ref = ctx.batch_device(b["frames"], n, stride=stride, fixed_len=flen, compact=compact)
        dt = REC32_DTYPE if compact else REC_DTYPE
        want = ref.cpu().numpy().reshape(-1).view(dt)
        del b, ref
        pkts = ldp_packets(ring, np.arange(n, dtype=np.uint64) * stride,
                           np.full(n, flen, np.uint16))
        outbuf = np.zeros(n, dtype=dt)                  # reused, as an rx loop's array
        if reg:
            ctx.register_ring(outbuf)
        res = {}
        for mode in ("staged", "ring"):
            if mode == "ring":
                ctx.register_ring(ring)
            got = ctx.batch_host(pkts, out=outbuf, compact=compact)
            if diff_records(got, want, dtype=dt):
                raise RuntimeError(f"e2e {key} {mode}: records differ from the device batch")
            reps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < seconds:
                ctx.batch_host(pkts, out=outbuf, compact=compact)
                reps += 1
            el = (time.perf_counter() - t0) / reps
            res[mode] = round(n / el / 1e6, 2)
            if mode == "ring":
                ctx.unregister_ring(ring)
        if reg:
            ctx.unregister_ring(outbuf)
        ctx.close()
        best = max(res, key=res.get)
        gbs = res[best] * flen / 1e3
        out[key] = {"mpkts": res[best], "path": best, "frame_gbs": round(gbs, 2),
                    "of_pcie": round(gbs / ceil, 3) if ceil else None, "frames": n,
                    "records": ("registered" if reg else "copied") + (" 32 B" if compact else " 64 B"),
                    "staged_mpkts": res["staged"], "ring_mpkts": res["ring"]}
        del ring, pkts, outbuf, want
        release(dev)


def forced_ms(ctx, b, recs, n, variant, steps, warmup=3):
    """Median kernel ms of this batch with the kernel variant forced (e.g.
    CMIX through M6, the kernel that bins each tile's lanes by length --
    BASELINE.json configs[3]'s "lanes binned by length" -- beside the
    autotuned choice); records unchanged (checked), the forcing undone."""
    import torch
    from pptk_amd.rx import VARIANTS
    kw = (dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]) if "off" in b
          else dict(stride=b["stride"], fixed_len=b["fixed_len"]))
    want = recs.clone()
    ctx.set_tuning(VARIANTS.index(variant), -1)
    try:
        for _ in range(warmup):
            ctx.batch_device(b["frames"], n, recs=recs, **kw)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        for a, z in ev:
            a.record()
            ctx.batch_device(b["frames"], n, recs=recs, **kw)
            z.record()
        torch.cuda.synchronize()
        assert VARIANTS[ctx.last_variant()] == variant
    finally:
        ctx.set_tuning(-1, -1)
    same = bool(torch.equal(recs, want))
    del want
    return round(float(np.median([a.elapsed_time(z) for a, z in ev])), 4), same


def gather_bench(ctx, gb, ws, dev, steps, stream=None):
    """The all-gather of `per` u64 flow hashes per rank alone
    (pptk_rx_allgather_hash): time and bandwidths, on `stream`
    (default: the current one)."""
    import torch
    main = stream or torch.cuda.current_stream(dev)
    GATHER_STREAMS[:] = [(ctx, main)]
    for _ in range(3):
        gb.gather(ctx, stream=main)
    barrier(ws, dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        gb.gather(ctx, stream=main)
    barrier(ws, dev)
    t = max_over_ranks((time.perf_counter() - t0) / steps, ws, dev)
    alg, bus = gather_bw(gb.per, ws, t)
    return {"bytes_per_rank": gb.per * 8, "ms": round(t * 1e3, 4), "algbw_gbs": alg,
            "busbw_gbs": bus, "rccl_ranks": ctx.comm_info()[0]}


# the newest round's committed PMC summary (tools/pmc_summary.py)
PMC_SUMMARY = next((p for p in (os.path.join(ROOT, "profiles", r, "pmc_summary.json")
                                for r in ("r06", "r05", "r04", "r03", "r02", "r01")) if os.path.exists(p)),
                   os.path.join(ROOT, "profiles", "r01", "pmc_summary.json"))


def pmc_traffic(cfg, frames):
    """HBM bytes per launch of this config from the committed rocprofv3 PMC
    passes (FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected; see
    tools/pmc_summary.py), taken at N_PER_GPU frames per launch and scaled
    linearly to `frames` (every tile moves the same bytes); (None, None)
    when no summary exists."""
    try:
        with open(PMC_SUMMARY) as f:
            e = json.load(f)[cfg]
        return (int(e.get("traffic_bytes_per_call", e["traffic_bytes"]) * frames / N_PER_GPU),
                os.path.relpath(PMC_SUMMARY, ROOT))
    except (OSError, KeyError, ValueError):
        return None, None


_LIVE_PMC_FAILED = []   # after one failed pass the later configs skip theirs


def live_pmc(cfg, variant, n, timeout_s=60):
    """Same-run HBM traffic of this config's rx kernel: one FETCH_SIZE pass
    and one WRITE_SIZE pass (separate rocprofv3 runs, MI355X_MICROARCH.md
    HBM section), each a child process `bench.py --only cfg` of n frames
    with the kernel shape this run chose (PPTK_RX_VARIANT), killed after
    timeout_s (a pass takes 5-10 s).  Per launch, median over the child's
    launches; FETCH_SIZE x2 (gfx950 counts half of 16-byte/lane streaming
    reads), both in KiB.  Returns (traffic bytes, detail dict) or (None,
    reason); once a pass has failed, every later call returns at once, so a
    profiler that hangs costs the bench one time limit, not one per config."""
    if _LIVE_PMC_FAILED:
        return None, f"skipped: an earlier pass failed ({_LIVE_PMC_FAILED[0]})"
    import shutil
    import subprocess
    import tempfile
    from pptk_amd.rx import VARIANTS
    from tools.pmc_summary import counter
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rp):
        return None, "rocprofv3 not found"
    if (any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)
            or "rocprof" in os.environ.get("LD_PRELOAD", "")):
        return None, "already under rocprofv3"
    base = tempfile.mkdtemp(prefix="pptk_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    env = dict(os.environ, PPTK_RX_VARIANT=str(VARIANTS.index(variant)))
    got = {}
    t0 = time.perf_counter()
    try:
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(base, c)
            cmd = ["timeout", "-s", "KILL", str(timeout_s), rp, "--pmc", c,
                   "--kernel-include-regex", "rx_kernel", "-d", d, "-o", "run",
                   "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__),
                   "--only", cfg, "--frames", str(n), "--steps", "3", "--warmup", "1",
                   "--no-cpu", "--no-check", "--no-membench", "--no-rec32", "--no-place",
                   "--settle", "0.3", "--no-live-pmc"]
            r = subprocess.run(cmd, env=env, cwd=base, stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, timeout=timeout_s + 30)
            if r.returncode != 0:
                _LIVE_PMC_FAILED.append(f"{cfg} {c} exit {r.returncode}")
                return None, f"{c} pass exited {r.returncode}: {r.stderr.decode()[-200:]}"
            vals, _, kname = counter(d, c)
            got[c] = float(np.median(vals))
    except Exception as e:          # the committed summary stays the fallback
        _LIVE_PMC_FAILED.append(f"{cfg}: {type(e).__name__}")
        return None, f"{type(e).__name__}: {e}"
    finally:
        shutil.rmtree(base, ignore_errors=True)
    rd, wr = got["FETCH_SIZE"] * 2 * 1024, got["WRITE_SIZE"] * 1024
    return int(rd + wr), {"read_bytes": int(rd), "write_bytes": int(wr), "kernel": kname,
                          "seconds": round(time.perf_counter() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=N_PER_GPU,
                    help="frames per GPU (weak) or in total (strong)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak: --frames per GPU; strong: --frames split over the GPUs")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--only", default=None, help="run just this config (profiling)")
    ap.add_argument("--no-rec32", action="store_true",
                    help="skip the compact-record runs (profiling: one record format per trace)")
    ap.add_argument("--no-membench", action="store_true",
                    help="skip the in-process HBM read/copy ceiling probe")
    ap.add_argument("--settle", type=float, default=SETTLE_S,
                    help="seconds of untimed launches before the warmup steps")
    ap.add_argument("--no-place", action="store_true",
                    help="one record buffer as allocated, no placement probe")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the host-to-host (pptk_rx_batch) measurement")
    ap.add_argument("--detail", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="where the full result (every sub-measurement) is written; the "
                         "stdout line is its compact summary")
    ap.add_argument("--no-live-pmc", action="store_true",
                    help="no same-run rocprofv3 FETCH_SIZE/WRITE_SIZE passes (roofline.traffic "
                         "then comes from the committed summary)")
    args = ap.parse_args()
    launch_ranks(sys.argv[1:], args.gpus)

    import torch
    from pptk_amd.rx import RxContext
    from pptk_amd.shard import GatherBuffer, shard_range
    ws, rank, dev = dist_setup(args.gpus)
    ctx = RxContext(dev.index, KEY)
    place = not args.no_place
    # weak: --frames per GPU; strong: --frames in total, equal shards
    # (pptk_rx_shard_range: the last shards padded for the all-gather)
    n_total = args.frames * ws if args.scaling == "weak" else args.frames
    gbs = None
    comm_error = None
    split = None
    if dist_on(ws) and COLL_CUS > 0 and (ws > 1 or "PPTK_BENCH_COLL_CUS" in os.environ):
        # the batches on all CUs but COLL_CUS, the gather on those
        # (pptk_rx_stream_split; placement and autotune probes run split too),
        # BEFORE the communicator: the library caps its channels at COLL_CUS
        # (ncclConfig_t.maxCTAs), one RCCL block per CU left to the gather.
        # A one-rank gather (PPTK_BENCH_FORCE_DIST) launches nothing that
        # needs CUs: split only when asked.
        try:
            split = ctx.stream_split(COLL_CUS)
        except OSError as e:   # e.g. a partitioned GPU with fewer CUs: run unsplit
            log(f"[rank {rank}] no CU split ({e}); the gather shares the CUs")
    if dist_on(ws):
        comm_error = join_all(ctx, ws, rank)     # RCCL communicator in libpptkrx.so
        if comm_error:
            log(f"[rank {rank}] no all-gather: {comm_error}")
            if split:
                ctx.stream_join()
                split = None
        else:
            # the gather buffers are placed inside run_config, once the
            # batch's frame and record buffers are (placed_gather)
            gbs = "place" if place else [GatherBuffer(n_total, ws, rank, dev) for _ in range(2)]
        first, n, _ = shard_range(n_total, ws, rank)
    else:
        first, n = 0, n_total
    check = not args.no_check

    primary_cfg = args.only or "c1500"
    if split:
        torch.cuda.set_stream(split[0])
    prim = run_config(primary_cfg, n, ctx, dev, ws, rank, args.steps, args.warmup, gbs, check,
                      args.settle, first=first, place=place, n_gather_total=n_total,
                      coll_stream=split[1] if split else None)
    gbs = prim.pop("_gbs")
    log(f"[rank {rank}] {primary_cfg}: {prim['mpkts']:.1f} Mpkts/s, kernel {prim['kernel_ms']:.3f} ms")
    gat_split = None
    if split:
        torch.cuda.synchronize(dev)
        # the gather alone on the CUs the split left it
        gat_split = gather_bench(ctx, gbs[0], ws, dev, args.steps, stream=split[1])
        torch.cuda.synchronize(dev)
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
        GATHER_STREAMS[:] = [(ctx, torch.cuda.default_stream(dev))]   # (not the split's)
        ctx.stream_join()
        del split
    nog = gat = None
    if gbs:
        # same launches without the collective: the kernel-only duration the
        # roofline uses, and the rate "without the gather" 
        # (into the primary run's record buffer: the same placement, so the
        # difference is the collective's alone)
        nog = run_config(primary_cfg, n, ctx, dev, ws, rank, args.steps, args.warmup, None, False,
                         args.settle, batch=prim["_batch"], first=first, recs=prim["_recs"])
        del nog["_batch"], nog["_recs"]
        nog["mpkts"] = n_total * args.steps / nog["wall_s"] / 1e6
        gat = gather_bench(ctx, gbs[0], ws, dev, args.steps)
        if gat["rccl_ranks"] != ws:
            raise RuntimeError(f"the RCCL communicator has {gat['rccl_ranks']} ranks, not {ws}")
        gat["overlap_loss"] = round(1.0 - prim["mpkts"] / nog["mpkts"], 4)
        gat["coll_cus"] = COLL_CUS if gat_split else 0
        # the channel cap the library gave the communicator (ncclConfig_t.maxCTAs)
        gat["max_ctas"] = COLL_CUS if gat_split else None
        if gat_split:
            gat["split"] = {k: gat_split[k] for k in ("ms", "algbw_gbs", "busbw_gbs")}
        gat["buffer_placement"] = prim.get("gather_placement")
        if check:
            gat["gathered_check"] = gathered_check(prim, gbs, n, dev)
        log(f"[rank {rank}] no gather: {nog['mpkts']:.1f} Mpkts/s; all-gather {gat}")

    box = None
    if not args.no_membench:
        from harness.membench import measure
        box = measure(prim["_batch"]["frames"])
        sol = mix_sol(prim["_batch"], prim["_recs"], n)
        if sol:
            box["mix_ms"], box["mix_desc"] = sol
        log(f"[rank {rank}] box HBM: {box}")

    # every rank's kernel time (the scaling curve's per-GPU view)
    per_rank_ms = per_rank(round((nog or prim)["kernel_ms"], 4), ws)
    bytes_per_launch = prim["bytes"]
    # with N > 1 the primary run's event pair also spans the wait on the
    # previous batch's gather, so the kernel duration comes from the run
    # without the collective
    kernel_ms = (nog or prim)["kernel_ms"]
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic(primary_cfg, n)
    rw = (bytes_per_launch + prim["rec_bytes"]) / (kernel_ms * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "rw_achieved": round(rw, 1), "rw_frac": round(rw / HBM_PEAK_GBS, 4),
                "traffic_source": tsrc,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "kernel_ms": round(kernel_ms, 4), "kernel_variant": prim["variant"]}
    roofline.update(as_allocated(prim))
    if box and "mix_ms" in box:
        # fraction of this GPU's speed of light for the same read/write mix
        # (a trivial kernel moving the same bytes, tools/rwmix.hip)
        roofline["mix_sol_ms"] = box["mix_ms"]
        roofline["mix_sol_frac"] = round(box["mix_ms"] / kernel_ms, 4)
        # the best read-roofline fraction ANY kernel moving this launch's
        # bytes into these buffers reaches on this GPU: what the 1 GB of
        # record writes costs beside the 25 GB read (0.2-1.2 ms) follows the
        # buffers' placement (placed_buffers), and with a badly placed
        # buffer this ceiling itself is below 0.70
        ceil = bytes_per_launch / (box["mix_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS
        roofline["mix_sol_read_frac"] = round(ceil, 4)
        if roofline["frac"] < 0.70:
            roofline["below_target_note"] = (
                f"read-roofline fraction {roofline['frac']} < 0.70 on this GPU: the trivial "
                f"kernel moving the same bytes reaches only {round(ceil, 4)} here (record "
                f"writes cost {round(box['mix_ms'] - bytes_per_launch / box.get('read_nt_gbs', 1) / 1e6, 2)} "
                f"ms beside the read stream); the rx kernel is at {roofline['mix_sol_frac']} of it")

    # the same batch with compact 32-byte records (struct pptk_rx_rec32)
    rec32 = None
    if not args.no_rec32:
        r32 = run_config(primary_cfg, n, ctx, dev, ws, rank, args.steps, args.warmup, None,
                         check, args.settle, compact=True, batch=prim["_batch"], first=first,
                         place=place)
        rec32 = summary(r32, n)
        del r32["_batch"], r32["_recs"]
        log(f"[rank {rank}] {primary_cfg} rec32: {rec32['value']} Mpkts/s")

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu and primary_cfg == "c1500":
        cpu = cpu_baseline(prim["_batch"], seconds=args.cpu_seconds)
        log(f"cpu baseline: {cpu}")
    # tx side on the same frames (they are rewritten in place, so after
    # every receive measurement of this batch): pptk_tx_cksum_device
    tx = None
    if not args.no_secondary and args.only is None:
        tx = tx_bench(ctx, prim["_batch"], n, dev, args.steps, args.warmup)
        log(f"[rank {rank}] tx: {tx}")
    full_check = prim.get("full_batch_check")
    sample_check = prim.get("oracle_sample")
    del prim["_batch"], prim["_recs"]
    release(dev)

    secondary = {}
    if not args.no_secondary and args.only is None:
        for cfg in ("c64", "cmix", "imix", "jmix"):
            r = run_config(cfg, n, ctx, dev, ws, rank, args.steps, args.warmup, None, check,
                           args.settle, first=first, place=place)
            secondary[cfg] = summary(r, n)
            if not args.no_membench:
                sol = mix_sol(r["_batch"], r["_recs"], n)
                if sol:
                    secondary[cfg]["roofline"]["mix_sol_ms"] = sol[0]
                    secondary[cfg]["roofline"]["mix_sol_frac"] = round(sol[0] / r["kernel_ms"], 4)
            if cfg in ("cmix", "imix", "jmix"):
                secondary[cfg]["binned"] = binned_bench(ctx, r["_batch"], n, dev, args.steps,
                                                        args.warmup, recs=r["_recs"])
            if cfg == "cmix" and r["variant"] != "M6":
                # configs[3] as written, "lanes binned by length": the kernel
                # that bins each tile's lanes (M6), beside the autotuned shape
                ms, same = forced_ms(ctx, r["_batch"], r["_recs"], n, "M6", args.steps)
                secondary[cfg]["m6"] = {"kernel_ms": ms, "same_records": same,
                                        "frac": round(r["bytes"] / (ms * 1e-3) / 1e9
                                                      / HBM_PEAK_GBS, 4)}
            if cfg == "c64" and not args.no_rec32:
                r32 = run_config(cfg, n, ctx, dev, ws, rank, args.steps, args.warmup, None,
                                 check, args.settle, compact=True, batch=r["_batch"], first=first,
                                 place=place)
                secondary[cfg]["rec32"] = summary(r32, n)
                del r32["_batch"], r32["_recs"]
            if cfg == "c64" and rank == 0 and ws == 1 and not args.no_cpu:
                secondary[cfg]["cpu_baseline"] = cpu_baseline_small(
                    r["_batch"], seconds=max(1.0, args.cpu_seconds / 2.5))
            del r["_batch"], r["_recs"]
            release(dev)

    permit = rewrite = mss = None
    if not args.no_secondary and args.only is None:
        permit = permit_bench(n, dev, ws, rank, args.steps, args.warmup)
        log(f"[rank {rank}] permit: {permit}")
        if args.steps + args.warmup < 400:
            mss = mss_bench(ctx, n, dev, args.steps, args.warmup)
            log(f"[rank {rank}] mss: {mss}")
        if args.steps + args.warmup < 64:
            rewrite = rewrite_bench(ctx, n, dev, rank, args.steps, args.warmup)
            log(f"[rank {rank}] rewrite: {rewrite}")

    # end to end, host to host (rank 0 of a one-GPU run)
    e2e = None
    if rank == 0 and ws == 1 and not args.no_secondary and args.only is None and not args.no_e2e:
        try:
            e2e = e2e_bench(dev)
        except Exception as e:          # reported, never fatal to the device-resident line
            e2e = {"error": f"{type(e).__name__}: {e}"[:200]}
        log(f"e2e: {e2e}")

    # roofline.traffic from this run: rocprofv3 PMC passes over the same
    # workload and kernel shape, in child processes (rank 0 of a one-GPU
    # run; the committed summary is the fallback)
    if rank == 0 and ws == 1 and not args.no_live_pmc:
        t, info = live_pmc(primary_cfg, prim["variant"], n)
        if t is not None:
            roofline["traffic"] = t
            roofline["traffic_source"] = "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, this run"
            roofline["traffic_detail"] = info
        else:
            roofline["traffic_live_error"] = info
        log(f"live pmc {primary_cfg}: {t} {info}")
        for cfg, sec in secondary.items():
            t, info = live_pmc(cfg, sec["kernel_variant"], n)
            if t is not None:
                sec["roofline"]["traffic"] = t
                sec["roofline"]["traffic_detail"] = info
            else:
                sec["roofline"]["traffic_live_error"] = info
            log(f"live pmc {cfg}: {t} {info}")

    if rank == 0:
        full = {
            "metric": METRIC,
            "value": round(prim["mpkts"], 1),
            "unit": "Mpkts/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(prim["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"{primary_cfg.upper()}: {n} frames per GPU"
                                   + (" x 1500 B IPv4/TCP" if primary_cfg == "c1500" else ""),
                       "frames_per_gpu": n, "global_frames": n_total,
                       "parallelism": f"shard{ws}" + ("+rccl_allgather(flow_hash)" if gbs else ""),
                       "rccl_ranks": ctx.comm_info()[0] if gbs else None,
                       "key": "01..10"},
            "roofline": roofline,
            "record_placement": prim.get("placement"),
            "per_rank_kernel_ms": per_rank_ms,
            "cpu_baseline": cpu,
            "value_no_gather": None if nog is None else round(nog["mpkts"], 1),
            "rec32": rec32,
            "allgather": gat if gat else ({"error": comm_error} if comm_error else None),
            "box_hbm": box,
            "parity": {"full_batch": full_check, "oracle_sample": sample_check},
            "secondary": secondary,
            "permit": permit,
            "tx": tx,
            "rewrite": rewrite,
            "mss_clamp": mss,
            "e2e": e2e,
        }
        line = compact_line(full, detail_path=args.detail)
        problems = validate_line(line)
        if problems:
            line["line_problems"] = problems
        try:
            if os.path.dirname(args.detail):
                os.makedirs(os.path.dirname(args.detail), exist_ok=True)
            with open(args.detail, "w") as f:
                json.dump(full, f)
        except OSError as e:
            log(f"detail not written: {e}")
        log("full result: " + json.dumps(full))
        print(json.dumps(line), flush=True)
        if problems and dist_on(ws):
            raise SystemExit(f"multi-GPU line failed its checks: {problems}")
    if dist_on(ws):
        import torch.distributed as dist
        # every rank tears its RCCL communicator down at the same point,
        # after the last collective, before the control plane goes away
        barrier(ws, dev)
        if gbs:
            ctx.comm_destroy()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
