"""BENCH TOOLING: one batch operation alone, for rocprofv3 PMC passes.

    python tools/opbench.py OP [--steps K] [--warmup W]

OP: tx (pptk_tx_cksum_device on C1500), tx_cmix, rewrite (pptk_tx_rewrite_device
on C64), mss (pptk_tcp_mss_clamp_device, 16 M SYNs), permit
(pptk_rx_permit_device over 16 M C64 records), binned (CMIX through
pptk_rx_batch_device_mixed), allgather (a one-rank communicator's in-place
pptk_rx_allgather_hash after every C1500 launch), allgather_copy (the same
with a separate send buffer: one rank's collective then copies 128 MiB per
batch beside the rx grid), gather_emul (the HBM traffic of an 8-rank gather,
emulated by a device copy).  Uses bench.py's own
measurement functions; prints one JSON line with the timing and
`changed_bytes_per_launch` (the bytes the op must write), the denominator
of the write-amplification ratio WRITE_SIZE / changed bytes."""
import argparse
import json

import numpy as np
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

N = bench.N_PER_GPU


def gather_emul(ctx, dev, n, steps, warmup, world=8):
    """The HBM side of the C8G all-gather on one GPU: a ring all-gather of
    n u64 hashes per rank over `world` ranks makes every rank read and write
    (world - 1) * n * 8 bytes of its HBM per batch (it forwards world - 1
    chunks and lands world - 1 chunks).  Emulated by a device-to-device copy
    of that size on a second stream beside every C1500 launch, as bench.py
    overlaps the real gather; reports the launch rate with and without it.
    (xGMI link time is not emulated: it overlaps the kernel.)"""
    import time
    import torch
    from harness.synth import make_batch
    b = make_batch("c1500", n, dev)
    recs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    nbytes = (world - 1) * n * 8
    src = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    out = {}
    for mode in ("alone", "with_copy", "alone", "with_copy"):
        for k in range(warmup + steps):
            if k == warmup:
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
            ctx.batch_device(b["frames"], n, stride=1500, fixed_len=1500, recs=recs)
            if mode == "with_copy":
                ev = torch.cuda.Event()
                ev.record(main_s)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    dst.copy_(src)
        torch.cuda.synchronize(dev)
        out.setdefault(mode, []).append((time.perf_counter() - t0) / steps * 1e3)
    a, w = min(out["alone"]), min(out["with_copy"])
    return {"ms_per_batch_alone": round(a, 4), "ms_per_batch_with_gather_traffic": round(w, 4),
            "overlap_loss": round(1 - a / w, 4), "world": world,
            "gather_bytes_read_and_written_per_rank": nbytes,
            "changed_bytes_per_launch": 64 * n}


def gather_emul_place(ctx, dev, n, steps, warmup, world=8, ncand=6):
    """Does the destination of the gather's writes matter like the record
    buffer's does?  The emulated 8-rank gather traffic (a device copy of
    7 x 128 MiB beside every C1500 launch, frames and records placed as
    bench.py places them) into each of `ncand` destination buffers
    allocated 4 GB apart; ms per batch for each, and without the copy."""
    import time
    import torch
    import bench
    from harness.synth import make_batch
    b = make_batch("c1500", n, dev)
    kw = dict(stride=1500, fixed_len=1500)
    recs, place = bench.placed_buffers(ctx, b, n, dev, False, kw)
    nbytes = (world - 1) * n * 8
    src = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    hold, dsts = [], []
    for _ in range(ncand):
        hold.append(torch.empty(4 << 30, dtype=torch.uint8, device=dev))
        dsts.append(torch.empty(nbytes, dtype=torch.uint8, device=dev))
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)

    def run(dst):
        for k in range(warmup + steps):
            if k == warmup:
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
            ctx.batch_device(b["frames"], n, recs=recs, **kw)
            if dst is not None:
                ev = torch.cuda.Event()
                ev.record(main_s)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    dst.copy_(src)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / steps * 1e3
    res = {"alone": [], "dst": [[] for _ in dsts]}
    for _ in range(2):
        res["alone"].append(run(None))
        for i, d in enumerate(dsts):
            res["dst"][i].append(run(d))
    return {"ms_alone": round(min(res["alone"]), 4),
            "ms_with_copy_per_dst": [round(min(v), 4) for v in res["dst"]],
            "placement": place["chosen_ms"], "changed_bytes_per_launch": 64 * n}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("op")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    import torch
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    ctx = RxContext(0, bench.KEY)
    op, n = args.op, N
    if op in ("tx", "tx_cmix"):
        b = make_batch("c1500" if op == "tx" else "cmix", n, dev)
        r = bench.tx_bench(ctx, b, n, dev, args.steps, args.warmup)
        # IPv4 header checksum + TCP/UDP checksum: 2 + 2 bytes per frame
        r["changed_bytes_per_launch"] = 4 * n
    elif op == "rewrite":
        r = bench.rewrite_bench(ctx, n, dev, 0, args.steps, args.warmup)
        # TTL (1 B), IPv4 checksum (2), source and destination (8), ports
        # (4), UDP checksum (2): 17 bytes changed per frame
        r["changed_bytes_per_launch"] = 17 * n
    elif op == "mss":
        r = bench.mss_bench(ctx, n, dev, args.steps, args.warmup)
        r["changed_bytes_per_launch"] = 4 * n      # MSS value + TCP checksum
    elif op == "permit":
        r = bench.permit_bench(n, dev, 1, 0, args.steps, args.warmup)
        r["changed_bytes_per_launch"] = n          # one verdict byte per frame
    elif op.startswith("permit_"):   # one run of the rate limiter alone (PMC passes)
        run = op[len("permit_"):]
        r = bench.permit_bench(n, dev, 1, 0, args.steps, args.warmup, runs=(run,))
        r = r.get(run, r)
        r["changed_bytes_per_launch"] = n
    elif op == "binned":
        b = make_batch("cmix", n, dev)
        r = bench.binned_bench(ctx, b, n, dev, args.steps, args.warmup)
        r["changed_bytes_per_launch"] = 64 * n
    elif op == "binned_ab":
        # batch order and binned on the same CMIX batch and record buffer,
        # alternating rounds (PPTK_RX_BIN_BOUNDS sets the binned groups)
        b = make_batch("cmix", n, dev)
        recs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        kw = dict(off=b["off"], lens=b["lens"], max_len=b["max_len"], recs=recs)
        bo, bi = [], []
        for _ in range(3):
            for _ in range(args.warmup):
                ctx.batch_device(b["frames"], n, **kw)
            torch.cuda.synchronize(dev)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.steps)]
            for a, z in evs:
                a.record()
                ctx.batch_device(b["frames"], n, **kw)
                z.record()
            torch.cuda.synchronize(dev)
            bo += [a.elapsed_time(z) for a, z in evs]
            bi.append(bench.binned_bench(ctx, b, n, dev, args.steps, args.warmup,
                                         recs=recs)["ms_per_batch"])
        r = {"batch_order_ms": round(float(np.median(bo)), 4),
             "binned_ms": round(float(np.median(bi)), 4),
             "bounds": os.environ.get("PPTK_RX_BIN_BOUNDS", "default")}
    elif op in ("allgather", "allgather_copy"):
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        os.environ["PPTK_BENCH_FORCE_DIST"] = "1"
        import torch.distributed as dist
        from pptk_amd.shard import GatherBuffer, join
        dist.init_process_group("gloo", rank=0, world_size=1)
        join(ctx, 1, 0)
        # allgather_copy: a separate send buffer, so the one-rank collective
        # really moves the 128 MiB (an RCCL copy beside the rx grid)
        gbs = [GatherBuffer(n, 1, 0, dev, inplace=op == "allgather") for _ in range(2)]
        res = bench.run_config("c1500", n, ctx, dev, 1, 0, args.steps, args.warmup, gbs, False,
                               settle=0.3, first=0)
        nog = bench.run_config("c1500", n, ctx, dev, 1, 0, args.steps, args.warmup, None, False,
                               settle=0.3, first=0, batch=res["_batch"], recs=res["_recs"])
        r = {"kernel_ms": round(res["kernel_ms"], 4), "mpkts": round(res["mpkts"], 1),
             "mpkts_no_gather": round(nog["mpkts"], 1),
             "overlap_loss": round(1 - res["mpkts"] / nog["mpkts"], 4),
             "changed_bytes_per_launch": 64 * n + 8 * n}
        dist.destroy_process_group()
    elif op == "gather_emul":
        r = gather_emul(ctx, dev, n, args.steps, args.warmup)
    elif op == "gather_emul_place":
        r = gather_emul_place(ctx, dev, n, args.steps, args.warmup)
    else:
        raise SystemExit(f"unknown op {op}")
    r["op"] = op
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
