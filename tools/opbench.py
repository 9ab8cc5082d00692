"""BENCH TOOLING: one batch operation alone, for rocprofv3 PMC passes.

    python tools/opbench.py OP [--steps K] [--warmup W]

OP: tx (pptk_tx_cksum_device on C1500), tx_cmix, rewrite (pptk_tx_rewrite_device
on C64), mss (pptk_tcp_mss_clamp_device, 16 M SYNs), permit
(pptk_rx_permit_device over 16 M C64 records), binned (CMIX through
pptk_rx_batch_device_mixed), allgather (a one-rank communicator's in-place
pptk_rx_allgather_hash after every C1500 launch).  Uses bench.py's own
measurement functions; prints one JSON line with the timing and
`changed_bytes_per_launch` (the bytes the op must write), the denominator
of the write-amplification ratio WRITE_SIZE / changed bytes."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

N = bench.N_PER_GPU


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("op")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    import torch
    from pptk_amd.rx import RxContext
    from tools.synth import make_batch
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
    elif op == "binned":
        b = make_batch("cmix", n, dev)
        r = bench.binned_bench(ctx, b, n, dev, args.steps, args.warmup)
        r["changed_bytes_per_launch"] = 64 * n
    elif op == "allgather":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        os.environ["PPTK_BENCH_FORCE_DIST"] = "1"
        import torch.distributed as dist
        from pptk_amd.shard import GatherBuffer, join
        dist.init_process_group("gloo", rank=0, world_size=1)
        join(ctx, 1, 0)
        gbs = [GatherBuffer(n, 1, 0, dev) for _ in range(2)]
        res = bench.run_config("c1500", n, ctx, dev, 1, 0, args.steps, args.warmup, gbs, False,
                               settle=0.3, first=0)
        r = {"kernel_ms": round(res["kernel_ms"], 4), "mpkts": round(res["mpkts"], 1),
             "changed_bytes_per_launch": 64 * n + 8 * n}
        dist.destroy_process_group()
    else:
        raise SystemExit(f"unknown op {op}")
    r["op"] = op
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
