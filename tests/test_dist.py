"""World-size-2 gloo rehearsal of the multi-GPU path on CPU: each rank
computes the records of its contiguous shard (oracle stands in for the GPU
kernel here), the flow hashes are all-gathered, and the result must equal
the single-process batch bit for bit."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, load_golden


def _worker(rank, world, port, name, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from oracle.oracle import Oracle, make_opts
    from pptk_amd.records import F_PARSED
    from pptk_amd.shard import allgather_flow_hash, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = load_golden(name)
        n = len(z["off"])
        first, cnt = shard_range(n, world, rank)
        b4, b6, hs = (int(x) for x in z["iphash"])
        recs = Oracle().rx_batch(z["buf"], z["off"][first:first + cnt], z["len"][first:first + cnt],
                                 opts=make_opts(z["key"].tobytes(), b4, b6, hs))
        h = np.where(recs["flags"] & F_PARSED, recs["flow_hash"], 0).view(np.int64)
        # pad to equal shard size for all_gather_into_tensor
        per = (n + world - 1) // world
        loc = torch.zeros(per, dtype=torch.int64)
        loc[:cnt] = torch.from_numpy(h.copy())
        out = allgather_flow_hash(loc)
        if rank == 0:
            parts = [out[r * per:r * per + shard_range(n, world, r)[1]] for r in range(world)]
            q.put(torch.cat(parts).numpy().view(np.uint64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["c1500", "cmix", "edge"])
def test_sharded_allgather_equals_single(name):
    from pptk_amd.records import F_PARSED, as_records
    world, port = 2, 29500 + (os.getpid() % 1000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = as_records(load_golden(name)["recs"])
    assert np.array_equal(got, np.where(want["flags"] & F_PARSED, want["flow_hash"], 0))


@pytest.mark.parametrize("n,world", [(10, 3), (16, 4), (1, 2), (0, 2), (134217728, 8)])
def test_shard_range_partitions(n, world):
    from pptk_amd.shard import shard_range
    got = [shard_range(n, world, r) for r in range(world)]
    assert got[0][0] == 0
    for (f0, c0), (f1, _) in zip(got, got[1:]):
        assert f0 + c0 == f1
    assert sum(c for _, c in got) == n


def _bench_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cpu")
        bench.barrier(world, dev)
        mx = bench.max_over_ranks(float(rank + 1), world, dev)
        sm = bench.sum_over_ranks(float(rank + 1), world, dev)
        g = bench.gather_bench(1024, world, dev, 3)
        if rank == 0:
            q.put((mx, sm, g))
    finally:
        dist.destroy_process_group()


def test_bench_multi_rank_helpers():
    """bench.py's N > 1 bookkeeping (barrier, max/sum over ranks, the
    all-gather timing and its bus-bandwidth arithmetic) on gloo, world 2."""
    world, port = 2, 30600 + (os.getpid() % 1000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    mx, sm, g = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert mx == 2.0 and sm == 3.0
    assert g["bytes_per_rank"] == 1024 * 8 and g["ms"] > 0
    assert abs(g["busbw_gbs"] - g["algbw_gbs"] / 2) <= 0.1 + 1e-9
