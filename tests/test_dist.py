"""World-size-2 gloo rehearsal of the multi-GPU path on CPU: each rank
takes its shard by the C-ABI's equal-shard policy (pptk_rx_shard_range),
computes its records (the oracle stands in for the GPU kernel here), the
flow hashes are all-gathered in place into the padded layout the RCCL path
uses (gloo's all_gather_into_tensor stands in for pptk_rx_allgather_hash),
and the result must equal the single-process batch bit for bit."""
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
    from pptk_amd.shard import shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = load_golden(name)
        n = len(z["off"])
        first, cnt, per = shard_range(n, world, rank)
        b4, b6, hs = (int(x) for x in z["iphash"])
        recs = Oracle().rx_batch(z["buf"], z["off"][first:first + cnt], z["len"][first:first + cnt],
                                 opts=make_opts(z["key"].tobytes(), b4, b6, hs))
        h = np.where(recs["flags"] & F_PARSED, recs["flow_hash"], 0).view(np.int64)
        # the rank's slice of the gather buffer (GatherBuffer.local), padded
        out = torch.zeros(world * per, dtype=torch.int64)
        loc = out[rank * per:(rank + 1) * per].clone()
        loc[:cnt] = torch.from_numpy(h.copy())
        dist.all_gather_into_tensor(out, loc)
        if rank == 0:
            q.put(out[:n].numpy().view(np.uint64))
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


@pytest.mark.parametrize("n,world", [(10, 3), (16, 4), (1, 2), (0, 2), (2, 4), (7, 8),
                                     (134217728, 8), (134217727, 8)])
def test_shard_range_partitions(n, world):
    """pptk_rx_shard_range: contiguous, covering, equal per-rank gather size,
    and rank r's frames sit at gathered index r * per (global order)."""
    from pptk_amd.shard import shard_range
    got = [shard_range(n, world, r) for r in range(world)]
    per = got[0][2]
    assert per == (n + world - 1) // world
    assert got[0][0] == 0
    for (f0, c0, p0), (f1, _, _) in zip(got, got[1:]):
        assert f0 + c0 == f1 and p0 == per
    assert sum(c for _, c, _ in got) == n
    for r, (f, c, _) in enumerate(got):
        assert c <= per and (c == 0 or f == r * per)


def test_shard_range_rejects_bad_rank():
    from pptk_amd.shard import shard_range
    assert shard_range(10, 0, 0) == (0, 0, 0)
    assert shard_range(10, 2, 2) == (0, 0, 0)
    assert shard_range(10, 2, -1) == (0, 0, 0)


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
        g = bench.gather_bw(1024, world, 1e-3)
        pr = bench.per_rank(float(rank) + 0.5, world)
        if rank == 0:
            q.put((mx, sm, g, pr))
    finally:
        dist.destroy_process_group()


def test_bench_multi_rank_helpers():
    """bench.py's N > 1 bookkeeping (barrier, max/sum over ranks on its gloo
    control plane, the all-gather bandwidth arithmetic) on gloo, world 2."""
    world, port = 2, 30600 + (os.getpid() % 1000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    mx, sm, g, pr = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert mx == 2.0 and sm == 3.0 and pr == [0.5, 1.5]
    alg, bus = g
    assert alg == round(1024 * 2 * 8 / 1e-3 / 1e9, 1) and abs(bus - alg / 2) <= 0.1


class _FakeCommCtx:
    """Stands in for RxContext's communicator calls (no GPU, no RCCL)."""

    def __init__(self):
        self.calls = []

    def comm_abort(self):
        self.calls.append("abort")

    def comm_destroy(self):
        self.calls.append("destroy")


def _join_worker(rank, world, port, fail_ranks, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def join_fn(ctx, ws, r):
            if r in fail_ranks:
                raise RuntimeError("pptk_rx_comm_create: -110")
        ctx = _FakeCommCtx()
        err = bench.join_all(ctx, world, rank, join_fn)
        q.put((rank, err, ctx.calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_ranks", [(), (1,), (0, 1)])
def test_bench_joins_all_ranks_or_none(fail_ranks):
    """bench.join_all on gloo, world 2: when one rank cannot create its RCCL
    communicator every rank learns it, the ranks that did join abort and
    drop theirs, and the run goes on without the collective; the line then
    names the error and fails bench.validate_line (non-zero exit)."""
    import bench
    world, port = 2, 31700 + (os.getpid() % 1000) + 10 * len(fail_ranks)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_join_worker, args=(r, world, port, fail_ranks, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (e, c)) for r, e, c in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(world):
        err, calls = got[r]
        if not fail_ranks:
            assert err is None and calls == []
        elif r in fail_ranks:
            assert "-110" in err and calls == []
        else:
            assert "could not join" in err and calls == ["abort", "destroy"]
    if fail_ranks:
        full = {"n_gpus": world, "allgather": {"error": got[fail_ranks[0]][0]},
                "per_rank_kernel_ms": [4.0] * world, "config": {"workload": "C1500: x"},
                "roofline": {}}
        line = bench.compact_line(full, detail_path=None)
        assert line["allgather"] == {"error": got[fail_ranks[0]][0]}
        probs = bench.validate_line(line)
        assert len(probs) == 1 and probs[0].startswith("all-gather failed")


def test_bench_launches_ranks_itself(tmp_path, monkeypatch):
    """`python bench.py --gpus N` outside a launcher starts N ranks through
    torch.distributed.run (the command it builds, not run here)."""
    import subprocess
    import sys
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 0
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    monkeypatch.setattr(subprocess, "call", fake_call)
    with pytest.raises(SystemExit) as e:
        bench.launch_ranks(["--gpus", "4", "--steps", "3"], 4)
    assert e.value.code == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    monkeypatch.setenv("LOCAL_RANK", "0")
    bench.launch_ranks(["--gpus", "4"], 4)          # under a launcher: no-op
    bench.launch_ranks([], 1)


def _dist_line(ws):
    return {"n_gpus": ws, "value": 1.0, "value_no_gather": 1.1,
            "config": {"rccl_ranks": ws}, "per_rank_kernel_ms": [4.1] * ws,
            "allgather": {"ms": 0.2, "algbw_gbs": 600.0, "busbw_gbs": 525.0, "rccl_ranks": ws,
                          "overlap_loss": 0.05,
                          "gathered_check": {"own_slice_equals_records": True,
                                             "sampled_frames": 4096 * ws,
                                             "sampled_frames_per_rank": 4096,
                                             "sampled_mismatches": 0}}}


def test_bench_validates_multi_gpu_line():
    """bench.validate_line: the N > 1 fields the driver's 8-GPU line must
    carry (communicator spans every rank, gathered array checked on >= 4096
    frames per rank with no mismatch, every rank's kernel time), and what it
    flags when they are missing or wrong."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    for ws in (1, 2, 8):
        assert bench.validate_line(_dist_line(ws)) == []
    assert bench.validate_line({"n_gpus": 1, "per_rank_kernel_ms": [4.0]}) == []
    bad = _dist_line(8)
    bad["allgather"]["rccl_ranks"] = 1
    bad["config"]["rccl_ranks"] = 1
    assert len(bench.validate_line(bad)) == 2
    bad = _dist_line(8)
    bad["allgather"]["gathered_check"]["sampled_frames_per_rank"] = 64
    bad["allgather"]["gathered_check"]["sampled_mismatches"] = 3
    assert len(bench.validate_line(bad)) == 2
    bad = _dist_line(2)
    del bad["allgather"]
    assert bench.validate_line(bad) == ["N > 1 without an all-gather"]
    bad = _dist_line(4)
    bad["per_rank_kernel_ms"] = [4.0]
    assert bench.validate_line(bad) == ["per_rank_kernel_ms does not list every rank"]


def test_committed_forced_dist_line_passes():
    """The one-rank RCCL bench lines committed under profiles/ (rounds 4 and
    5, PPTK_BENCH_FORCE_DIST=1 on one MI355X; round 5's in the compact line
    format) carry every N > 1 field and pass bench.validate_line."""
    import glob
    import json
    import sys
    sys.path.insert(0, ROOT)
    import bench
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r04", "dist1", "bench_dist1*.json"))
                   + glob.glob(os.path.join(ROOT, "profiles", "r05", "*", "bench_dist1*.json")))
    if not files:
        pytest.skip("no round-4 forced one-rank line committed yet")
    for f in files:
        with open(f) as fh:
            line = json.loads([ln for ln in fh.read().splitlines() if ln.startswith("{")][-1])
        assert line["allgather"]["rccl_ranks"] == line["n_gpus"] == line["config"]["rccl_ranks"]
        assert bench.validate_line(line) == [], f
