"""The multi-GPU part of the C-ABI (include/pptk_rx.h "Multi-GPU",
pptk_amd/csrc/rx_comm.hip) on the GPU: RCCL communicators built through the
C-ABI (one process: pptk_rx_comm_uid + pptk_rx_comm_create, and
pptk_rx_comm_create_all), the kernel writing flow hashes into the rank's
slice of the gather buffer, and the in-place pptk_rx_allgather_hash, checked
against the reference-made golden flow hashes.  One GPU on the test box, so
the communicators have one rank; the N-rank layout is the same code with
per-rank offsets (tests/test_dist.py rehearses N = 2 on gloo)."""
import ctypes

import numpy as np
import pytest

from conftest import load_golden
from pptk_amd.records import as_records

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
EINVAL = 22


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _ctx(z):
    from pptk_amd.rx import RxContext
    b4, b6, hs = (int(x) for x in z["iphash"])
    return RxContext(0, z["key"].tobytes(), b4, b6, hs, max_frame=65535)


def _gather_set(ctx, z, dev, world=1, rank=0):
    from pptk_amd.shard import GatherBuffer
    n = len(z["off"])
    gb = GatherBuffer(n, world, rank, dev)
    frames = torch.from_numpy(z["buf"]).to(dev)
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    f, c = gb.first, gb.count
    recs = ctx.batch_device(frames, c, off=off[f:f + c], lens=lens[f:f + c],
                            max_len=int(z["len"].max()), hash_out=gb.local[:c])
    got = gb.gather(ctx)
    torch.cuda.synchronize()
    return got.cpu().numpy().view(np.uint64), recs.cpu().numpy().reshape(-1)


@pytest.mark.parametrize("name", ["edge", "fuzz", "cmix", "c1500"])
def test_comm_create_one_rank_allgather_equals_golden(dev, name):
    from pptk_amd.rx import comm_uid
    z = load_golden(name)
    ctx = _ctx(z)
    ctx.comm_create(1, 0, comm_uid())
    assert ctx.comm_info() == (1, 0)
    got, recs = _gather_set(ctx, z, dev)
    want = as_records(z["recs"])["flow_hash"]
    assert np.array_equal(got, want)
    assert np.array_equal(as_records(recs)["flow_hash"], want)
    ctx.comm_destroy()
    assert ctx.comm_info() is None
    ctx.close()


def test_comm_create_all_one_gpu(dev):
    from pptk_amd.rx import comm_create_all
    z = load_golden("cmix")
    ctx = _ctx(z)
    comm_create_all([ctx])
    assert ctx.comm_info() == (1, 0)
    got, _ = _gather_set(ctx, z, dev)
    assert np.array_equal(got, as_records(z["recs"])["flow_hash"])
    ctx.close()                                   # destroys the communicator too


def test_comm_repeated_gathers_and_reuse(dev):
    """Many batches and gathers on one communicator, then destroy and a new
    communicator on the same context."""
    from pptk_amd.rx import comm_uid
    z = load_golden("edge")
    ctx = _ctx(z)
    want = as_records(z["recs"])["flow_hash"]
    for _ in range(2):
        ctx.comm_create(1, 0, comm_uid())
        for _ in range(5):
            got, _ = _gather_set(ctx, z, dev)
            assert np.array_equal(got, want)
        ctx.comm_destroy()
    ctx.close()


def test_comm_contract_errors(dev):
    from pptk_amd.rx import comm_create_all, comm_uid
    z = load_golden("edge")
    ctx = _ctx(z)
    h = torch.zeros(8, dtype=torch.int64, device=dev)
    with pytest.raises(OSError) as e:                       # no communicator yet
        ctx.allgather_hash(h, 8, h)
    assert e.value.errno == EINVAL
    uid = comm_uid()
    for nr, r in ((0, 0), (1, 1), (2, -1)):
        with pytest.raises(OSError) as e:
            ctx.comm_create(nr, r, uid)
        assert e.value.errno == EINVAL
    ctx.comm_create(1, 0, uid)
    with pytest.raises(OSError) as e:                       # one per context
        ctx.comm_create(1, 0, comm_uid())
    assert e.value.errno == EINVAL
    with pytest.raises(OSError) as e:
        comm_create_all([ctx])                              # already has one
    assert e.value.errno == EINVAL
    with pytest.raises(OSError) as e:                       # null buffers
        ctx.allgather_hash(None, 8, h)
    assert e.value.errno == EINVAL
    ctx.allgather_hash(None, 0, h)                          # n == 0: nothing to do
    ctx.comm_destroy()
    ctx.comm_destroy()                                      # idempotent
    other = _ctx(z)
    with pytest.raises(OSError) as e:                       # two ranks on one GPU
        comm_create_all([ctx, other])
    assert e.value.errno == EINVAL
    other.close()
    ctx.close()


def test_entry_points_restore_callers_device(dev):
    """An entry point leaves the calling thread on its current device (with
    one GPU on the box this checks the restore path runs cleanly; the
    device switch itself needs two GPUs)."""
    from pptk_amd.rx import lib
    hip = ctypes.CDLL("libamdhip64.so")
    cur = ctypes.c_int(-1)
    z = load_golden("edge")
    ctx = _ctx(z)
    frames = torch.from_numpy(z["buf"]).to(dev)
    ctx.batch_device(frames, 4, off=torch.from_numpy(z["off"][:4].view(np.int64)).to(dev),
                     lens=torch.from_numpy(z["len"][:4].view(np.int16)).to(dev), max_len=1500)
    torch.cuda.synchronize()
    assert hip.hipGetDevice(ctypes.byref(cur)) == 0 and cur.value == 0
    assert lib().pptk_rx_device_count() >= 1
    ctx.close()


@pytest.mark.parametrize("frames,scaling", [(1 << 20, "weak"), ((1 << 20) + 77, "strong")])
def test_bench_one_rank_rccl_path(tmp_path, frames, scaling):
    """bench.py's multi-GPU path end to end on one GPU (PPTK_BENCH_FORCE_DIST:
    a one-rank RCCL communicator through the C-ABI, the gloo control plane,
    the double-buffered in-place gather on a second stream, the gathered-hash
    parity check), small batch; strong scaling with a frame count that is not
    a multiple of 64."""
    import json
    import os
    import subprocess
    import sys
    from conftest import ROOT
    env = dict(os.environ, PPTK_BENCH_FORCE_DIST="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(29600 + os.getpid() % 300))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--frames", str(frames),
                          "--scaling", scaling, "--steps", "3", "--warmup", "1", "--no-secondary",
                          "--no-cpu", "--no-rec32", "--no-membench", "--settle", "0.1"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["config"]["rccl_ranks"] == 1
    assert line["config"]["global_frames"] == frames
    g = line["allgather"]
    assert g["rccl_ranks"] == 1 and g["bytes_per_rank"] == frames * 8
    assert g["gathered_check"]["own_slice_equals_records"]
    assert g["gathered_check"]["sampled_mismatches"] == 0
    c = line["configs"]["c1500"]
    assert c["oracle_mismatches"] == 0 and c["verdicts_ok"] is True
    assert g["placement"]["alloc"] == "pptk_rx_gather_alloc"


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("name", ["fuzz", "cmix"])
def test_sharded_layout_n_ranks_one_gpu(dev, name, world):
    """The N-rank data path without the collective: `world` contexts on the
    one GPU each run their shard (pptk_rx_shard_range: equal shards, the
    last padded) with the kernel writing the flow hashes into their slice of
    ONE shared gather buffer -- the array an N-rank in-place all-gather
    leaves on every rank.  It must hold global frame i's hash at index i, the
    padding untouched, and every shard's records must equal the golden
    records of its frames."""
    from pptk_amd.shard import GatherBuffer
    z = load_golden(name)
    n = len(z["off"])
    frames = torch.from_numpy(z["buf"]).to(dev)
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    want = as_records(z["recs"])
    shared = None
    covered = 0
    for rank in range(world):
        ctx = _ctx(z)
        gb = GatherBuffer(n, world, rank, dev, out=shared)
        if shared is None:
            shared = gb.out
            shared.fill_(-1)
        f, c = gb.first, gb.count
        assert f == covered and gb.per * world >= n
        covered += c
        if c:
            recs = ctx.batch_device(frames, c, off=off[f:f + c], lens=lens[f:f + c],
                                    max_len=int(z["len"].max()), hash_out=gb.local[:c])
            torch.cuda.synchronize()
            got = recs.cpu().numpy().reshape(-1).view(want.dtype)
            assert np.array_equal(got, want[f:f + c])
        ctx.close()
    assert covered == n
    h = shared.cpu().numpy().view(np.uint64)
    assert np.array_equal(h[:n], want["flow_hash"])
    per = -(-n // world)
    pad = np.concatenate([h[r * per + max(0, min(per, n - r * per)):(r + 1) * per]
                          for r in range(world)])
    assert (pad == np.uint64(0xFFFFFFFFFFFFFFFF)).all()


ETIMEDOUT, ECANCELED = 110, 125


def test_comm_rank_never_joins_times_out_then_recovers(dev):
    """Failure containment (pptk_rx.h "Multi-GPU"): a 2-rank communicator
    whose rank 1 never joins.  pptk_rx_comm_create must give up with
    ETIMEDOUT within opts.comm_timeout_ms (plus RCCL's abort), leave the
    context without a communicator, and the same context must then build a
    1-rank communicator whose gather equals the golden flow hashes."""
    import time
    from pptk_amd.rx import RxContext, comm_uid
    z = load_golden("edge")
    b4, b6, hs = (int(x) for x in z["iphash"])
    ctx = RxContext(0, z["key"].tobytes(), b4, b6, hs, max_frame=65535, comm_timeout_ms=3000)
    t0 = time.monotonic()
    with pytest.raises(OSError) as e:
        ctx.comm_create(2, 0, comm_uid())
    took = time.monotonic() - t0
    assert e.value.errno == ETIMEDOUT, e.value
    assert 2.5 < took < 30, took
    assert ctx.comm_info() is None
    ctx.comm_create(1, 0, comm_uid())
    got, _ = _gather_set(ctx, z, dev)
    assert np.array_equal(got, as_records(z["recs"])["flow_hash"])
    assert ctx.comm_sync() == 0
    ctx.close()


def test_comm_sync_and_abort(dev):
    """pptk_rx_comm_sync after gathers returns 0 with the golden hashes in
    place; after pptk_rx_comm_abort every call on the communicator returns
    ECANCELED until it is destroyed, and a new one works."""
    from pptk_amd.rx import comm_uid
    z = load_golden("cmix")
    ctx = _ctx(z)
    want = as_records(z["recs"])["flow_hash"]
    ctx.comm_create(1, 0, comm_uid())
    s = torch.cuda.Stream(dev)
    n = len(z["off"])
    from pptk_amd.shard import GatherBuffer
    gb = GatherBuffer(n, 1, 0, dev)
    frames = torch.from_numpy(z["buf"]).to(dev)
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    with torch.cuda.stream(s):
        for _ in range(4):
            ctx.batch_device(frames, n, off=off, lens=lens, max_len=int(z["len"].max()),
                             hash_out=gb.local[:n], stream=s)
            gb.gather(ctx, stream=s)
    assert ctx.comm_sync(s, 10000) == 0
    assert np.array_equal(gb.out[:n].cpu().numpy().view(np.uint64), want)
    ctx.comm_abort()
    ctx.comm_abort()                                        # once is enough; no error
    with pytest.raises(OSError) as e:
        gb.gather(ctx, stream=s)
    assert e.value.errno == ECANCELED
    assert ctx.comm_info() == (1, 0)
    ctx.comm_destroy()
    assert ctx.comm_sync(s, 1000) == 0                      # plain bounded stream wait
    ctx.comm_create(1, 0, comm_uid())
    got, _ = _gather_set(ctx, z, dev)
    assert np.array_equal(got, want)
    ctx.close()


def _timed_create(ctx, nranks, rank, uid):
    import time
    t0 = time.monotonic()
    try:
        ctx.comm_create(nranks, rank, uid)
        rc = 0
    except OSError as e:
        rc = -e.errno
    return rc, time.monotonic() - t0


def test_comm_abort_during_create_cancels(dev):
    """pptk_rx_comm_abort from another thread while pptk_rx_comm_create is
    still waiting (a 2-rank communicator whose rank 1 never joins, 30 s
    deadline): the create returns ECANCELED well inside its deadline, the
    context is left without a communicator, and then builds a 1-rank one
    whose gather equals the golden flow hashes (reference model: the queue
    threads of ldp/ldprecvmt.c:174-182 share nothing)."""
    import threading
    import time
    from pptk_amd.rx import RxContext, comm_uid
    z = load_golden("edge")
    b4, b6, hs = (int(x) for x in z["iphash"])
    ctx = RxContext(0, z["key"].tobytes(), b4, b6, hs, max_frame=65535, comm_timeout_ms=30000)
    res = {}
    th = threading.Thread(target=lambda: res.update(r=_timed_create(ctx, 2, 0, comm_uid())))
    th.start()
    time.sleep(1.0)
    ctx.comm_abort()
    th.join(20)
    assert not th.is_alive()
    rc, took = res["r"]
    assert rc == -ECANCELED, rc
    assert took < 10, took
    assert ctx.comm_info() is None
    ctx.comm_create(1, 0, comm_uid())
    got, _ = _gather_set(ctx, z, dev)
    assert np.array_equal(got, as_records(z["recs"])["flow_hash"])
    assert ctx.comm_sync() == 0
    ctx.close()


def test_comm_pending_abort(dev):
    """An abort that reaches a context before its pptk_rx_comm_create (a
    sibling failed first) is kept: that create returns ECANCELED at once
    instead of waiting for ranks that will never come; the next create
    works.  comm_destroy drops a pending abort."""
    from pptk_amd.rx import comm_uid
    z = load_golden("cmix")
    ctx = _ctx(z)
    ctx.comm_abort()
    ctx.comm_abort()                                        # still one pending abort
    rc, took = _timed_create(ctx, 2, 0, comm_uid())
    assert rc == -ECANCELED and took < 1.0, (rc, took)
    assert ctx.comm_info() is None
    ctx.comm_abort()
    ctx.comm_destroy()                                      # drops it
    ctx.comm_create(1, 0, comm_uid())
    got, _ = _gather_set(ctx, z, dev)
    assert np.array_equal(got, as_records(z["recs"])["flow_hash"])
    ctx.close()


def test_comm_warmup_gather_stall_is_bounded(dev, monkeypatch):
    """A peer that inits but never issues its part of the creation's
    warm-up gather (staged on one GPU by PPTK_RX_COMM_TEST_WARMUP_STALL_MS,
    which holds the warm-up stream behind a 4 s spin): the create returns
    ETIMEDOUT at its 1.5 s deadline instead of waiting; the helper aborts
    the new communicator, so once the stall is over the queued gather
    returns and a device-wide synchronize completes (nothing of the
    abandoned creation is left running: RCCL's own abort waits for that
    stream, so the wait below is the stall, not a hang); the same context
    then builds a communicator that gathers the golden hashes."""
    import time
    from conftest import HOOKS_LIB
    from pptk_amd.rx import RxContext, comm_uid
    z = load_golden("fuzz")
    b4, b6, hs = (int(x) for x in z["iphash"])
    # (the knob exists only in the test build of the library)
    ctx = RxContext(0, z["key"].tobytes(), b4, b6, hs, max_frame=65535, comm_timeout_ms=1500,
                    lib_path=HOOKS_LIB)
    monkeypatch.setenv("PPTK_RX_COMM_TEST_WARMUP_STALL_MS", "4000")
    rc, took = _timed_create(ctx, 1, 0, comm_uid(lib_path=HOOKS_LIB))
    assert rc == -ETIMEDOUT and 1.2 < took < 3.5, (rc, took)
    monkeypatch.delenv("PPTK_RX_COMM_TEST_WARMUP_STALL_MS")
    t0 = time.monotonic()
    torch.cuda.synchronize()
    assert time.monotonic() - t0 < 15
    time.sleep(1.0)          # (the helper frees its buffers after the drain)
    ctx.comm_create(1, 0, comm_uid(lib_path=HOOKS_LIB))
    got, _ = _gather_set(ctx, z, dev)
    assert np.array_equal(got, as_records(z["recs"])["flow_hash"])
    ctx.close()


@pytest.mark.parametrize("name", ["cmix", "c1500"])
def test_placed_gather_buffers_gather_golden(dev, name):
    """pptk_rx_gather_alloc: the library places this rank's two gather
    buffers by running the batch into each candidate region (as the
    multi-GPU bench and examples/rx_multigpu.c now take them); on a one-rank
    communicator the kernel writes the rank's hashes into each buffer's
    slice and the in-place all-gather leaves the golden flow hashes, in both
    buffers; the padding past the frames stays zero; the report is
    consistent; the memory comes back when the buffers go."""
    import gc
    from pptk_amd.rx import comm_uid, shard_range
    from pptk_amd.shard import GatherBuffer
    z = load_golden(name)
    ctx = _ctx(z)
    ctx.comm_create(1, 0, comm_uid())
    n = len(z["off"])
    frames = torch.from_numpy(z["buf"]).to(dev)
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    kw = dict(off=off, lens=lens, max_len=int(z["len"].max()))
    n_total = n + 5                       # padded shard: 5 slots no frame fills
    first, count, per = shard_range(n_total, 1, 0)
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info(dev)
    g = ctx.gather_alloc(frames, n, per, 1, 0, cands=3, reps=2, **kw)
    rep = g.report
    assert rep["candidates"] == 3 and 0 <= rep["chosen"] < 3 and rep["chosen_ms"] > 0
    assert rep["freed_bytes"] > 0
    want = as_records(z["recs"])["flow_hash"]
    for k in range(2):
        gb = GatherBuffer(n_total, 1, 0, dev, out=g.out[k])
        assert int(gb.out.abs().sum().item()) == 0          # zeroed
        recs = ctx.batch_device(frames, n, hash_out=gb.local[:n], **kw)
        got = gb.gather(ctx).cpu().numpy().view(np.uint64)
        torch.cuda.synchronize()
        assert np.array_equal(got[:n], want), k
        assert (got[n:] == 0).all()
        assert np.array_equal(as_records(recs.cpu().numpy().reshape(-1))["flow_hash"], want)
    del g, gb
    gc.collect()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info(dev)
    assert free1 >= free0 - (64 << 20)
    ctx.close()


def test_gather_alloc_rejects(dev):
    """Bad gather specs: -EINVAL before anything is allocated."""
    z = load_golden("edge")
    ctx = _ctx(z)
    frames = torch.zeros(4096, dtype=torch.uint8, device=dev)
    for args in ((10, 0, 0), (10, 2, 2), (10, 1, -1), (0, 1, 0), (5, 1, 0)):   # (per, nranks, rank)
        with pytest.raises(OSError) as e:
            ctx.gather_alloc(frames, 10, *args, stride=64, fixed_len=64)
        assert e.value.errno == EINVAL, args
    ctx.close()


def test_gather_alloc_n_rank_slice_probe(dev):
    """pptk_rx_gather_alloc for rank 2 of 4 on one GPU (no collective: the
    probe is rank-local): every probe launch lands the bytes the 4-rank
    gather would -- device copies into the other three slices beside the
    batch -- and the kept buffers come back zeroed; the kernel then writes
    the golden hashes into rank 2's slice of either buffer, and nothing
    else changes."""
    from pptk_amd.rx import shard_range
    from pptk_amd.shard import GatherBuffer
    z = load_golden("fuzz")
    ctx = _ctx(z)
    n = len(z["off"])
    frames = torch.from_numpy(z["buf"]).to(dev)
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    kw = dict(off=off, lens=lens, max_len=int(z["len"].max()))
    n_total = 4 * n
    first, count, per = shard_range(n_total, 4, 2)
    assert count == n
    g = ctx.gather_alloc(frames, n, per, 4, 2, cands=2, reps=1, **kw)
    assert g.report["candidates"] == 2 and len(g.report["candidate_ms"]) == 2
    want = as_records(z["recs"])["flow_hash"]
    for k in range(2):
        gb = GatherBuffer(n_total, 4, 2, dev, out=g.out[k])
        assert int(gb.out.abs().sum().item()) == 0
        ctx.batch_device(frames, n, hash_out=gb.local[:n], **kw)
        torch.cuda.synchronize()
        got = gb.out.cpu().numpy().view(np.uint64)
        assert np.array_equal(got[2 * per:2 * per + n], want), k
        assert (got[:2 * per] == 0).all() and (got[2 * per + n:] == 0).all()
    ctx.close()


def _rccl_log(split_cus):
    """Child process: one-rank communicator on a context split (or not), with
    RCCL's INFO log on; the log."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import torch; torch.cuda.init()\n"   # (torch's HIP runtime first, as in the tests)
        "from pptk_amd.rx import RxContext, comm_uid\n"
        "ctx = RxContext(0, bytes(range(1, 17)))\n"
        "if %d: ctx.stream_split(%d)\n"
        "ctx.comm_create(1, 0, comm_uid())\n"
        "ctx.close()\n"
        "print('child ok')\n") % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                  split_cus, split_cus)
    env = dict(os.environ, NCCL_DEBUG="INFO")
    env.pop("NCCL_MAX_NCHANNELS", None)
    env.pop("NCCL_MAX_CTAS", None)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         timeout=120, env=env)
    assert out.returncode == 0 and "child ok" in out.stdout, out.stderr[-2000:]
    return out.stdout + out.stderr


def test_split_streams_owned_by_context_and_channel_cap(dev):
    """pptk_rx_stream_split before the communicator: the context owns the two
    streams (a second split to the same count returns them; a split to
    another count once a communicator exists is EBUSY), the gather runs on
    the collective stream beside the batches' stream bit-exact,
    pptk_rx_stream_destroy of either stream before the context is EBUSY --
    the 'wrong' destroy order that hung in round 5 is refused, not queued --
    and the context's teardown (communicator, then its streams) returns
    promptly; afterwards the destroy of the retired handle is a no-op 0."""
    import time
    from pptk_amd.rx import comm_uid
    z = load_golden("cmix")
    ctx = _ctx(z)
    L = ctx._L
    rx, coll = ctx.stream_split(32)
    rx2, coll2 = ctx.stream_split(32)
    assert (rx2.cuda_stream, coll2.cuda_stream) == (rx.cuda_stream, coll.cuda_stream)
    ctx.comm_create(1, 0, comm_uid())
    with pytest.raises(OSError) as e:                   # the cap is fixed now
        ctx.stream_split(64)
    assert e.value.errno == 16
    ctx.stream_join()                                   # grids on the whole chip: allowed
    rx3, coll3 = ctx.stream_split(32)                   # the same pair again
    assert coll3.cuda_stream == coll.cuda_stream
    from pptk_amd.shard import GatherBuffer
    n = len(z["off"])
    gb = GatherBuffer(n, 1, 0, dev)
    frames = torch.from_numpy(z["buf"]).to(dev)
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    torch.cuda.synchronize()
    ctx.batch_device(frames, n, off=off, lens=lens, max_len=int(z["len"].max()),
                     hash_out=gb.local[:n], stream=rx)
    ev = torch.cuda.Event()
    ev.record(rx)
    coll.wait_event(ev)
    ctx.allgather_hash(gb.local, gb.per, gb.out, stream=coll)
    assert ctx.comm_sync(coll) == 0
    got = gb.out.cpu().numpy().view(np.uint64)[:n]
    assert np.array_equal(got, as_records(z["recs"])["flow_hash"])
    for s in (coll, rx):                                # the context's: refused
        assert L.pptk_rx_stream_destroy(ctypes.c_void_p(s.cuda_stream)) == -16
    handles = (coll.cuda_stream, rx.cuda_stream)
    t0 = time.monotonic()
    ctx.close()                                         # communicator, then the streams
    assert time.monotonic() - t0 < 30
    for h in handles:                                   # destroyed by the context
        assert L.pptk_rx_stream_destroy(ctypes.c_void_p(h)) == 0
    # without a communicator a split may change its CU count (new pair)
    c2 = _ctx(z)
    c2.stream_split(32)
    _, b = c2.stream_split(64)
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ctypes.c_uint32 * (ncu // 32))()
    assert hip.hipExtStreamGetCUMask(ctypes.c_void_p(b.cuda_stream), len(words), words) == 0
    assert sum(bin(w).count("1") for w in words) == 64
    c2.close()


def test_split_caps_rccl_channels(dev):
    """RCCL's own log: a communicator created on a split context reports the
    library's cap ("Comm config Max CTAs set to 32": ncclConfig_t.maxCTAs,
    which RCCL applies to the blocks of each collective), and one created
    without a split reports none.  (The ring set RCCL builds at init stays
    at its own count either way -- 128 channels here; only
    NCCL_MAX_NCHANNELS shrinks that, profiles/r06/rccl_cap/.  How many blocks
    a gather launches shows only with more than one rank: a one-rank gather
    launches none.)"""
    capped = _rccl_log(32)
    free = _rccl_log(0)
    assert "Comm config Max CTAs set to 32" in capped
    assert "Comm config Max CTAs" not in free
