"""Parity of the HIP rx transform (through the C-ABI) with the golden
fixtures produced by the reference's own functions (tests/golden/), bit for
bit, in every addressing mode and kernel variant.  Needs an MI355X."""
import numpy as np
import pytest

from conftest import GOLDEN_SETS, load_golden
from pptk_amd.records import F_PARSED, REC32_DTYPE, as_records, diff_records, to_rec32

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _ctx(z, bucket=True, max_frame=65535):
    from pptk_amd.rx import RxContext
    b4, b6, hs = (int(x) for x in z["iphash"])
    if not bucket:
        b4 = b6 = 0
    return RxContext(0, z["key"].tobytes(), b4, b6, hs, max_frame=max_frame)


def _upload(buf, dev, shift=0):
    big = torch.zeros(buf.size + shift + 64, dtype=torch.uint8, device=dev)
    big[shift:shift + buf.size] = torch.from_numpy(buf).to(dev)
    return big, big[shift:]


def _run(ctx, z, dev, shift=0, perm=False, hash_out=False, max_len=None,
         stride=None, compact=False):
    buf, off, lens = z["buf"], z["off"], z["len"]
    n = len(off)
    _keep, frames = _upload(buf, dev, shift)
    lens_t = torch.from_numpy(lens.view(np.int16)).to(dev)
    kw = {}
    if stride is None:
        kw["off"] = torch.from_numpy(off.view(np.int64)).to(dev)
        kw["lens"] = lens_t
        kw["max_len"] = int(lens.max()) if max_len is None else max_len
    else:
        assert np.all(off == np.arange(n, dtype=np.uint64) * stride)
        kw["stride"] = stride
        kw["fixed_len"] = int(lens[0])
    p = ctx.bin_device(lens_t, n) if perm else None
    h = torch.full((n,), -1, dtype=torch.int64, device=dev) if hash_out else None
    recs = ctx.batch_device(frames, n, perm=p, hash_out=h, compact=compact, **kw)
    torch.cuda.synchronize()
    out = recs.cpu().numpy().reshape(-1)
    if hash_out:
        return out, h.cpu().numpy().view(np.uint64), (None if p is None else p.cpu().numpy())
    return out


@pytest.mark.parametrize("name", GOLDEN_SETS)
@pytest.mark.parametrize("shift", [0, 1, 6, 15])
def test_offsets_mode(name, shift, dev):
    z = load_golden(name)
    ctx = _ctx(z)
    got = _run(ctx, z, dev, shift=shift)
    d = diff_records(got, z["recs"])
    assert not d, d


@pytest.mark.parametrize("name", GOLDEN_SETS)
@pytest.mark.parametrize("max_len", [1, 40, 100, 200, 400, 900, 1500, 65535])
def test_every_variant(name, max_len, dev):
    """max_len is a tuning hint: a wrong hint selects another kernel variant
    (T4S1 ... T64S2) but must never change a result."""
    z = load_golden(name)
    got = _run(_ctx(z), z, dev, shift=3, max_len=max_len)
    d = diff_records(got, z["recs"])
    assert not d, d


@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_every_forced_variant(name, dev):
    """pptk_rx_set_tuning: every kernel variant, offsets and fixed-stride
    layouts, aligned and misaligned buffers -- identical records."""
    from pptk_amd.rx import lib
    z = load_golden(name)
    ctx = _ctx(z)
    for v in range(lib().pptk_rx_variant_count()):
        ctx.set_tuning(v, (v % 4) | (256 if v % 2 else 0))   # 256: blocked tile order
        for shift in (0, 5):
            got = _run(ctx, z, dev, shift=shift)
            d = diff_records(got, z["recs"])
            assert not d, f"variant {v} shift {shift}: {d}"
        if name in ("c64", "c1500"):
            got = _run(ctx, z, dev, shift=3, stride=64 if name == "c64" else 1500)
            d = diff_records(got, z["recs"])
            assert not d, f"variant {v} fixed stride: {d}"


@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_compact_records(name, dev):
    """d_recs32: the 32-byte record is the projection of the full one, in
    every variant, identity and binned order, offsets and fixed stride."""
    from pptk_amd.rx import lib
    z = load_golden(name)
    want = to_rec32(z["recs"])
    ctx = _ctx(z)
    for v in list(range(lib().pptk_rx_variant_count())) + [-1]:
        ctx.set_tuning(v, -1 if v < 0 else (v % 4) | 32)
        for shift, perm in ((0, False), (9, False), (3, True)):
            got = _run(ctx, z, dev, shift=shift, perm=perm, compact=True)
            d = diff_records(got, want, dtype=REC32_DTYPE)
            assert not d, f"variant {v} shift {shift} perm {perm}: {d}"
        if name in ("c64", "c1500"):
            got = _run(ctx, z, dev, shift=5, stride=64 if name == "c64" else 1500, compact=True)
            d = diff_records(got, want, dtype=REC32_DTYPE)
            assert not d, f"variant {v} fixed stride: {d}"


@pytest.mark.parametrize("name,stride", [("c64", 64), ("c1500", 1500)])
@pytest.mark.parametrize("shift", [0, 4, 5, 13])
def test_fixed_stride(name, stride, shift, dev):
    z = load_golden(name)
    got = _run(_ctx(z), z, dev, shift=shift, stride=stride)
    d = diff_records(got, z["recs"])
    assert not d, d


@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_binned_order_and_hash_out(name, dev):
    z = load_golden(name)
    got, h, perm = _run(_ctx(z), z, dev, perm=True, hash_out=True)
    d = diff_records(got, z["recs"])
    assert not d, d
    want = as_records(z["recs"])
    assert np.array_equal(h, np.where(want["flags"] & F_PARSED, want["flow_hash"], 0))
    # the permutation is a stable sort of indices by length group
    n = len(z["off"])
    assert np.array_equal(np.sort(perm), np.arange(n))
    assert np.array_equal(perm, np.argsort(_group_of(z["len"]), kind="stable"))


GROUP_MAX_LEN = [113, 1521]   # rx_internal.h kGroupMaxLen


def _group_of(lens):
    return np.searchsorted(np.array(GROUP_MAX_LEN), lens.astype(np.int64), side="left")


def _mixed_perm(lens, max_len=0):
    """The processing order pptk_rx_batch_device_mixed reports
    (include/pptk_rx.h): batch order when the max_len hint is at most 1521;
    otherwise binned (stable by length group) when the batch mixes frames
    over 1521 bytes with shorter ones, else batch order."""
    n = len(lens)
    if max_len and max_len <= GROUP_MAX_LEN[-1]:
        return np.arange(n)
    g = _group_of(lens)
    if (g == 2).any() and (g < 2).any():
        return np.argsort(g, kind="stable")
    return np.arange(n)


def _run_mixed(ctx, z, dev, shift=0, max_len=0):
    buf, off, lens = z["buf"], z["off"], z["len"]
    n = len(off)
    _keep, frames = _upload(buf, dev, shift)
    lens_t = torch.from_numpy(lens.view(np.int16)).to(dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    perm = torch.full((n,), -1, dtype=torch.int32, device=dev)
    h = torch.full((n,), -1, dtype=torch.int64, device=dev)
    recs = ctx.batch_device_mixed(frames, n, off_t, lens_t, hash_out=h, max_len=max_len,
                                  perm=perm)
    torch.cuda.synchronize()
    return (recs.cpu().numpy().reshape(-1), h.cpu().numpy().view(np.uint64),
            perm.cpu().numpy().view(np.uint32))


@pytest.mark.parametrize("name", GOLDEN_SETS)
@pytest.mark.parametrize("shift", [0, 7])
@pytest.mark.parametrize("max_len", [0, 100, 600, 1500])
def test_mixed_length_groups(name, shift, max_len, dev):
    """pptk_rx_batch_device_mixed: device binning + one launch per length
    group; max_len is a hint (a low one folds the upper groups into one
    launch) -- records, hashes and the order are exact either way."""
    z = load_golden(name)
    got, h, perm = _run_mixed(_ctx(z), z, dev, shift=shift, max_len=max_len)
    d = diff_records(got, z["recs"])
    assert not d, d
    want = as_records(z["recs"])
    assert np.array_equal(h, np.where(want["flags"] & F_PARSED, want["flow_hash"], 0))
    assert np.array_equal(perm, _mixed_perm(z["len"], max_len))


class _HipBuf:
    """A device buffer of exactly `nbytes` from its own hipMalloc (not the
    torch caching allocator, which keeps the bytes past a tensor mapped)."""

    def __init__(self, nbytes):
        import ctypes
        self._hip = ctypes.CDLL("libamdhip64.so")
        self._p = ctypes.c_void_p()
        assert self._hip.hipMalloc(ctypes.byref(self._p), ctypes.c_size_t(nbytes)) == 0
        self.nbytes = nbytes

    def data_ptr(self):
        return self._p.value

    def numpy(self, dtype):
        import ctypes
        out = np.empty(self.nbytes // np.dtype(dtype).itemsize, dtype)
        assert self._hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), self._p,
                                   ctypes.c_size_t(self.nbytes), 2) == 0   # D2H
        return out

    def free(self):
        self._hip.hipFree(self._p)


def test_mixed_empty_trailing_groups_perm_own_allocation(dev):
    """Advisor round 1: with max_len = 0 every length group is launched, and
    an empty trailing group's range starts at n -- one past the permutation.
    The permutation here is its own page-sized hipMalloc (1 024 entries) and
    no frame is longer than 1 009 bytes, so the last group (past 1 521 bytes)
    is empty: its launch must return before reading any descriptor."""
    import framegen
    from oracle.oracle import Oracle, make_opts
    rng = np.random.default_rng(1009)
    n = 1024
    sizes = rng.integers(60, 1010, n)
    frames = [_frame_of_len(framegen, rng, int(L)) for L in sizes]
    off = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
    buf = np.zeros(int(off[-1]) + len(frames[-1]) + 64, np.uint8)
    for i, f in enumerate(frames):
        buf[int(off[i]):int(off[i]) + len(f)] = np.frombuffer(f, np.uint8)
    lens = np.array([len(f) for f in frames], np.uint16)
    key = bytes(range(1, 17))
    want = Oracle().rx_batch(buf, off, lens, opts=make_opts(key, 24, 48, 1 << 12))
    z = {"key": np.frombuffer(key, np.uint8), "iphash": np.array([24, 48, 1 << 12])}
    ctx = _ctx(z)
    _keep, fr = _upload(buf, dev)
    perm = _HipBuf(4 * n)
    try:
        recs = ctx.batch_device_mixed(fr, n, torch.from_numpy(off.view(np.int64)).to(dev),
                                      torch.from_numpy(lens.view(np.int16)).to(dev),
                                      max_len=0, perm=perm)
        torch.cuda.synchronize()
        got_perm = perm.numpy(np.uint32)
    finally:
        torch.cuda.synchronize()
        perm.free()
    d = diff_records(recs.cpu().numpy().reshape(-1), want)
    assert not d, d
    assert np.array_equal(got_perm, _mixed_perm(lens))


def _frame_of_len(fg, rng, L):
    """A frame of exactly L bytes: IPv4/IPv6 TCP/UDP when it fits, else the
    truncated head of one (malformed)."""
    proto = 6 if rng.random() < 0.5 else 17
    v6 = rng.random() < 0.3
    need = 14 + (40 if v6 else 20) + (20 if proto == 6 else 8)
    if L >= need:
        return fg.frame_v6(rng, proto, L) if v6 else fg.frame_v4(rng, proto, L)
    return fg.frame_v4(rng, 17, 64)[:L]


def test_mixed_every_group_boundary(dev):
    """Frames at both sides of every group bound (and jumbo frames past the
    last one), in random order, through the grouped launches."""
    import framegen
    from oracle.oracle import Oracle, make_opts
    rng = np.random.default_rng(77)
    sizes = []
    for b in GROUP_MAX_LEN:
        sizes += [b - 1, b, b + 1]
    sizes += [14, 42, 60, 64, 2000, 4000, 9000, 9018]
    sizes = np.array(sizes * 40)
    rng.shuffle(sizes)
    frames = [_frame_of_len(framegen, rng, int(L)) for L in sizes]
    off = np.zeros(len(frames), np.uint64)
    pos = 0
    for i, f in enumerate(frames):
        off[i] = pos
        pos += len(f) + int(rng.integers(0, 5))
    buf = np.zeros(pos + 64, np.uint8)
    for i, f in enumerate(frames):
        buf[int(off[i]):int(off[i]) + len(f)] = np.frombuffer(f, np.uint8)
    lens = np.array([len(f) for f in frames], np.uint16)
    key = bytes(range(1, 17))
    want = Oracle().rx_batch(buf, off, lens, opts=make_opts(key, 24, 48, 1 << 12))
    z = {"buf": buf, "off": off, "len": lens, "key": np.frombuffer(key, np.uint8),
         "iphash": np.array([24, 48, 1 << 12])}
    got, _, perm = _run_mixed(_ctx(z), z, dev, shift=3)
    d = diff_records(got, want)
    assert not d, d
    assert np.array_equal(perm, _mixed_perm(lens))


@pytest.mark.parametrize("case", ["hint_1500", "no_jumbo", "few_jumbo", "all_jumbo",
                                  "jumbo_no_perm"])
def test_mixed_plan(case, dev):
    """The mixed call's choice between batch order and binning (include/
    pptk_rx.h): 2 000 frames of 60..1500 bytes, plus jumbo frames (1522..
    9018 B) in some cases; records bit-exact against the oracle whatever the
    choice, and the reported processing order is the one the rule names
    (binned only for a mix of jumbo and shorter frames without a low max_len
    hint; with d_perm NULL the binned permutation lives in the scratch)."""
    import framegen
    from oracle.oracle import Oracle, make_opts
    rng = np.random.default_rng(sum(case.encode()))
    n = 2000
    sizes = rng.integers(60, 1501, n)
    if case in ("few_jumbo", "jumbo_no_perm"):
        sizes[rng.choice(n, 40, replace=False)] = rng.integers(1522, 9019, 40)
    elif case == "all_jumbo":
        sizes = rng.integers(1522, 9019, n)
    max_len = 1500 if case == "hint_1500" else 0
    frames = [_frame_of_len(framegen, rng, int(L)) for L in sizes]
    off = np.cumsum([0] + [(len(f) + 3) & ~3 for f in frames[:-1]]).astype(np.uint64)
    buf = np.zeros(int(off[-1]) + len(frames[-1]) + 64, np.uint8)
    for i, f in enumerate(frames):
        buf[int(off[i]):int(off[i]) + len(f)] = np.frombuffer(f, np.uint8)
    lens = np.array([len(f) for f in frames], np.uint16)
    key = bytes(range(1, 17))
    want = Oracle().rx_batch(buf, off, lens, opts=make_opts(key, 24, 48, 1 << 12))
    z = {"buf": buf, "off": off, "len": lens, "key": np.frombuffer(key, np.uint8),
         "iphash": np.array([24, 48, 1 << 12])}
    ctx = _ctx(z)
    if case == "jumbo_no_perm":
        _keep, fr = _upload(buf, dev)
        recs = ctx.batch_device_mixed(fr, n, torch.from_numpy(off.view(np.int64)).to(dev),
                                      torch.from_numpy(lens.view(np.int16)).to(dev))
        torch.cuda.synchronize()
        d = diff_records(recs.cpu().numpy().reshape(-1), want)
        assert not d, d
        return
    got, h, perm = _run_mixed(ctx, z, dev, max_len=max_len)
    d = diff_records(got, want)
    assert not d, d
    expect = _mixed_perm(lens, max_len)
    assert np.array_equal(perm, expect)
    assert (perm != np.arange(n)).any() == (case == "few_jumbo")


@pytest.mark.parametrize("name", ["edge", "cmix"])
def test_bucket_disabled(name, dev):
    z = load_golden(name)
    got = _run(_ctx(z, bucket=False), z, dev)
    want = as_records(z["recs"]).copy()
    want["src_bucket"] = 0
    d = diff_records(got, want)
    assert not d, d


@pytest.mark.parametrize("name", ["edge", "fuzz", "cmix"])
def test_host_batch_ldp_packets(name, dev):
    """pptk_rx_batch: borrowed host frames (ldp_packet[]) in, records out."""
    from pptk_amd.rx import ldp_packets
    z = load_golden(name)
    ctx = _ctx(z)
    buf = np.ascontiguousarray(z["buf"])
    pkts = ldp_packets(buf, z["off"], z["len"])
    ancillary_before = [p.ancillary64 for p in pkts]
    got = ctx.batch_host(pkts)
    d = diff_records(got, z["recs"])
    assert not d, d
    assert [p.ancillary64 for p in pkts] == ancillary_before


@pytest.mark.parametrize("max_batch,threads", [(97, 1), (4096, 1), (1500, 6)])
@pytest.mark.parametrize("name", ["fuzz", "cmix"])
def test_host_batch_chunked_and_ring(name, max_batch, threads, dev):
    """pptk_rx_batch in chunks of max_batch (double-buffered pipeline), from
    staging and from a registered zero-copy ring; then unregistered."""
    from pptk_amd.rx import RxContext, ldp_packets
    z = load_golden(name)
    b4, b6, hs = (int(x) for x in z["iphash"])
    ctx = RxContext(0, z["key"].tobytes(), b4, b6, hs, max_batch=max_batch, max_frame=65535,
                    gather_threads=threads)
    ring = np.zeros(z["buf"].size + 4096, dtype=np.uint8)
    ring[:z["buf"].size] = z["buf"]
    pkts = ldp_packets(ring, z["off"], z["len"])
    d = diff_records(ctx.batch_host(pkts), z["recs"])
    assert not d, "staged: " + d
    ctx.register_ring(ring)
    d = diff_records(ctx.batch_host(pkts), z["recs"])
    assert not d, "ring: " + d
    ctx.unregister_ring(ring)
    d = diff_records(ctx.batch_host(pkts), z["recs"])
    assert not d, "after unregister: " + d


def _pages(nbytes):
    """A zeroed uint8 buffer starting on a page boundary, whole pages long
    (nbytes rounded up), with a free page after it."""
    pg = 4096
    size = (nbytes + pg - 1) // pg * pg
    raw = np.zeros(size + 2 * pg, dtype=np.uint8)
    a = (-raw.ctypes.data) % pg
    return raw[a:a + size]


@pytest.mark.parametrize("max_batch,threads", [(97, 1), (1500, 6), (65536, 8)])
@pytest.mark.parametrize("name", ["fuzz", "cmix"])
def test_host_batch_registered_records(name, max_batch, threads, dev):
    """A registered record array receives the records in place (the kernel
    writes them over PCIe, nothing is copied back), with staged frames and
    with frames from a registered ring; an unregistered array and a record
    array only partly inside a registered region take the copy path; every
    record against the golden set, and the bytes around the array untouched."""
    from pptk_amd.records import REC_DTYPE
    from pptk_amd.rx import RxContext, ldp_packets
    z = load_golden(name)
    n = len(z["off"])
    b4, b6, hs = (int(x) for x in z["iphash"])
    ctx = RxContext(0, z["key"].tobytes(), b4, b6, hs, max_batch=max_batch, max_frame=65535,
                    gather_threads=threads)
    # page-aligned buffers of whole pages: no two registrations share a page
    ring = _pages(z["buf"].size + 4096)
    ring[:z["buf"].size] = z["buf"]
    pkts = ldp_packets(ring, z["off"], z["len"])
    # the record array inside a larger registered region, 8 records in
    region = _pages((n + 16) * 64)
    region[:] = 0x5A
    region = region[:(n + 16) * 64]
    out = region[8 * 64:(8 + n) * 64].view(REC_DTYPE)
    ctx.register_ring(region)
    for ring_too in (False, True):
        if ring_too:
            ctx.register_ring(ring)
        for _ in range(2):
            out[:] = np.zeros(1, dtype=REC_DTYPE)
            got = ctx.batch_host(pkts, out=out)
            d = diff_records(got, z["recs"])
            assert not d, f"ring={ring_too}: " + d
            assert (region[:8 * 64] == 0x5A).all() and (region[(8 + n) * 64:] == 0x5A).all()
    ctx.unregister_ring(ring)
    # straddling the region's end: the copy path
    tail = _pages((n + 4) * 64)
    ctx.register_ring(tail[: (n // 2) * 64])
    d = diff_records(ctx.batch_host(pkts, out=tail[64:(n + 1) * 64].view(REC_DTYPE)),
                     z["recs"])
    assert not d, "straddling: " + d
    ctx.unregister_ring(tail[: (n // 2) * 64])
    ctx.unregister_ring(region)
    d = diff_records(ctx.batch_host(pkts, out=out), z["recs"])
    assert not d, "after unregister: " + d


def _packet_slice(pkts, lo, hi):
    """pkts[lo:hi] as a ctypes LdpPacket array aliasing `pkts` (no copy)."""
    import ctypes
    from pptk_amd.rx import LdpPacket
    s = (LdpPacket * (hi - lo)).from_address(ctypes.addressof(pkts) + lo * ctypes.sizeof(LdpPacket))
    s._keep = pkts
    return s


MAX_INFLIGHT = 4   # include/pptk_rx.h PPTK_RX_MAX_INFLIGHT


@pytest.mark.parametrize("mode,depth", [("staged", 2), ("ring", 2), ("ring_recs", 2),
                                        ("staged", 4), ("ring_recs", 4)])
@pytest.mark.parametrize("name", ["fuzz", "cmix", "c64", "c1500"])
def test_host_batch_pipelined(name, mode, depth, dev):
    """pptk_rx_batch_submit / _complete as an LDP rx loop uses them: ragged
    batches of 1 .. max_batch frames submitted `depth` deep (staged frames,
    frames in a registered ring, and records into a registered array too),
    every record against the golden set; and the queue contract: FIFO frame
    counts, -EBUSY for a submission beyond PPTK_RX_MAX_INFLIGHT and for
    pptk_rx_batch while any is outstanding, -EINVAL above max_batch, -ENOENT
    on an empty queue, and a context destroyed with submissions outstanding."""
    import errno
    from pptk_amd.records import REC_DTYPE
    from pptk_amd.rx import RxContext, ldp_packets
    z = load_golden(name)
    n = len(z["off"])
    b4, b6, hs = (int(x) for x in z["iphash"])
    max_batch = 1024
    ctx = RxContext(0, z["key"].tobytes(), b4, b6, hs, max_batch=max_batch, max_frame=65535,
                    gather_threads=4)
    ring = _pages(z["buf"].size + 4096)
    ring[:z["buf"].size] = z["buf"]
    pkts = ldp_packets(ring, z["off"], z["len"])
    region = _pages(n * 64)
    out = region[:n * 64].view(REC_DTYPE)
    if mode != "staged":
        ctx.register_ring(ring)
    if mode == "ring_recs":
        ctx.register_ring(region)
    rng = np.random.default_rng(7)
    sizes, pos = [], 0
    while pos < n:
        k = int(min(n - pos, rng.choice([1, 3, 64, 500, max_batch, int(rng.integers(1, max_batch))])))
        sizes.append((pos, k))
        pos += k
    for lap in range(2):
        out[:] = np.zeros(1, dtype=REC_DTYPE)
        queue = []
        for i, (lo, k) in enumerate(sizes):
            ctx.submit_host(_packet_slice(pkts, lo, lo + k), out[lo:lo + k])
            queue.append(k)
            if lap == 0 and i == 1:
                with pytest.raises(OSError) as e:
                    ctx.batch_host(_packet_slice(pkts, 0, 1), out=np.zeros(1, REC_DTYPE))
                assert e.value.errno == errno.EBUSY
            if ctx.pending_host() == depth:
                assert ctx.complete_host() == queue.pop(0)
        while queue:
            assert ctx.complete_host() == queue.pop(0)
        assert ctx.pending_host() == 0
        d = diff_records(out.copy(), z["recs"])
        assert not d, f"{mode} depth {depth} lap {lap}: " + d
    with pytest.raises(OSError) as e:
        ctx.complete_host()
    assert e.value.errno == errno.ENOENT
    if n > max_batch:
        with pytest.raises(OSError) as e:
            ctx.submit_host(_packet_slice(pkts, 0, max_batch + 1), out[:max_batch + 1])
        assert e.value.errno == errno.EINVAL
    # the synchronous call works again on the same slots
    d = diff_records(ctx.batch_host(pkts), z["recs"])
    assert not d, f"{mode} sync after async: " + d
    # the queue is full at PPTK_RX_MAX_INFLIGHT; the context is destroyed
    # with every submission outstanding: it waits for them, no fault
    k = min(n, max_batch)
    spare = [np.zeros(k, REC_DTYPE) for _ in range(MAX_INFLIGHT)]
    for j in range(MAX_INFLIGHT):
        ctx.submit_host(_packet_slice(pkts, 0, k), spare[j])
    with pytest.raises(OSError) as e:
        ctx.submit_host(_packet_slice(pkts, 0, k), out[:k])
    assert e.value.errno == errno.EBUSY
    assert ctx.pending_host() == MAX_INFLIGHT
    ctx.close()


def test_ring_edge_falls_back(dev):
    """A frame whose 16-byte-rounded end leaves the registered region makes
    the batch use staging; results stay exact."""
    from pptk_amd.rx import RxContext, ldp_packets
    z = load_golden("edge")
    i = int(np.argmax(z["len"] % 16 == 7))
    fr = z["buf"][int(z["off"][i]):int(z["off"][i]) + int(z["len"][i])]
    ring = np.zeros(int(z["len"][i]) + 3, dtype=np.uint8)   # end not 16-rounded
    ring[:fr.size] = fr
    ctx = _ctx(z)
    ctx.register_ring(ring)
    got = ctx.batch_host(ldp_packets(ring, [0], [fr.size]))
    d = diff_records(got, z["recs"][i:i + 1])
    assert not d, d
    ctx.unregister_ring(ring)


def test_host_batch_max_frame(dev):
    """Frames longer than opts.max_frame come back MALFORMED-only."""
    from pptk_amd.records import F_MALFORMED
    from pptk_amd.rx import ldp_packets
    z = load_golden("edge")
    ctx = _ctx(z, max_frame=1514)
    buf = np.ascontiguousarray(z["buf"])
    got = ctx.batch_host(ldp_packets(buf, z["off"], z["len"]))
    long = z["len"] > 1514
    assert long.any()
    assert np.all(got["flags"][long] == F_MALFORMED)
    assert not diff_records(got[~long], z["recs"][~long])


def test_empty_and_single(dev):
    z = load_golden("edge")
    ctx = _ctx(z)
    frames = torch.zeros(64, dtype=torch.uint8, device=dev)
    recs = torch.zeros((1, 64), dtype=torch.uint8, device=dev)
    ctx.batch_device(frames, 0, stride=64, fixed_len=64, recs=recs)  # n = 0: no-op
    torch.cuda.synchronize()
    assert int(recs.sum()) == 0
    for i in range(0, len(z["off"]), 37):
        one = {"buf": z["buf"][int(z["off"][i]):int(z["off"][i]) + int(z["len"][i])].copy(),
               "off": np.zeros(1, np.uint64), "len": z["len"][i:i + 1].copy(),
               "key": z["key"], "iphash": z["iphash"]}
        got = _run(ctx, one, dev)
        d = diff_records(got, z["recs"][i:i + 1])
        assert not d, f"frame {i}: {d}"


def _small_fixed_batches():
    """Every golden frame of at most 64 bytes, grouped by length (a fixed-stride
    batch has one length), with the records the reference produced."""
    groups = {}
    for name in GOLDEN_SETS:
        z = load_golden(name)
        for i in np.flatnonzero(z["len"] <= 64):
            L = int(z["len"][i])
            fr = z["buf"][int(z["off"][i]):int(z["off"][i]) + L]
            groups.setdefault(L, ([], []))
            groups[L][0].append(fr)
            groups[L][1].append(z["recs"][i])
    return groups


@pytest.mark.parametrize("stride_kind", ["tight", "64", "96"])
@pytest.mark.parametrize("compact", [False, True])
def test_lane_kernel(stride_kind, compact, dev):
    """RX_L4 (lane kernel: fixed stride, 16-byte aligned frames <= 64 B) on
    every golden frame that short -- VLAN, IPv6, malformed, fragments, padded
    and odd-length frames (the generic per-lane path) and plain IPv4 (the
    register fast path) -- bit-exact, with the flow-hash array."""
    from pptk_amd.rx import RX_L4
    zk = load_golden("edge")
    ctx = _ctx(zk)
    groups = _small_fixed_batches()
    assert len(groups) > 20
    for L, (frs, recs) in sorted(groups.items()):
        stride = {"tight": max(16, (L + 15) // 16 * 16), "64": 64, "96": 96}[stride_kind]
        n = len(frs)
        buf = np.zeros(n * stride + 16, np.uint8)
        for k, fr in enumerate(frs):
            buf[k * stride:k * stride + L] = fr
            buf[k * stride + L:(k + 1) * stride] = 0xA5   # garbage after the frame
        want = np.array(recs)
        frames = torch.from_numpy(buf).to(dev)
        h = torch.full((n,), -1, dtype=torch.int64, device=dev)
        got = ctx.batch_device(frames, n, stride=stride, fixed_len=L, hash_out=h,
                               compact=compact)
        torch.cuda.synchronize()
        assert ctx.last_variant() == RX_L4, f"len {L}: lane kernel not selected"
        got = got.cpu().numpy().reshape(-1)
        if compact:
            d = diff_records(got, to_rec32(want), dtype=REC32_DTYPE)
        else:
            d = diff_records(got, want)
        assert not d, f"len {L} stride {stride}: {d}"
        w = as_records(want)
        hh = h.cpu().numpy().view(np.uint64)
        assert np.array_equal(hh, np.where(w["flags"] & F_PARSED, w["flow_hash"], 0)), L


def test_lane_kernel_large_batch(dev):
    """Many tiles per wave (the prefetch loop), a ragged last tile, every 7th
    frame corrupted, against the oracle; misaligned buffers fall back to the
    team kernels with the same results."""
    import framegen
    from oracle.oracle import Oracle, make_opts
    from pptk_amd.rx import RX_L4, RxContext
    rng = np.random.default_rng(5)
    n = 300_001
    base = framegen.frame_v4(rng, 17, 64)
    buf = np.tile(np.frombuffer(base, np.uint8), n).copy()
    # vary addresses / ports / payload so every record differs
    rnd = rng.integers(0, 256, size=(n, 64), dtype=np.uint8)
    v = buf.reshape(n, 64)
    v[:, 26:38] = rnd[:, 26:38]
    v[:, 42:64] = rnd[:, 42:64]
    v[::7, 50] ^= 0x5A                               # corrupt the UDP checksum of some
    v[::11, 0] = 0                                   # (L2 bytes are not covered)
    off = np.arange(n, dtype=np.uint64) * 64
    lens = np.full(n, 64, np.uint16)
    key = bytes(range(1, 17))
    want = Oracle().rx_batch(buf, off, lens, opts=make_opts(key, 24, 48, 1 << 12))
    ctx = RxContext(0, key, 24, 48, 1 << 12)
    big = torch.zeros(buf.size + 64, dtype=torch.uint8, device=dev)
    big[:buf.size] = torch.from_numpy(buf).to(dev)
    for shift, lane in ((0, True), (16, True), (8, False)):
        fr = big[shift:]
        if shift:
            fr[:buf.size] = torch.from_numpy(buf).to(dev)
        got = ctx.batch_device(fr, n, stride=64, fixed_len=64)
        torch.cuda.synchronize()
        assert (ctx.last_variant() == RX_L4) == lane
        d = diff_records(got.cpu().numpy().reshape(-1), want)
        assert not d, f"shift {shift}: {d}"
    # the coalesced tile loads (64-byte stride, four chunks per frame) under
    # every memory policy: temporal / non-temporal loads and stores
    big[:buf.size] = torch.from_numpy(buf).to(dev)   # (the shifted runs moved it)
    for flags in (0x0, 0x1, 0x20, 0x21):
        ctx.set_tuning(RX_L4, flags)
        got = ctx.batch_device(big, n, stride=64, fixed_len=64)
        torch.cuda.synchronize()
        assert ctx.last_variant() == RX_L4
        d = diff_records(got.cpu().numpy().reshape(-1), want)
        assert not d, f"flags {flags:#x}: {d}"
    ctx.set_tuning(-1, -1)


@pytest.mark.parametrize("cfg", ["c64", "c1500"])
def test_host_batch_worker_pool_large_chunks(cfg, dev):
    """Chunks big enough that the worker pool splits both the frame gather
    and the record copy-out (>= 2 MiB of records per chunk), over repeated
    calls on one context and then from two contexts on two host threads at
    once: every record equals the CPU oracle's."""
    import threading
    from oracle.oracle import Oracle, make_opts
    from pptk_amd.rx import RxContext, ldp_packets
    from harness.synth import make_batch
    n = 200_000 if cfg == "c64" else 70_000
    b = make_batch(cfg, n, dev)
    stride = b["stride"]
    ring = b["frames"][: n * stride + 64].cpu().numpy()
    want = Oracle().rx_batch(ring, None, None, stride=stride, fixed_len=b["fixed_len"], n=n,
                             opts=make_opts(bytes(range(1, 17))), nthreads=8)
    want = want.view(np.uint8).reshape(n, 64)
    pkts = ldp_packets(ring, np.arange(n, dtype=np.uint64) * stride,
                       np.full(n, b["fixed_len"], np.uint16))
    ctxs = [RxContext(0, bytes(range(1, 17)), max_batch=65536, max_frame=1518,
                      gather_threads=8) for _ in range(2)]
    for _ in range(2):
        got = ctxs[0].batch_host(pkts)
        assert np.array_equal(got.view(np.uint8).reshape(n, 64), want)
    out = [None, None]

    def run(k):
        out[k] = ctxs[k].batch_host(pkts)

    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for k in range(2):
        assert np.array_equal(out[k].view(np.uint8).reshape(n, 64), want)
        ctxs[k].close()


@pytest.mark.parametrize("gap,pct", [(0, None), (7, None), (1500, None), (548, 70)])
def test_registered_ring_span_dma(gap, pct, dev):
    """A registered ring holding 70 000 C1500 frames `gap` bytes apart
    (tests/ringcase.py): dense chunks (gap 0 or 7) go down as one DMA span
    with rebased offsets; a sparse ring (gap 1500: half the span is frames)
    is read in place by the kernel; with the threshold lowered to 70 %
    (PPTK_RX_RING_DMA_PCT, read once per process: a child process) 2 KB
    netmap-style slots (gap 548: 73 % frames) go down by DMA too, into a
    device buffer grown for the longer span.  The short last chunk runs
    direct.  Every record equals the CPU oracle's, and the same through
    staging."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    if pct is None:
        sys.path.insert(0, here)
        import ringcase
        ringcase.run(gap)
        return
    env = dict(os.environ, PPTK_RX_RING_DMA_PCT=str(pct))
    r = subprocess.run([sys.executable, os.path.join(here, "ringcase.py"), str(gap)],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("seed", [0, 1])
def test_large_fresh_batches_vs_oracle(seed, oracle_lib, dev):
    """Fresh seeds, not in any fixture: 60 K fuzzed frames (malformed,
    truncated, odd lengths, extension chains, jumbo) and 60 K CMIX frames,
    interleaved in one batch and packed at an odd alignment, through the
    default variant and the compact records: bit-exact against the CPU
    restatement (itself pinned to the reference by the golden fixtures)."""
    import framegen
    from oracle.oracle import make_opts
    fb, fo, fl = framegen.gen_fuzz(60000, seed=0x7100 + seed)
    cb, co, cl = framegen.gen_cmix(60000, seed=0x7200 + seed)
    frames = []
    for k in range(60000):
        frames.append(fb[int(fo[k]):int(fo[k]) + int(fl[k])].tobytes())
        frames.append(cb[int(co[k]):int(co[k]) + int(cl[k])].tobytes())
    buf, off, lens = framegen.pack(frames, align=1 + 2 * seed)
    key = bytes(range(3, 19))
    z = {"buf": buf, "off": off, "len": lens, "key": np.frombuffer(key, np.uint8),
         "iphash": np.array([22, 56, 1 << 14])}
    want = oracle_lib.rx_batch(buf, off, lens, opts=make_opts(key, 22, 56, 1 << 14), nthreads=8)
    ctx = _ctx(z)
    got = _run(ctx, z, dev, shift=3)
    d = diff_records(got, want)
    assert not d, d
    got32 = _run(ctx, z, dev, shift=3, compact=True)
    d = diff_records(got32, to_rec32(want), dtype=REC32_DTYPE)
    assert not d, d
    from pptk_amd.rx import VARIANTS
    ctx.set_tuning(VARIANTS.index("M6"), -1)   # lanes binned by length inside the tile
    got = _run(ctx, z, dev, shift=5)
    d = diff_records(got, want)
    assert not d, d


@pytest.mark.parametrize("cfg", ["imix", "cmix", "jmix"])
def test_mixed_shape_kernel_vs_oracle(cfg, oracle_lib, dev):
    """RX_M6 (each tile's frames binned by chunk count into 4-, 8- and
    16-lane team rounds) on 2^17-frame synthetic batches of every mixed
    config: records, dense flow hashes and compact records bit-exact against
    the CPU oracle, in batch order and in a binned processing order."""
    from oracle.oracle import make_opts
    from pptk_amd.rx import RxContext, VARIANTS
    from harness.synth import make_batch
    n = 1 << 17
    b = make_batch(cfg, n, dev)
    host = b["frames"].cpu().numpy()
    off = b["off"].cpu().numpy().view(np.uint64)
    lens = b["lens"].cpu().numpy().view(np.uint16)
    key = bytes(range(1, 17))
    want = oracle_lib.rx_batch(host, off, lens, opts=make_opts(key, 24, 48, 1 << 12), nthreads=8)
    ctx = RxContext(0, key, 24, 48, 1 << 12)
    ctx.set_tuning(VARIANTS.index("M6"), -1)
    kw = dict(off=b["off"], lens=b["lens"], max_len=b["max_len"])
    h = torch.full((n,), -1, dtype=torch.int64, device=dev)
    recs = ctx.batch_device(b["frames"], n, hash_out=h, **kw)
    torch.cuda.synchronize()
    assert ctx.last_variant() == VARIANTS.index("M6")
    got = recs.cpu().numpy().reshape(-1)
    d = diff_records(got, want)
    assert not d, d
    assert np.array_equal(h.cpu().numpy().view(np.uint64), want["flow_hash"])
    r32 = ctx.batch_device(b["frames"], n, compact=True, **kw)
    torch.cuda.synchronize()
    d = diff_records(r32.cpu().numpy().reshape(-1), to_rec32(want), dtype=REC32_DTYPE)
    assert not d, d
    p = ctx.bin_device(b["lens"], n)
    recs = ctx.batch_device(b["frames"], n, perm=p, **kw)
    torch.cuda.synchronize()
    d = diff_records(recs.cpu().numpy().reshape(-1), want)
    assert not d, d
    ctx.close()


@pytest.mark.parametrize("cfg", ["imix", "cmix"])
def test_mixed_shape_kernel_full_size(cfg, dev):
    """BASELINE sizes (16 M frames): M6 and the team kernel T16S6 write
    byte-identical records for the whole batch, every frame parses, and
    every IP / L4 verdict equals what the generator planted (its own
    checksums, ~1 % of frames corrupted) -- size-independent properties."""
    from pptk_amd.records import F_IP_OK, F_L4_OK, F_PARSED
    from pptk_amd.rx import RxContext, VARIANTS
    from harness.synth import make_batch
    n = 1 << 24
    b = make_batch(cfg, n, dev)
    kw = dict(off=b["off"], lens=b["lens"], max_len=b["max_len"])
    ctx = RxContext(0, bytes(range(1, 17)))
    ctx.set_tuning(VARIANTS.index("M6"), -1)
    got = ctx.batch_device(b["frames"], n, **kw)
    ctx.set_tuning(VARIANTS.index("T16S6"), -1)
    ref = ctx.batch_device(b["frames"], n, **kw)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    r = got.view(torch.int16)[:, 27].to(torch.int32) & 0xFFFF      # flags @54
    exp = b["expect"].to(torch.int32)
    assert bool(((r & F_PARSED) != 0).all().item())
    assert bool((((r & F_IP_OK) != 0).to(torch.int32) == (exp & 1)).all().item())
    assert bool((((r & F_L4_OK) != 0).to(torch.int32) == ((exp >> 1) & 1)).all().item())
    assert int((exp != 3).sum().item()) > n // 200                 # corrupted frames present
    ctx.close()


@pytest.mark.parametrize("cfg", ["c64", "cmix", "imix"])
def test_full_size_windows_vs_oracle(cfg, oracle_lib, dev):
    """BASELINE sizes (16 M frames) on the product's own choices -- the lane
    kernel's coalesced tiles at 4 tiles per wave (C64), the streaming shapes
    and M6 on the oversubscribed grid at 8 (CMIX, IMIX) -- checked bit-exact
    against the CPU oracle on 24 windows of 2 048 consecutive frames spread
    over the batch (first, last and random tiles), records and compact
    records."""
    from oracle.oracle import make_opts
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    n = 1 << 24
    b = make_batch(cfg, n, dev)
    key = bytes(range(1, 17))
    ctx = RxContext(0, key)
    fixed = "off" not in b
    kw = (dict(stride=b["stride"], fixed_len=b["fixed_len"]) if fixed else
          dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]))
    got = ctx.batch_device(b["frames"], n, **kw)
    got32 = ctx.batch_device(b["frames"], n, compact=True, **kw)
    torch.cuda.synchronize()
    w = 2048
    rng = np.random.default_rng(11)
    starts = sorted({0, n - w, *(int(x) * 64 for x in rng.integers(0, (n - w) // 64, 22))})
    if fixed:
        off_all = None
    else:
        off_all = b["off"].cpu().numpy().view(np.uint64)
        len_all = b["lens"].cpu().numpy().view(np.uint16)
    opts = make_opts(key)
    for s0 in starts:
        if fixed:
            lo, hi = s0 * b["stride"], (s0 + w) * b["stride"]
            off = np.arange(w, dtype=np.uint64) * np.uint64(b["stride"])
            lens = np.full(w, b["fixed_len"], np.uint16)
        else:
            lo = int(off_all[s0]) & ~15
            hi = int(off_all[s0 + w - 1]) + int(len_all[s0 + w - 1])
            off = off_all[s0:s0 + w] - np.uint64(lo)
            lens = len_all[s0:s0 + w]
        host = b["frames"][lo:hi + 16].cpu().numpy()
        want = oracle_lib.rx_batch(host, off, lens, opts=opts, nthreads=8)
        d = diff_records(got[s0:s0 + w].cpu().numpy().reshape(-1), want)
        assert not d, f"{cfg} frames {s0}..{s0 + w}: {d}"
        d = diff_records(got32[s0:s0 + w].cpu().numpy().reshape(-1), to_rec32(want),
                         dtype=REC32_DTYPE)
        assert not d, f"{cfg} compact, frames {s0}..{s0 + w}: {d}"
    ctx.close()


@pytest.mark.parametrize("layout", ["fixed", "offsets"])
def test_autotune_keeps_records(layout, dev):
    """pptk_rx_autotune picks one of the interchangeable shapes for a
    C1500-class batch; later batches launch it and their records equal the
    CPU oracle's, bit for bit."""
    from oracle.oracle import Oracle, make_opts
    from pptk_amd.rx import RxContext, VARIANTS
    from harness.synth import make_batch
    n = 1 << 17
    b = make_batch("c1500" if layout == "fixed" else "cmix", n, dev)
    kw = (dict(stride=b["stride"], fixed_len=b["fixed_len"]) if "off" not in b else
          dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]))
    host = b["frames"].cpu().numpy()
    opts = make_opts(bytes(range(1, 17)))
    if "off" in b:
        w = Oracle().rx_batch(host, b["off"].cpu().numpy().view(np.uint64),
                              b["lens"].cpu().numpy().view(np.uint16), opts=opts, nthreads=8)
    else:
        w = Oracle().rx_batch(host, None, None, stride=b["stride"], fixed_len=b["fixed_len"],
                              n=n, opts=opts, nthreads=8)
    want = torch.from_numpy(w.view(np.uint8).reshape(n, 64).copy())
    ctx = RxContext(0, bytes(range(1, 17)))
    name = ctx.autotune(b["frames"], n, reps=2, **kw)
    assert name in (("T16S6", "T32S3", "T32S3D7", "T16S7L") +
                    (("M6",) if layout == "offsets" else ()))
    got = ctx.batch_device(b["frames"], n, **kw)
    torch.cuda.synchronize()
    assert VARIANTS[ctx._L.pptk_rx_last_variant(ctx._ctx)] == name
    assert torch.equal(got.cpu(), want)
    ctx.set_tuning(VARIANTS.index("T16S2"), -1)        # a forced variant still wins
    ctx.batch_device(b["frames"], n, **kw)
    torch.cuda.synchronize()
    assert VARIANTS[ctx._L.pptk_rx_last_variant(ctx._ctx)] == "T16S2"


def test_host_batch_error_paths(dev):
    """pptk_rx_batch's per-packet and contract error paths on hardware: a
    NULL frame pointer comes back MALFORMED-only (no fault, no error), the
    other frames of the batch are exact; a NULL packet table or record array
    with num > 0 and a negative num are -EINVAL; num == 0 is a no-op; an
    unknown ring cannot be unregistered; a batch still works afterwards."""
    import ctypes
    from pptk_amd.records import F_MALFORMED
    from pptk_amd.rx import ldp_packets
    z = load_golden("cmix")
    ctx = _ctx(z)
    buf = np.ascontiguousarray(z["buf"])
    pkts = ldp_packets(buf, z["off"], z["len"])
    holes = [0, 7, len(pkts) - 1]
    for i in holes:
        pkts[i].data = None
    got = ctx.batch_host(pkts)
    want = np.array(z["recs"]).reshape(-1).view(np.uint8).reshape(-1, 64).copy()
    from pptk_amd.records import as_records
    for i in holes:
        assert got["flags"][i] == F_MALFORMED
    keep = np.setdiff1d(np.arange(len(pkts)), holes)
    assert not diff_records(got[keep], as_records(want)[keep])
    L, c = ctx._L, ctx._ctx
    recs = np.zeros(4, dtype=got.dtype)
    rp = ctypes.c_void_p(recs.ctypes.data)
    assert L.pptk_rx_batch(c, None, 4, rp) == -22
    assert L.pptk_rx_batch(c, ctypes.cast(pkts, ctypes.c_void_p), 4, None) == -22
    assert L.pptk_rx_batch(c, ctypes.cast(pkts, ctypes.c_void_p), -1, rp) == -22
    assert L.pptk_rx_batch(c, None, 0, None) == 0
    other = np.zeros(4096, np.uint8)
    assert L.pptk_rx_unregister_ring(c, ctypes.c_void_p(other.ctypes.data)) == -22
    pkts2 = ldp_packets(buf, z["off"][:64], z["len"][:64])
    assert not diff_records(ctx.batch_host(pkts2), z["recs"][:64])
    ctx.close()


@pytest.mark.parametrize("compact", [False, True])
def test_place_records(compact, dev):
    """pptk_rx_place_records runs the batch into every candidate record
    buffer, returns the fastest's index and per-candidate times; every
    candidate holds the exact records afterwards."""
    z = load_golden("cmix")
    n = len(z["off"])
    ctx = _ctx(z)
    frames = torch.from_numpy(z["buf"]).to(dev)
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    rb = 32 if compact else 64
    cands = [torch.zeros((n, rb), dtype=torch.uint8, device=dev) for _ in range(3)]
    best, ms = ctx.place_records(frames, n, cands, off=off, lens=lens, max_len=1500,
                                 compact=compact, reps=2)
    assert 0 <= best < 3 and len(ms) == 3 and ms[best] == min(ms) and all(m > 0 for m in ms)
    want = to_rec32(z["recs"]) if compact else z["recs"]
    for c in cands:
        d = diff_records(c.cpu().numpy().reshape(-1), want,
                         dtype=REC32_DTYPE if compact else as_records(z["recs"]).dtype)
        assert not d, d
    with pytest.raises(OSError):
        ctx.place_records(frames, n, [], off=off, lens=lens)
    ctx.close()


def test_stream_split(dev):
    """pptk_rx_stream_split: the collective's stream holds the top 32 CU-mask
    bits (4 CUs of every XCC, one per shader engine), the batches' stream the
    rest; other counts are -EINVAL; records are the same on either stream,
    split or not, and after the join."""
    import ctypes
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    n = 1 << 16
    b = make_batch("c1500", n, dev)
    kw = dict(stride=b["stride"], fixed_len=b["fixed_len"])
    ctx = RxContext(0, bytes(range(1, 17)))
    want = ctx.batch_device(b["frames"], n, **kw)
    torch.cuda.synchronize()
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    for bad in (-1, 16, 33, ncu):
        with pytest.raises(OSError) as e:
            ctx.stream_split(bad)
        assert e.value.errno == 22
    rx, coll = ctx.stream_split(32)
    hip = ctypes.CDLL("libamdhip64.so")
    for s, lo, hi in ((rx, 0, ncu - 32), (coll, ncu - 32, ncu)):
        words = (ctypes.c_uint32 * (ncu // 32))()
        assert hip.hipExtStreamGetCUMask(ctypes.c_void_p(s.cuda_stream), len(words), words) == 0
        bits = [i for i in range(ncu) if words[i // 32] >> (i % 32) & 1]
        assert bits == list(range(lo, hi))
    for s in (rx, coll):
        got = ctx.batch_device(b["frames"], n, stream=s, **kw)
        s.synchronize()
        assert torch.equal(got, want)
    # the rate limiter's one-launch path (grid barriers) on the batches'
    # stream: its grid fits the CUs the split leaves it
    rng = np.random.default_rng(5)
    nk, hs = 1 << 22, 1 << 16
    keys = torch.from_numpy(rng.integers(0, hs, nk).astype(np.int32)).to(dev)
    tok0 = torch.from_numpy(rng.integers(0, 64, hs).astype(np.int32)).to(dev)
    pctx = RxContext(0, bytes(range(1, 17)), iphash_bits4=24, iphash_bits6=48, iphash_size=hs)
    t_ref = tok0.clone()
    v_ref = pctx.permit_keys_device(keys, 4, t_ref)
    torch.cuda.synchronize()
    prx, _ = pctx.stream_split(32)
    t_got = tok0.clone()
    scratch = torch.empty(pctx._L.pptk_rx_permit_scratch_bytes(nk, hs), dtype=torch.uint8,
                          device=dev)
    v_got = pctx.permit_keys_device(keys, 4, t_got, scratch=scratch, stream=prx)
    assert pctx.permit_status(scratch, stream=prx) == 0
    assert torch.equal(v_got, v_ref) and torch.equal(t_got, t_ref)
    pctx.stream_join()
    pctx.close()
    ctx.stream_join()
    got = ctx.batch_device(b["frames"], n, **kw)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    ctx.close()


def test_tuning_rejects_diagnostic_bits(dev):
    """The product library accepts only the result-preserving tuning bits:
    the diagnostic ones (skip record stores 0x8, skip the per-frame phase
    0x10, half the record bytes 0x80, skip tx writes 0x200) are -EINVAL."""
    z = load_golden("edge")
    ctx = _ctx(z)
    for bad in (0x8, 0x10, 0x80, 0x200, 0x21 | 0x8):
        with pytest.raises(OSError) as e:
            ctx.set_tuning(-1, bad)
        assert e.value.errno == 22
    for good in (0x1, 0x2, 0x20, 0x40, 0x100, 0x163):
        ctx.set_tuning(-1, good)
    ctx.close()


def test_place_buffers(dev):
    """pptk_rx_place_buffers times the batch on every (frames, records) pair
    of candidates (frame candidates hold the same bytes) and returns the
    fastest pair; every record candidate holds the exact records."""
    z = load_golden("fuzz")
    n = len(z["off"])
    ctx = _ctx(z)
    f0 = torch.from_numpy(z["buf"]).to(dev)
    frames = [f0, f0.clone(), f0.clone()]
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    recs = [torch.zeros((n, 64), dtype=torch.uint8, device=dev) for _ in range(2)]
    fi, ri, ms = ctx.place_buffers(frames, n, recs, off=off, lens=lens, max_len=1500, reps=2)
    assert 0 <= fi < 3 and 0 <= ri < 2 and len(ms) == 6 and ms[fi * 2 + ri] == min(ms)
    for r in recs:
        d = diff_records(r.cpu().numpy().reshape(-1), z["recs"])
        assert not d, d
    with pytest.raises(OSError):
        ctx.place_buffers([], n, recs, off=off, lens=lens)
    ctx.close()


@pytest.mark.parametrize("compact", [False, True])
def test_ring_alloc(compact, dev):
    """pptk_rx_ring_alloc: the library allocates and probes candidate (frames,
    records) pairs and keeps the fastest; the rings it returns are sized as
    asked, the report is consistent, the golden batch written into the frame
    ring gives the exact records in the record ring, and the rings are freed
    when the last tensor over them goes (the device memory comes back)."""
    import gc
    z = load_golden("cmix")
    n = len(z["off"])
    ctx = _ctx(z)
    rb = 32 if compact else 64
    fbytes = max(z["buf"].size, 1500 * 4096)
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info(dev)
    ring = ctx.ring_alloc(fbytes, n, rb, frame_cands=2, rec_cands=3, reps=2)
    rep = ring.report
    assert ring.frames.numel() == fbytes + 64 and tuple(ring.recs.shape) == (n, rb)
    assert rep["frame_cands"] == 2 and rep["rec_cands"] == 3
    assert 0 <= rep["chosen_frames"] < 2 and 0 <= rep["chosen_recs"] < 3
    assert 0 < rep["chosen_ms"] <= rep["first_ms"] or rep["chosen_frames"] + rep["chosen_recs"] == 0
    assert rep["probe_frames"] == min(n, fbytes // 1500) and rep["freed_bytes"] > 0
    ring.frames[:z["buf"].size].copy_(torch.from_numpy(z["buf"]).to(dev))
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    ctx.batch_device(ring.frames, n, off=off, lens=lens, max_len=1500, recs=ring.recs,
                     compact=compact)
    torch.cuda.synchronize()
    want = to_rec32(z["recs"]) if compact else z["recs"]
    d = diff_records(ring.recs.cpu().numpy().reshape(-1), want,
                     dtype=REC32_DTYPE if compact else as_records(z["recs"]).dtype)
    assert not d, d
    del ring
    gc.collect()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info(dev)
    assert free1 >= free0 - (64 << 20)
    ctx.close()


def test_ring_alloc_two_queues_on_one_gpu(dev):
    """Two rx queues of one GPU, a context each (reference ldp/ldprecvmt.c:
    16-67), set up their rings at the same time from two threads, each with
    a memory budget: the library runs the two placement probes one after the
    other (so neither sizes its candidates from memory the other is holding,
    nor times its probe beside the other's), both calls succeed with more
    than one candidate pair, and both rings give the golden records."""
    import threading
    z = load_golden("cmix")
    n = len(z["off"])
    ctxs = [_ctx(z), _ctx(z)]
    fbytes = max(z["buf"].size, 1500 * 4096)
    rings, errs = [None, None], []

    def setup(k):
        try:
            rings[k] = ctxs[k].ring_alloc(fbytes, n, 64, frame_cands=2, rec_cands=4, reps=2,
                                          budget_bytes=12 << 30,
                                          stream=torch.cuda.Stream(dev))
        except Exception as e:          # (reported below)
            errs.append(repr(e))

    th = [threading.Thread(target=setup, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    for ctx, ring in zip(ctxs, rings):
        rep = ring.report
        assert rep["frame_cands"] * rep["rec_cands"] > 1, rep
        ring.frames[:z["buf"].size].copy_(torch.from_numpy(z["buf"]).to(dev))
        ctx.batch_device(ring.frames, n, off=off, lens=lens, max_len=1500, recs=ring.recs)
        torch.cuda.synchronize()
        d = diff_records(ring.recs.cpu().numpy().reshape(-1), z["recs"])
        assert not d, d
    assert rings[0].frames.data_ptr() != rings[1].frames.data_ptr()
    del rings
    for ctx in ctxs:
        ctx.close()


def test_ring_alloc_budget_limits_candidates(dev):
    """A budget smaller than the default candidate set: fewer candidates
    are probed (the spacers and candidates must fit in it), the ring is
    still returned and correct in size."""
    z = load_golden("edge")
    ctx = _ctx(z)
    fbytes = 1500 * 4096
    ring = ctx.ring_alloc(fbytes, 4096, 64, budget_bytes=3 << 30)
    rep = ring.report
    assert rep["frame_cands"] * rep["rec_cands"] < 3 * 8, rep
    assert ring.frames.numel() == fbytes + 64 and tuple(ring.recs.shape) == (4096, 64)
    del ring
    ctx.close()


def test_ring_alloc_rejects(dev):
    """Bad ring specs are -EINVAL before anything is allocated."""
    z = load_golden("edge")
    ctx = _ctx(z)
    for kw in (dict(frame_bytes=0, nrec=10), dict(frame_bytes=1 << 20, nrec=0),
               dict(frame_bytes=1 << 20, nrec=10, rec_bytes=48),
               dict(frame_bytes=1 << 20, nrec=10, probe_len=63),
               dict(frame_bytes=1 << 20, nrec=10, probe_len=1537),
               dict(frame_bytes=1 << 20, nrec=10, frame_cands=9),
               dict(frame_bytes=1 << 20, nrec=10, rec_cands=17),
               dict(frame_bytes=100, nrec=10)):          # no probe frame fits
        with pytest.raises(OSError) as e:
            ctx.ring_alloc(**kw)
        assert e.value.errno == 22, kw
    ctx.close()


@pytest.mark.parametrize("name,stride", [("c64", 64), ("c1500", 1500)])
def test_m6_fixed_stride_forced(name, stride, dev):
    """The mixed-shape kernel (M6) forced on a fixed-stride batch -- its
    masked-sum instantiation, rx_kernel_mixed<NT, false>, which autotune
    never picks (it is a candidate for offset-described batches only): the
    launch really is M6, and the records are exact, full and compact."""
    from pptk_amd.rx import VARIANTS
    z = load_golden(name)
    ctx = _ctx(z)
    m6 = VARIANTS.index("M6")
    for flags in (0, 1):
        ctx.set_tuning(m6, flags)
        for shift in (0, 3):
            got = _run(ctx, z, dev, shift=shift, stride=stride)
            assert ctx.last_variant() == m6
            d = diff_records(got, z["recs"])
            assert not d, f"shift {shift} flags {flags}: {d}"
            got = _run(ctx, z, dev, shift=shift, stride=stride, compact=True)
            d = diff_records(got, to_rec32(z["recs"]), dtype=REC32_DTYPE)
            assert not d, f"compact shift {shift} flags {flags}: {d}"


@pytest.mark.parametrize("name,stride", [("c1500", 1500), ("c64", 64), ("cmix", None)])
@pytest.mark.parametrize("compact", [False, True])
def test_dense_hash_misaligned_and_ragged(name, stride, compact, dev):
    """The dense flow-hash array (d_hash) as the flush stores it -- one run
    of 16-byte stores per tile from the record slots' spare bytes -- into a
    destination 8 bytes off a 16-byte boundary (a rank's slice of a gather
    buffer with an odd per-rank count) and for a frame count that leaves the
    last tile ragged: every hash equals the golden flow hash, the words
    around the slice are untouched, every variant the batch may run, full
    and compact records."""
    from pptk_amd.rx import VARIANTS
    z = load_golden(name)
    n_all = len(z["off"])
    n = n_all - 37 if n_all > 100 else n_all    # ragged last tile
    zz = dict(z)
    zz["off"], zz["len"], zz["recs"] = z["off"][:n], z["len"][:n], z["recs"][:n]
    ctx = _ctx(z)
    _keep, frames = _upload(zz["buf"], dev, 0)
    kw = (dict(stride=stride, fixed_len=int(zz["len"][0])) if stride else
          dict(off=torch.from_numpy(zz["off"].view(np.int64)).to(dev),
               lens=torch.from_numpy(zz["len"].view(np.int16)).to(dev),
               max_len=int(zz["len"].max())))
    want = as_records(zz["recs"])["flow_hash"]
    variants = [-1] + ([VARIANTS.index(v) for v in ("T16S6", "T16S7L", "M6")] if name != "c64"
                       else [VARIANTS.index(v) for v in ("L4", "T4S2", "M6")])
    for v in variants:
        ctx.set_tuning(v, -1)
        big = torch.full((n + 3,), -7, dtype=torch.int64, device=dev)
        assert (big[1:].data_ptr() % 16) == 8
        ctx.batch_device(frames, n, hash_out=big[1:n + 1], compact=compact, **kw)
        torch.cuda.synchronize()
        got = big.cpu().numpy()
        assert np.array_equal(got[1:n + 1].view(np.uint64), want), VARIANTS[ctx.last_variant()]
        assert got[0] == -7 and (got[n + 1:] == -7).all()
    ctx.close()


@pytest.mark.parametrize("max_batch,threads", [(97, 1), (4096, 4), (65536, 8)])
@pytest.mark.parametrize("mode", ["staged", "ring", "ring_recs"])
@pytest.mark.parametrize("name", ["edge", "fuzz", "cmix", "c64", "c1500"])
def test_host_batch_compact_records(name, mode, max_batch, threads, dev):
    """pptk_rx_batch32 (compact 32-byte records host to host): staged frames,
    frames in a registered ring, and records written in place into a
    registered array; small chunks (direct: the kernel reads the pinned
    staging and writes pinned records) and large ones (DMA both ways); every
    record equals to_rec32 of the reference-made golden record, and the bytes
    around an in-place array are untouched.  Then the pipelined form
    (pptk_rx_batch_submit32) interleaved with 64-byte submissions in one
    queue: each completes into its own record size."""
    from pptk_amd.records import REC32_DTYPE, REC_DTYPE, to_rec32
    from pptk_amd.rx import RxContext, ldp_packets
    z = load_golden(name)
    n = len(z["off"])
    b4, b6, hs = (int(x) for x in z["iphash"])
    ctx = RxContext(0, z["key"].tobytes(), b4, b6, hs, max_batch=max_batch, max_frame=65535,
                    gather_threads=threads)
    ring = _pages(z["buf"].size + 4096)
    ring[:z["buf"].size] = z["buf"]
    pkts = ldp_packets(ring, z["off"], z["len"])
    want32 = to_rec32(z["recs"])
    region = _pages((n + 16) * 32)
    region[:] = 0x5A
    out = region[8 * 32:(8 + n) * 32].view(REC32_DTYPE)
    if mode != "staged":
        ctx.register_ring(ring)
    if mode == "ring_recs":
        ctx.register_ring(region)
    for _ in range(2):
        out[:] = np.zeros(1, dtype=REC32_DTYPE)
        got = ctx.batch_host(pkts, out=out, compact=True)
        d = diff_records(got, want32, dtype=REC32_DTYPE)
        assert not d, d
        assert (region[:8 * 32] == 0x5A).all() and (region[(8 + n) * 32:] == 0x5A).all()
    k = min(n, max_batch, 500)
    o32 = [np.zeros(k, REC32_DTYPE) for _ in range(2)]
    o64 = [np.zeros(k, REC_DTYPE) for _ in range(2)]
    for j in range(2):
        ctx.submit_host(_packet_slice(pkts, 0, k), o32[j])
        ctx.submit_host(_packet_slice(pkts, 0, k), o64[j])
    for _ in range(4):
        assert ctx.complete_host() == k
    for j in range(2):
        d = diff_records(o32[j], want32[:k], dtype=REC32_DTYPE)
        assert not d, d
        d = diff_records(o64[j], z["recs"][:k])
        assert not d, d
    ctx.close()


@pytest.mark.parametrize("layout", ["slots", "slots_swapped", "packed_odd", "scattered"])
@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("name", ["c64", "c1500"])
def test_host_batch_uniform_chunks(name, layout, compact, dev):
    """Chunks whose frames all have one length run as fixed-stride batches
    without descriptors (staged: at 16-byte-rounded offsets; registered ring:
    at the ring's own stride from the first frame).  Layouts: netmap-like
    2 KB slots in order (fixed stride); the same with two frames swapped (the
    stride breaks: descriptors again); frames packed at an odd stride; frames
    scattered (ring path impossible -> staged).  Staged and ring, small and
    large chunks, 64- and 32-byte records: every record equals the golden
    record of its frame."""
    from pptk_amd.records import REC32_DTYPE, to_rec32
    from pptk_amd.rx import RxContext, ldp_packets
    z = load_golden(name)
    n, flen = len(z["off"]), int(z["len"][0])
    frames = [z["buf"][o:o + flen] for o in z["off"].astype(np.int64)]
    order = np.arange(n)
    if layout == "slots_swapped":
        order[[5, n - 7]] = order[[n - 7, 5]]
    pitch = {"slots": 2048, "slots_swapped": 2048, "packed_odd": flen + 3, "scattered": 4096}[layout]
    ring = _pages(n * pitch + 8192)
    offs = np.arange(n, dtype=np.int64) * pitch
    if layout == "scattered":
        offs = np.random.default_rng(3).permutation(n).astype(np.int64) * pitch
    for k in range(n):
        ring[offs[k]:offs[k] + flen] = frames[order[k]]
    want = as_records(z["recs"])[order]
    if compact:
        want = to_rec32(want)
    dt = REC32_DTYPE if compact else None
    b4, b6, hs = (int(x) for x in z["iphash"])
    for max_batch in (97, 65536):
        ctx = RxContext(0, z["key"].tobytes(), b4, b6, hs, max_batch=max_batch, max_frame=65535,
                        gather_threads=4)
        pkts = ldp_packets(ring, offs, np.full(n, flen, np.uint16))
        for ring_too in (False, True):
            if ring_too:
                ctx.register_ring(ring)
            got = ctx.batch_host(pkts, compact=compact)
            d = diff_records(got, want, **({"dtype": dt} if dt is not None else {}))
            assert not d, f"{layout} max_batch {max_batch} ring {ring_too}: " + d
        ctx.close()
