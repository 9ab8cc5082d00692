"""Batched ip_permitted / ipv6_permitted on the GPU (pptk_rx_permit_device,
pptk_rx_tokens_refill_device) against the reference's own rate limiter
(tests/golden/permit.npz, made by calling ip_permitted once per frame in
frame order) and, for long chains and large batches, against the C
restatement pinned to it (tests/test_oracle.py).  Needs an MI355X."""
import numpy as np
import pytest

from conftest import load_golden
from pptk_amd.records import REC32_DTYPE, REC_DTYPE, diff_records, to_rec32

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


PERMIT_PASSES = 0x400   # PPTK_RX_TUNE_PERMIT_PASSES: the four-launch path
_PATH = ["fused"]


@pytest.fixture(params=["fused", "passes"], autouse=True)
def permit_path(request):
    """Every test runs on both rate-limiter paths: the one-launch fused
    kernel (the default wherever it applies) and the four-launch path."""
    _PATH[0] = request.param
    yield request.param


def _ctx(z):
    from pptk_amd.rx import RxContext
    b4, b6, hs = (int(x) for x in z["iphash"])
    ctx = RxContext(0, z["key"].tobytes(), b4, b6, hs)
    if _PATH[0] == "passes":
        ctx.set_tuning(-1, PERMIT_PASSES)
    return ctx


def _gpu_records(ctx, z, dev, compact=False):
    frames = torch.zeros(z["buf"].size + 64, dtype=torch.uint8, device=dev)
    frames[:z["buf"].size] = torch.from_numpy(z["buf"]).to(dev)
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    recs = ctx.batch_device(frames, len(z["off"]), off=off, lens=lens, max_len=int(z["len"].max()),
                            compact=compact)
    torch.cuda.synchronize()
    return recs


@pytest.mark.parametrize("compact", [False, True])
def test_permit_matches_reference(compact, dev):
    """Records from the GPU rx transform, then the GPU rate limiter: every
    verdict and every bucket's tokens as the reference's per-frame calls."""
    z = load_golden("permit")
    ctx = _ctx(z)
    recs = _gpu_records(ctx, z, dev, compact)
    want = z["recs"].reshape(-1).view(REC_DTYPE)
    got = recs.cpu().numpy().reshape(-1)
    d = (diff_records(got, to_rec32(want), dtype=REC32_DTYPE) if compact
         else diff_records(got, want))
    assert not d, d
    for k, (fam, init, has_subj) in enumerate(z["case_meta"]):
        tok = torch.from_numpy(z["case_tok_in"][k].view(np.int32).copy()).to(dev)
        subj = torch.from_numpy(z["case_subject"][k]).to(dev) if has_subj else None
        v = ctx.permit_device(recs, int(fam), tok, subject=subj, compact=compact)
        torch.cuda.synchronize()
        assert np.array_equal(v.cpu().numpy(), z["case_verdict"][k]), (fam, init, has_subj)
        assert np.array_equal(tok.cpu().numpy().view(np.uint32), z["case_tok_out"][k])


def test_refill_matches_reference(dev):
    z = load_golden("permit")
    ctx = _ctx(z)
    for (init, add, lo, hi), tin, tout in zip(z["refill_meta"], z["refill_in"], z["refill_out"]):
        tok = torch.from_numpy(tin.view(np.int32).copy()).to(dev)
        ctx.tokens_refill_device(tok, int(lo), int(hi), int(add), int(init))
        torch.cuda.synchronize()
        assert np.array_equal(tok.cpu().numpy().view(np.uint32), tout)


def test_permit_chain_with_refills(dev):
    """Five batches with timer refills in between, one token array carried
    through: identical to the frame-by-frame restatement."""
    from oracle.oracle import Oracle
    z = load_golden("permit")
    ctx = _ctx(z)
    recs = _gpu_records(ctx, z, dev)
    host = z["recs"].reshape(-1).view(REC_DTYPE)
    O = Oracle()
    hs, init = int(z["iphash"][2]), 40
    tok_h = np.full(hs, init, np.uint32)
    tok = torch.from_numpy(tok_h.view(np.int32).copy()).to(dev)
    n = len(host)
    cuts = [0, 100, 900, 1500, 2999, n]
    for step, (a, b) in enumerate(zip(cuts, cuts[1:])):
        v = ctx.permit_device(recs[a:b], 4 if step % 2 == 0 else 6, tok)
        vh, tok_h = O.permit_batch(host[a:b], 4 if step % 2 == 0 else 6, None, tok_h)
        torch.cuda.synchronize()
        assert np.array_equal(v.cpu().numpy(), vh), step
        lo = (step * 16) % hs
        ctx.tokens_refill_device(tok, lo, lo + 16, 3, init)
        tok_h = O.tokens_refill(tok_h, lo, lo + 16, 3, init)
        torch.cuda.synchronize()
        assert np.array_equal(tok.cpu().numpy().view(np.uint32), tok_h), step


def test_permit_large_skewed_batch(dev):
    """1 M synthetic records, Zipf-skewed buckets (one bucket holds ~10 % of
    the frames), 2^16 buckets: GPU == frame-by-frame restatement."""
    from oracle.oracle import Oracle
    from pptk_amd.records import F_IPV6, F_PARSED
    rng = np.random.default_rng(11)
    n, hs = 1 << 20, 1 << 16
    r = np.zeros(n, dtype=REC_DTYPE)
    r["flags"] = np.where(rng.random(n) < 0.97, F_PARSED, 0) | np.where(rng.random(n) < 0.2,
                                                                        F_IPV6, 0)
    r["src_bucket"] = np.minimum(rng.zipf(1.3, n) - 1, hs - 1)
    tok_h = rng.integers(0, 500, hs).astype(np.uint32)
    subj = (rng.random(n) < 0.9).astype(np.uint8)
    ctx = _ctx({"key": np.arange(1, 17, dtype=np.uint8), "iphash": np.array([24, 48, hs])})
    recs = torch.from_numpy(r.view(np.uint8).reshape(n, 64)).to(dev)
    tok = torch.from_numpy(tok_h.view(np.int32).copy()).to(dev)
    v = ctx.permit_device(recs, 4, tok, subject=torch.from_numpy(subj).to(dev))
    vh, th = Oracle().permit_batch(r, 4, subj, tok_h)
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), vh)
    assert np.array_equal(tok.cpu().numpy().view(np.uint32), th)
    assert (vh == 0).sum() > 1000 and (vh == 1).sum() > 1000


def test_permit_rejects_disabled_family(dev):
    ctx = _ctx({"key": np.zeros(16, np.uint8), "iphash": np.array([24, 0, 64])})
    recs = torch.zeros((4, 64), dtype=torch.uint8, device=dev)
    tok = torch.zeros(64, dtype=torch.int32, device=dev)
    with pytest.raises(OSError):
        ctx.permit_device(recs, 6, tok)


@pytest.mark.parametrize("n", [(1 << 20) + 3, 4097])
def test_permit_ragged_batch_unaligned_verdicts(n, dev):
    """A frame count that is not a multiple of 4 (the bounds and verdict
    passes take four frames per thread, the ragged rest one by one), on the
    onesweep (> 1 M) and the small-batch sort paths, into a verdict array
    that starts at an odd address (byte stores instead of 4-byte ones):
    GPU == frame-by-frame restatement."""
    from oracle.oracle import Oracle
    from pptk_amd.records import F_IPV6, F_PARSED
    rng = np.random.default_rng(n)
    hs = 1 << 16
    r = np.zeros(n, dtype=REC_DTYPE)
    r["flags"] = np.where(rng.random(n) < 0.95, F_PARSED, 0) | np.where(rng.random(n) < 0.1,
                                                                        F_IPV6, 0)
    r["src_bucket"] = np.minimum(rng.zipf(1.5, n) - 1, hs - 1)
    tok_h = rng.integers(0, 50, hs).astype(np.uint32)
    ctx = _ctx({"key": np.arange(1, 17, dtype=np.uint8), "iphash": np.array([24, 48, hs])})
    recs = torch.from_numpy(r.view(np.uint8).reshape(n, 64)).to(dev)
    tok = torch.from_numpy(tok_h.view(np.int32).copy()).to(dev)
    vbuf = torch.full((n + 8,), 0xEE, dtype=torch.uint8, device=dev)
    v = ctx.permit_device(recs, 4, tok, verdict=vbuf[1:n + 1])
    vh, th = Oracle().permit_batch(r, 4, None, tok_h)
    torch.cuda.synchronize()
    got = vbuf.cpu().numpy()
    assert np.array_equal(got[1:n + 1], vh)
    assert got[0] == 0xEE and (got[n + 1:] == 0xEE).all()
    assert np.array_equal(tok.cpu().numpy().view(np.uint32), th)
    assert v.data_ptr() == vbuf.data_ptr() + 1


def _dense_keys(r):
    """The d_key encoding (include/pptk_rx.h) of host records r."""
    from pptk_amd.records import F_IPV6, F_PARSED
    k = r["src_bucket"].astype(np.uint32)
    k = np.where(r["flags"] & F_IPV6, k | np.uint32(0x80000000), k)
    return np.where(r["flags"] & F_PARSED, k, np.uint32(0xFFFFFFFF)).astype(np.uint32)


def test_dense_keys_written_by_rx_and_permit_from_keys(dev):
    """pptk_rx_dev_batch.d_key: the rx kernel's dense keys equal the encoding
    of the golden records, and pptk_rx_permit_keys_device on them gives the
    reference's verdicts and tokens for every golden case."""
    z = load_golden("permit")
    ctx = _ctx(z)
    n = len(z["off"])
    frames = torch.zeros(z["buf"].size + 64, dtype=torch.uint8, device=dev)
    frames[:z["buf"].size] = torch.from_numpy(z["buf"]).to(dev)
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.batch_device(frames, n, off=off, lens=lens, max_len=int(z["len"].max()), key_out=keys)
    torch.cuda.synchronize()
    want = z["recs"].reshape(-1).view(REC_DTYPE)
    assert np.array_equal(keys.cpu().numpy().view(np.uint32), _dense_keys(want))
    for k, (fam, init, has_subj) in enumerate(z["case_meta"]):
        tok = torch.from_numpy(z["case_tok_in"][k].view(np.int32).copy()).to(dev)
        subj = torch.from_numpy(z["case_subject"][k]).to(dev) if has_subj else None
        v = ctx.permit_keys_device(keys, int(fam), tok, subject=subj)
        torch.cuda.synchronize()
        assert np.array_equal(v.cpu().numpy(), z["case_verdict"][k]), (fam, init, has_subj)
        assert np.array_equal(tok.cpu().numpy().view(np.uint32), z["case_tok_out"][k])


@pytest.mark.parametrize("case", ["heavy_hitter", "all_over_budget", "mixed_v6", "big_table",
                                  "tiny_table"])
def test_permit_regimes_against_oracle(case, dev):
    """The block-histogram path in the regimes that exercise its resolve
    pass (one bucket holding most frames and running out inside a late block;
    every bucket over budget; IPv6 with a subject mask), the sort fallback
    (hash_size 2^17) and a 2-bucket table, on records and on dense keys: GPU ==
    frame-by-frame restatement."""
    from oracle.oracle import Oracle
    from pptk_amd.records import F_IPV6, F_PARSED
    rng = np.random.default_rng(sum(case.encode()))
    n = (3 << 20) + 17
    hs = {"big_table": 1 << 17, "tiny_table": 2}.get(case, 1 << 16)
    r = np.zeros(n, dtype=REC_DTYPE)
    fam = 6 if case == "mixed_v6" else 4
    r["flags"] = np.where(rng.random(n) < 0.97, F_PARSED, 0) | np.where(
        rng.random(n) < (0.6 if fam == 6 else 0.1), F_IPV6, 0)
    if case == "heavy_hitter":
        b = np.where(rng.random(n) < 0.9, 7, rng.integers(0, hs, n))
        tok_h = rng.integers(0, 40, hs).astype(np.uint32)
        tok_h[7] = 2_000_000            # runs out inside a late histogram block
    elif case == "all_over_budget":
        b = rng.integers(0, hs, n)
        tok_h = rng.integers(0, 30, hs).astype(np.uint32)
    else:
        b = np.minimum(rng.zipf(1.2, n) - 1, hs - 1)
        tok_h = rng.integers(0, 300, hs).astype(np.uint32)
    r["src_bucket"] = b
    subj = (rng.random(n) < 0.8).astype(np.uint8) if case == "mixed_v6" else None
    ctx = _ctx({"key": np.arange(1, 17, dtype=np.uint8), "iphash": np.array([24, 48, hs])})
    vh, th = Oracle().permit_batch(r, fam, subj, tok_h)
    assert (vh == 0).sum() > 100 and (vh == 1).sum() > 100
    sub_t = None if subj is None else torch.from_numpy(subj).to(dev)
    for via_keys in (False, True):
        tok = torch.from_numpy(tok_h.view(np.int32).copy()).to(dev)
        if via_keys:
            keys = torch.from_numpy(_dense_keys(r).view(np.int32)).to(dev)
            v = ctx.permit_keys_device(keys, fam, tok, subject=sub_t)
        else:
            recs = torch.from_numpy(r.view(np.uint8).reshape(n, 64)).to(dev)
            v = ctx.permit_device(recs, fam, tok, subject=sub_t)
        torch.cuda.synchronize()
        assert np.array_equal(v.cpu().numpy(), vh), via_keys
        assert np.array_equal(tok.cpu().numpy().view(np.uint32), th), via_keys


def _np_permit(k, hs, tok):
    """Frame-by-frame ip_permitted semantics on subject keys k (bucket, or
    -1: not a subject), vectorised: the rank of each frame among the earlier
    frames of its bucket (stable sort) against the bucket's tokens."""
    k = k.astype(np.int64)
    subj = k >= 0
    idx = np.nonzero(subj)[0]
    kb = k[idx]
    order = np.argsort(kb, kind="stable")
    sk = kb[order]
    start = np.searchsorted(sk, sk, side="left")
    rank = np.empty(len(idx), np.int64)
    rank[order] = np.arange(len(idx)) - start
    v = np.full(len(k), 2, np.uint8)
    v[idx] = (rank < tok[kb].astype(np.int64)).astype(np.uint8)
    cnt = np.bincount(kb, minlength=hs).astype(np.int64)
    t2 = (tok.astype(np.int64) - np.minimum(tok.astype(np.int64), cnt)).astype(np.uint32)
    return v, t2


def test_np_permit_matches_oracle():
    """The vectorised restatement used below equals the C restatement (which
    is pinned to the reference's own calls, tests/test_oracle.py)."""
    from oracle.oracle import Oracle
    from pptk_amd.records import F_PARSED
    rng = np.random.default_rng(5)
    n, hs = 200_000, 1 << 12
    r = np.zeros(n, dtype=REC_DTYPE)
    r["flags"] = np.where(rng.random(n) < 0.9, F_PARSED, 0)
    r["src_bucket"] = np.minimum(rng.zipf(1.3, n) - 1, hs - 1)
    tok = rng.integers(0, 60, hs).astype(np.uint32)
    vh, th = Oracle().permit_batch(r, 4, None, tok)
    k = np.where(r["flags"] & F_PARSED, r["src_bucket"].astype(np.int64), -1)
    v, t = _np_permit(k, hs, tok)
    assert np.array_equal(v, vh) and np.array_equal(t, th)


@pytest.mark.parametrize("case", ["whole_segment", "spread", "bunched"])
def test_permit_keys_full_size(case, dev):
    """16 M dense keys (BASELINE's C64 batch size: one 65 536-frame segment
    per CU on the fused path).  whole_segment: the first segment is one
    bucket throughout (its u16 histogram counter wraps: the fused kernel
    detects it) with the bucket's T_b-th frame inside it, and a second
    bucket whose budget ends in a late segment; spread: 2^16 buckets, random
    budgets, half the frames denied (few boundary frames per segment: the
    fused kernel ranks them in its LDS hash table); bunched: every bucket's
    budget 128 of its ~256 frames, so the boundaries crowd into the middle
    segments (more candidates than the hash table takes there: the ordered
    walk; the hash table elsewhere) -- bench.py's keys_denying.  GPU ==
    restatement, both paths."""
    rng = np.random.default_rng({"spread": 77, "whole_segment": 78, "bunched": 79}[case])
    n, hs = 1 << 24, 1 << 16
    k = rng.integers(0, hs, n).astype(np.int64)
    k[rng.random(n) < 0.02] = -1
    if case == "whole_segment":
        k[rng.random(n) < 0.3] = 9
        k[:65536] = 5                    # last: the first segment is bucket 5 throughout
        tok = rng.integers(0, 400, hs).astype(np.uint32)
        tok[5] = 30000
        tok[9] = 4_000_000
    elif case == "spread":
        tok = rng.integers(0, 256, hs).astype(np.uint32)
    else:
        tok = np.full(hs, 128, np.uint32)
    v_want, t_want = _np_permit(k, hs, tok)
    assert (v_want == 0).sum() > 1000 and (v_want == 1).sum() > 1000
    ctx = _ctx({"key": np.arange(1, 17, dtype=np.uint8), "iphash": np.array([24, 48, hs])})
    keys = torch.from_numpy(np.where(k >= 0, k, 0xFFFFFFFF).astype(np.uint32).view(np.int32)).to(dev)
    tokt = torch.from_numpy(tok.view(np.int32).copy()).to(dev)
    v = ctx.permit_keys_device(keys, 4, tokt)
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), v_want)
    assert np.array_equal(tokt.cpu().numpy().view(np.uint32), t_want)


def test_permit_keys_hash_class_overflow_falls_back(dev):
    """The fused kernel's hash-table ranking takes a segment's candidates in
    bucket-class passes of at most 2 048; a class over that (3 000
    candidates, every one of a bucket in class 0 of two passes: the same
    multiplicative hash as rx_permit.hip's cls) must fall back to the
    ordered walk with the same verdicts.  The first segment holds three
    frames each of 1 000 such buckets (one token each: the first frame
    permitted, the others denied; at 1 M frames a segment is 4 096 frames),
    the rest is non-subject filler; later segments hold random keys."""
    rng = np.random.default_rng(81)
    n, hs = 1 << 20, 1 << 16
    b = np.arange(hs, dtype=np.uint64)
    cls2 = (((((b * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)) >> np.uint64(8)) & np.uint64(0xFFFF))
            * np.uint64(2)) >> np.uint64(16)
    S = np.nonzero(cls2 == 0)[0][:1000].astype(np.int64)
    k = rng.integers(0, hs, n).astype(np.int64)
    sl = n // 256                                  # the fused kernel's segment at this n
    seg = np.full(sl, -1, np.int64)
    seg[rng.permutation(sl)[:3000]] = np.repeat(S, 3)[rng.permutation(3000)]
    k[:sl] = seg
    rest = k[sl:]
    rest[np.isin(rest, S)] = -1                    # S's frames only in the first segment
    tok = np.full(hs, 1 << 20, np.uint32)
    tok[S] = 1
    v_want, t_want = _np_permit(k, hs, tok)
    assert (v_want[:sl] == 0).sum() == 2000 and (v_want[:sl] == 1).sum() == 1000
    ctx = _ctx({"key": np.arange(1, 17, dtype=np.uint8), "iphash": np.array([24, 48, hs])})
    keys = torch.from_numpy(np.where(k >= 0, k, 0xFFFFFFFF).astype(np.uint32).view(np.int32)).to(dev)
    tokt = torch.from_numpy(tok.view(np.int32).copy()).to(dev)
    v = ctx.permit_keys_device(keys, 4, tokt)
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), v_want)
    assert np.array_equal(tokt.cpu().numpy().view(np.uint32), t_want)


def test_permit_keys_out_of_range_are_not_subjects(dev):
    """Caller-made keys whose bucket is >= iphash_size are not subjects:
    verdict 2, no token touched (they used to index past the tables)."""
    rng = np.random.default_rng(3)
    n, hs = 300_001, 1 << 10
    kr = rng.integers(0, 4 * hs, n).astype(np.int64)
    tok = rng.integers(0, 100, hs).astype(np.uint32)
    v_want, t_want = _np_permit(np.where(kr < hs, kr, -1), hs, tok)
    ctx = _ctx({"key": np.arange(1, 17, dtype=np.uint8), "iphash": np.array([24, 48, hs])})
    keys = torch.from_numpy(kr.astype(np.uint32).view(np.int32)).to(dev)
    tokt = torch.from_numpy(tok.view(np.int32).copy()).to(dev)
    v = ctx.permit_keys_device(keys, 4, tokt)
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), v_want)
    assert np.array_equal(tokt.cpu().numpy().view(np.uint32), t_want)


ETIMEDOUT = 110


def _keys_case(n, hs, seed):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, hs, n).astype(np.int64)
    k[rng.random(n) < 0.02] = -1
    tok = rng.integers(0, 2 * n // hs, hs).astype(np.uint32)     # ~half denied
    keys = np.where(k >= 0, k, 0xFFFFFFFF).astype(np.uint32)
    return k, tok, keys


def test_permit_keys_two_contexts_two_streams_at_once(dev):
    """Two rx queues on one GPU (a context each, as ldp/ldprecvmt.c:16-67
    runs one thread per queue) issue the rate limiter on two streams at the
    same time, four batches each with their own token arrays.  The fused
    launches need every workgroup resident; two of them at once could split
    the CUs and each wait for the other's: the library orders
    them, so both chains equal the frame-by-frame semantics, no launch
    aborts (status 0 on both scratch buffers) and nothing waits out the
    2 s barrier bound."""
    import time
    n, hs, reps = 1 << 22, 1 << 16, 4
    cases = [_keys_case(n, hs, 91 + i) for i in range(2)]
    want = []
    for k, tok, _ in cases:
        t, vs = tok, []
        for _ in range(reps):
            v, t = _np_permit(k, hs, t)
            vs.append(v)
        want.append((vs, t))
    ctxs = [_ctx({"key": np.arange(1, 17, dtype=np.uint8), "iphash": np.array([24, 48, hs])})
            for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    keys = [torch.from_numpy(c[2].view(np.int32)).to(dev) for c in cases]
    toks = [torch.from_numpy(c[1].view(np.int32).copy()).to(dev) for c in cases]
    scratch = [torch.empty(ctxs[0]._L.pptk_rx_permit_scratch_bytes(n, hs), dtype=torch.uint8,
                           device=dev) for _ in range(2)]
    verdicts = [[torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(reps)]
                for _ in range(2)]
    torch.cuda.synchronize()
    t0 = time.monotonic()
    for r in range(reps):
        for i in range(2):
            ctxs[i].permit_keys_device(keys[i], 4, toks[i], verdict=verdicts[i][r],
                                       scratch=scratch[i], stream=streams[i])
    torch.cuda.synchronize()
    took = time.monotonic() - t0
    for i in range(2):
        assert ctxs[i].permit_status(scratch[i], stream=streams[i]) == 0
        for r in range(reps):
            assert np.array_equal(verdicts[i][r].cpu().numpy(), want[i][0][r]), (i, r)
        assert np.array_equal(toks[i].cpu().numpy().view(np.uint32), want[i][1]), i
    assert took < 1.5, took


def test_permit_beside_oversubscribed_batches(dev):
    """The rate limiter on one stream while another context's receive
    batches run on another: offset-described (CMIX) and C64 batches launch
    more blocks than fit (rx_capi.hip grid_for), so the dispatcher hands CUs
    back and forth between the two kernels instead of one waiting for the
    other to end.  The fused launch needs all its workgroups resident at
    once; it must still get them well inside its 2 s bound: no abort
    (status 0), verdicts and tokens equal to the frame-by-frame semantics,
    and the batches' records equal to the same batches run alone."""
    import time
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    n, hs, reps = 1 << 22, 1 << 16, 6
    k, tok_h, keys_h = _keys_case(n, hs, 93)
    want_v, t = [], tok_h
    for _ in range(reps):
        v, t = _np_permit(k, hs, t)
        want_v.append(v)
    pctx = _ctx({"key": np.arange(1, 17, dtype=np.uint8), "iphash": np.array([24, 48, hs])})
    rctx = RxContext(0, bytes(range(1, 17)))
    batches = [make_batch(cfg, 1 << 22, dev) for cfg in ("cmix", "c64")]
    kws = [dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]) if "off" in b else
           dict(stride=b["stride"], fixed_len=b["fixed_len"]) for b in batches]
    alone = [rctx.batch_device(b["frames"], 1 << 22, **kw) for b, kw in zip(batches, kws)]
    torch.cuda.synchronize()
    s_rx, s_pm = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    keys = torch.from_numpy(keys_h.view(np.int32)).to(dev)
    tok = torch.from_numpy(tok_h.view(np.int32).copy()).to(dev)
    scratch = torch.empty(pctx._L.pptk_rx_permit_scratch_bytes(n, hs), dtype=torch.uint8,
                          device=dev)
    verdicts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(reps)]
    outs = [[torch.empty_like(a) for a in alone] for _ in range(reps)]
    torch.cuda.synchronize()
    t0 = time.monotonic()
    for r in range(reps):
        for b, kw, o in zip(batches, kws, outs[r]):
            rctx.batch_device(b["frames"], 1 << 22, recs=o, stream=s_rx, **kw)
        pctx.permit_keys_device(keys, 4, tok, verdict=verdicts[r], scratch=scratch, stream=s_pm)
    torch.cuda.synchronize()
    took = time.monotonic() - t0
    assert pctx.permit_status(scratch, stream=s_pm) == 0
    for r in range(reps):
        assert np.array_equal(verdicts[r].cpu().numpy(), want_v[r]), r
        for a, o in zip(alone, outs[r]):
            assert torch.equal(a, o), r
    assert np.array_equal(tok.cpu().numpy().view(np.uint32), t)
    assert took < 1.5, took
    rctx.close()
    pctx.close()


@pytest.mark.parametrize("stall_at", [1, 2])
def test_permit_fused_abort_leaves_tokens_and_reports(dev, monkeypatch, stall_at):
    """Fault injection (the test build of the library, PPTK_RX_TEST_HOOKS):
    one workgroup of the fused launch is held 600 ms before grid barrier
    `stall_at` while the others' barrier gives up after 200 ms.  The launch
    aborts: pptk_rx_permit_status reports -ETIMEDOUT, the token array is
    exactly as before the call (the commit comes after the last barrier) and
    the launch fails closed (every subject frame's verdict 0, the reference's
    iphash/iphash.c:164-196 never admits without a token).
    The same call repeated without the stall gives the frame-by-frame
    verdicts and tokens, and status 0."""
    from conftest import HOOKS_LIB
    from pptk_amd.rx import RxContext
    if _PATH[0] == "passes":
        pytest.skip("the four-launch path has no grid barrier")
    n, hs = 1 << 20, 1 << 16
    k, tok_h, keys_h = _keys_case(n, hs, 97)
    v_want, t_want = _np_permit(k, hs, tok_h)
    ctx = RxContext(0, bytes(range(1, 17)), 24, 48, hs, lib_path=HOOKS_LIB)
    keys = torch.from_numpy(keys_h.view(np.int32)).to(dev)
    tok = torch.from_numpy(tok_h.view(np.int32).copy()).to(dev)
    scratch = torch.empty(ctx._L.pptk_rx_permit_scratch_bytes(n, hs), dtype=torch.uint8,
                          device=dev)
    monkeypatch.setenv("PPTK_RX_TEST_PERMIT_STALL_MS", "600")
    monkeypatch.setenv("PPTK_RX_TEST_PERMIT_SPIN_MS", "200")
    monkeypatch.setenv("PPTK_RX_TEST_PERMIT_STALL_AT", str(stall_at))
    v = ctx.permit_keys_device(keys, 4, tok, scratch=scratch)
    assert ctx.permit_status(scratch) == -ETIMEDOUT
    assert np.array_equal(tok.cpu().numpy().view(np.uint32), tok_h)
    # fails closed: every subject frame denied, the others "not a subject"
    assert np.array_equal(v.cpu().numpy(), np.where(k >= 0, 0, 2).astype(np.uint8))
    for name in ("PPTK_RX_TEST_PERMIT_STALL_MS", "PPTK_RX_TEST_PERMIT_SPIN_MS",
                 "PPTK_RX_TEST_PERMIT_STALL_AT"):
        monkeypatch.delenv(name)
    assert ctx.permit_status(scratch) == 0          # (queried: nothing since)
    v = ctx.permit_keys_device(keys, 4, tok, scratch=scratch)
    assert ctx.permit_status(scratch) == 0
    assert np.array_equal(v.cpu().numpy(), v_want)
    assert np.array_equal(tok.cpu().numpy().view(np.uint32), t_want)
    ctx.close()


def test_permit_fused_commit_decision_is_agreed(dev, monkeypatch):
    """the last workgroup is held before barrier 2 (the commit
    point) for 20 ms while the others wait there for 20 ms + delta, delta
    stepping through -40 .. +60 us in 2-us steps (51 launches; the outcome
    flipped between +0 and +20 us in a coarser sweep), so the held
    workgroup's arrival lands before, at and after their deadlines:
    across the sweep the outcome flips from abort to commit, and the
    launches at the flip race the decision.  Whatever each launch decides,
    all workgroups act on the one decision word: either status 0 with the
    frame-by-frame verdicts and tokens (chained through the launches), or
    -ETIMEDOUT with the tokens exactly as before that launch and every
    subject denied -- never some buckets committed and others not."""
    from conftest import HOOKS_LIB
    from pptk_amd.rx import RxContext
    if _PATH[0] == "passes":
        pytest.skip("the four-launch path has no grid barrier")
    n, hs = 1 << 20, 1 << 16
    k, tok_h, keys_h = _keys_case(n, hs, 98)
    ctx = RxContext(0, bytes(range(1, 17)), 24, 48, hs, lib_path=HOOKS_LIB)
    keys = torch.from_numpy(keys_h.view(np.int32)).to(dev)
    tok = torch.from_numpy(tok_h.view(np.int32).copy()).to(dev)
    scratch = torch.empty(ctx._L.pptk_rx_permit_scratch_bytes(n, hs), dtype=torch.uint8,
                          device=dev)
    monkeypatch.setenv("PPTK_RX_TEST_PERMIT_STALL_US", "20000")
    monkeypatch.setenv("PPTK_RX_TEST_PERMIT_STALL_AT", "2")
    t_cur = tok_h.copy()
    outcomes = []
    denied = np.where(k >= 0, 0, 2).astype(np.uint8)
    cap = np.uint32(2 * n // hs)
    for delta in range(-40, 61, 2):
        monkeypatch.setenv("PPTK_RX_TEST_PERMIT_SPIN_US", str(20000 + delta))
        v = ctx.permit_keys_device(keys, 4, tok, scratch=scratch)
        st = ctx.permit_status(scratch)
        got_t = tok.cpu().numpy().view(np.uint32)
        got_v = v.cpu().numpy()
        if st == 0:
            v_want, t_next = _np_permit(k, hs, t_cur)
            assert np.array_equal(got_v, v_want), delta
            assert np.array_equal(got_t, t_next), delta
            t_cur = t_next
        else:
            assert st == -ETIMEDOUT
            assert np.array_equal(got_t, t_cur), delta
            assert np.array_equal(got_v, denied), delta
        outcomes.append((delta, "C" if st == 0 else "A"))
        # a refill, so later launches still hold buckets that run out and some that do not
        t_cur = np.minimum(t_cur + np.uint32(3), cap).astype(np.uint32)
        tok.copy_(torch.from_numpy(t_cur.view(np.int32).copy()).to(dev))
    print("delta us -> outcome: " + " ".join(f"{d}{o}" for d, o in outcomes))
    ctx.close()
