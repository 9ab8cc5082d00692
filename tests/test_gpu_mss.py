"""TCP MSS clamping on the GPU (pptk_tcp_mss_clamp_device) against the
reference's tcp_parse_options + tcp_set_mss_cksum_update
(tests/golden/mss.npz), byte for byte with the per-frame status, at several
buffer misalignments; against the oracle on fresh random batches in both
layouts; and, on a large batch, the property that clamping keeps every TCP
checksum verdict of the receive transform.  Needs an MI355X."""
import numpy as np
import pytest

import framegen
from test_oracle import mss_case

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def ctx():
    from pptk_amd.rx import RxContext
    c = RxContext(0, bytes(range(1, 17)))
    yield c
    c.close()


def _clamp(ctx, buf, off, lens, mss, flags, dev, shift=0, stride=None, fixed_len=0):
    big = torch.zeros(buf.size + shift + 64, dtype=torch.uint8, device=dev)
    big[shift:shift + buf.size] = torch.from_numpy(buf).to(dev)
    frames = big[shift:]
    n = len(off) if off is not None else buf.size // stride
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    if stride is None:
        ctx.mss_clamp_device(frames, n, mss, syn_only=bool(flags & 1),
                             off=torch.from_numpy(off.view(np.int64)).to(dev),
                             lens=torch.from_numpy(lens.view(np.int16)).to(dev), status=st)
    else:
        ctx.mss_clamp_device(frames, n, mss, syn_only=bool(flags & 1), stride=stride,
                             fixed_len=fixed_len, status=st)
    torch.cuda.synchronize()
    return big, frames[:buf.size].cpu().numpy(), st.cpu().numpy()


@pytest.mark.parametrize("k", range(4))
@pytest.mark.parametrize("shift", [0, 3, 64])
def test_mss_clamp_matches_reference(ctx, k, shift, dev):
    z, buf, want, mss, flags, status = mss_case(k)
    big, got, st = _clamp(ctx, buf, z["off"], z["len"], mss, flags, dev, shift)
    assert np.array_equal(st, status)
    assert np.array_equal(got, want), int((got != want).sum())
    assert int(big[:shift].sum()) == 0 and int(big[shift + buf.size:].sum()) == 0


@pytest.mark.parametrize("seed", range(3))
def test_mss_clamp_matches_oracle_random(ctx, oracle_lib, seed, dev):
    frames = framegen.gen_mss(20000, seed=0x4000 + seed)
    buf, off, lens = framegen.pack(frames, align=(1, 2, 16)[seed])
    for mss, flags in ((1220, 0), (1400, 1)):
        want, sw = oracle_lib.mss_clamp_batch(buf, mss, flags, off=off, lens=lens)
        _, got, st = _clamp(ctx, buf, off, lens, mss, flags, dev)
        assert np.array_equal(st, sw)
        assert np.array_equal(got, want), int((got != want).sum())


def test_mss_clamp_fixed_stride(ctx, oracle_lib, dev):
    """Fixed-stride layout: 96-byte slots holding SYNs with options at both
    MSS parities (IPv4 and IPv6)."""
    rng = np.random.default_rng(77)
    fr = []
    for i in range(4096):
        opts = (b"\x01" if i & 1 else b"") + b"\x02\x04" + int(rng.integers(1000, 9000)).to_bytes(2, "big")
        opts += b"\x01" * ((-len(opts)) % 4)
        fr.append(framegen.frame_tcp_opts(rng, v6=bool(i & 2), opts=opts, payload=b""))
    stride = 96
    buf = np.zeros(len(fr) * stride, np.uint8)
    lens = set()
    for i, f in enumerate(fr):
        buf[i * stride:i * stride + len(f)] = np.frombuffer(f, np.uint8)
        lens.add(len(f))
    L = max(lens)   # frames shorter than L: Ethernet padding, excluded by the parse
    want, sw = oracle_lib.mss_clamp_batch(buf, 1200, 1, stride=stride, fixed_len=L)
    _, got, st = _clamp(ctx, buf, None, None, 1200, 1, dev, stride=stride, fixed_len=L)
    assert (sw & 4).sum() > 3000
    assert np.array_equal(st, sw) and np.array_equal(got, want)


def test_mss_clamp_keeps_verdicts_large(ctx, dev):
    """1 M random TCP/other frames: after clamping, the receive transform's
    records are unchanged except for frames it clamped, which still verify."""
    from pptk_amd.records import F_L4_OK, MSS_ST_CLAMPED, as_records
    frames = framegen.gen_mss(1 << 16, seed=0x5151)
    buf, off, lens = framegen.pack(frames, align=1)
    rep = 16
    big = np.concatenate([buf] * rep)
    offs = np.concatenate([off + np.uint64(r * buf.size) for r in range(rep)])
    ln = np.concatenate([lens] * rep)
    d = torch.from_numpy(big).to(dev)
    o = torch.from_numpy(offs.view(np.int64)).to(dev)
    l = torch.from_numpy(ln.view(np.int16)).to(dev)
    n = len(offs)
    before = as_records(ctx.batch_device(d, n, off=o, lens=l, max_len=int(ln.max())).cpu().numpy().reshape(-1))
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    ctx.mss_clamp_device(d, n, 1100, off=o, lens=l, status=st)
    after = as_records(ctx.batch_device(d, n, off=o, lens=l, max_len=int(ln.max())).cpu().numpy().reshape(-1))
    s = st.cpu().numpy()
    cl = (s & MSS_ST_CLAMPED) != 0
    assert cl.sum() > 100000
    assert np.array_equal(before["flags"] & F_L4_OK, after["flags"] & F_L4_OK)
    assert np.array_equal(before[~cl], after[~cl])


def test_mss_clamp_rejects_bad_args(ctx, dev):
    frames = torch.zeros(128, dtype=torch.uint8, device=dev)
    with pytest.raises(OSError):
        ctx.mss_clamp_device(frames, 2, 1200, stride=0)      # no layout
    from pptk_amd.rx import _dp
    rc = ctx._L.pptk_tcp_mss_clamp_device(ctx._ctx, _dp(frames), None, None, 64, 64, 2, 1200, 2,
                                          None, None)
    assert rc == -22                                          # unknown flag bit
