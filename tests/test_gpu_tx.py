"""Tx-side checksum setting on the GPU (pptk_tx_cksum_device) against the
reference's ip_set_hdr_cksum_calc / tcp/udp(6)_set_cksum_calc
(tests/golden/tx.npz), byte for byte, in both layouts, every kernel variant,
and round-tripped through the receive transform.  Needs an MI355X."""
import numpy as np
import pytest

from conftest import load_golden
from pptk_amd.records import F_IP_OK, F_IPV6, F_L4, F_L4_OK, F_MALFORMED, F_PARSED

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SETS = ["edge", "fuzz", "cmix", "c64"]


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _case(name):
    z = load_golden(name)
    t = load_golden("tx")
    pos = t[f"{name}_pos"].astype(np.int64)
    buf_in = z["buf"].copy()
    buf_in[pos] = t[f"{name}_in"]
    buf_out = buf_in.copy()
    buf_out[pos] = t[f"{name}_out"]
    return z, buf_in, buf_out


def _ctx():
    from pptk_amd.rx import RxContext
    return RxContext(0, bytes(range(1, 17)))


def _tx(ctx, z, buf, dev, shift, stride=None):
    big = torch.zeros(buf.size + shift + 64, dtype=torch.uint8, device=dev)
    big[shift:shift + buf.size] = torch.from_numpy(buf).to(dev)
    frames = big[shift:]
    n = len(z["off"])
    if stride is None:
        ctx.tx_cksum_device(frames, n, off=torch.from_numpy(z["off"].view(np.int64)).to(dev),
                            lens=torch.from_numpy(z["len"].view(np.int16)).to(dev),
                            max_len=int(z["len"].max()))
    else:
        ctx.tx_cksum_device(frames, n, stride=stride, fixed_len=int(z["len"][0]))
    torch.cuda.synchronize()
    return big, frames


@pytest.mark.parametrize("name", SETS)
@pytest.mark.parametrize("shift", [0, 3, 8, 64])
def test_tx_matches_reference(name, shift, dev):
    z, buf_in, buf_out = _case(name)
    big, frames = _tx(_ctx(), z, buf_in, dev, shift)
    got = frames[:buf_in.size].cpu().numpy()
    bad = np.nonzero(got != buf_out)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"
    # nothing outside the frame buffer is touched
    assert not big[:shift].any().item() and not frames[buf_in.size:].any().item()


@pytest.mark.parametrize("shift", [0, 5, 6])
def test_tx_fixed_stride(shift, dev):
    """Fixed-stride batches run in two passes (streaming pass -> side array
    -> field writes; 16-bit stores at even addresses, byte stores at odd
    ones): every variant, even and odd frame addresses."""
    from pptk_amd.rx import lib
    z, buf_in, buf_out = _case("c64")
    assert np.all(z["off"] == np.arange(len(z["off"]), dtype=np.uint64) * 64)
    ctx = _ctx()
    for v in [-1] + list(range(lib().pptk_rx_variant_count())):
        ctx.set_tuning(v, -1 if v < 0 else v % 4)
        big, frames = _tx(ctx, z, buf_in, dev, shift, stride=64)
        assert np.array_equal(frames[:buf_in.size].cpu().numpy(), buf_out), f"variant {v}"
        assert not big[:shift].any().item() and not frames[buf_in.size:].any().item()


def test_tx_c1500_fixed_stride_vs_oracle(dev):
    """20 000 C1500 frames (fixed stride 1500, ~1 % corrupted checksums)
    through the two-pass tx against the CPU restatement's tx_batch, twice
    (the second call reuses the context's side array)."""
    from oracle.oracle import Oracle
    from harness.synth import make_batch
    n = 20_000
    b = make_batch("c1500", n, dev)
    host = b["frames"][: n * 1500].cpu().numpy().copy()
    want = Oracle().tx_batch(host, stride=1500, fixed_len=1500, n=n)
    assert (want != host).any()
    ctx = _ctx()
    for _ in range(2):
        fr = torch.from_numpy(host).to(dev)
        ctx.tx_cksum_device(fr, n, stride=1500, fixed_len=1500)
        torch.cuda.synchronize()
        assert np.array_equal(fr.cpu().numpy(), want)


def test_tx_every_variant(dev):
    from pptk_amd.rx import lib
    z, buf_in, buf_out = _case("cmix")
    ctx = _ctx()
    for v in range(lib().pptk_rx_variant_count()):
        ctx.set_tuning(v, v % 4)
        _, frames = _tx(ctx, z, buf_in, dev, 0 if v % 2 else 1)
        got = frames[:buf_in.size].cpu().numpy()
        assert np.array_equal(got, buf_out), f"variant {v}"


@pytest.mark.parametrize("name", ["edge", "cmix"])
def test_tx_then_rx_verifies(name, dev):
    """Set on the GPU, verify on the GPU: every parsed IPv4 header and every
    L4 header checks out."""
    z, buf_in, _ = _case(name)
    ctx = _ctx()
    _, frames = _tx(ctx, z, buf_in, dev, 0)
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    recs = ctx.batch_device(frames, len(z["off"]), off=off, lens=lens, max_len=65535)
    torch.cuda.synchronize()
    fl = recs.view(torch.int16)[:, 27].cpu().numpy().astype(np.int64) & 0xFFFF
    v4 = ((fl & F_PARSED) != 0) & ((fl & F_MALFORMED) == 0) & ((fl & F_IPV6) == 0)
    assert v4.sum() > 10 and ((fl[v4] & F_IP_OK) != 0).all()
    l4 = (fl & F_L4) != 0
    assert l4.sum() > 10 and ((fl[l4] & F_L4_OK) != 0).all()


def test_tx_two_streams_one_context(dev):
    """Two fixed-stride tx batches of one context queued on two streams at
    once (the two-pass side array must not be shared): each
    call's side array comes from the context's stream-ordered pool, so both
    batches get exactly the reference's checksums; repeated so the pool's
    reuse is exercised too."""
    from oracle.oracle import Oracle
    from harness.synth import make_batch
    n = 40_000
    ba = make_batch("c1500", n, dev, first=0)
    bb = make_batch("c1500", n, dev, first=n)
    ha = ba["frames"][: n * 1500].cpu().numpy().copy()
    hb = bb["frames"][: n * 1500].cpu().numpy().copy()
    wa = Oracle().tx_batch(ha, stride=1500, fixed_len=1500, n=n)
    wb = Oracle().tx_batch(hb, stride=1500, fixed_len=1500, n=n)
    ctx = _ctx()
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for _ in range(3):
        fa, fb = torch.from_numpy(ha).to(dev), torch.from_numpy(hb).to(dev)
        torch.cuda.synchronize()
        for _ in range(2):          # idempotent: a second pass sets the same fields
            ctx.tx_cksum_device(fa, n, stride=1500, fixed_len=1500, stream=sa)
            ctx.tx_cksum_device(fb, n, stride=1500, fixed_len=1500, stream=sb)
        torch.cuda.synchronize()
        assert np.array_equal(fa.cpu().numpy(), wa)
        assert np.array_equal(fb.cpu().numpy(), wb)


def test_tx_m6_fixed_stride_forced(dev):
    """Tx with the mixed-shape kernel forced on a fixed-stride batch (its
    masked-sum instantiation): the launch is M6 and the frames are exact."""
    from pptk_amd.rx import VARIANTS
    z, buf_in, buf_out = _case("c64")
    ctx = _ctx()
    m6 = VARIANTS.index("M6")
    ctx.set_tuning(m6, 0)
    for shift in (0, 5):
        big, frames = _tx(ctx, z, buf_in, dev, shift, stride=64)
        assert ctx.last_variant() == m6
        assert np.array_equal(frames[:buf_in.size].cpu().numpy(), buf_out), shift
