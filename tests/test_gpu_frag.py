"""The fragment side record (struct pptk_rx_frag, pptk_rx_dev_batch.d_frag)
on the GPU, bit for bit against the reference-made fixtures
(tests/golden/frag.npz: ip_id / ip_frag_off / ip_more_frags / ip_dont_frag
and ipv6_const_proto_hdr_2's frag_hdr_off / proto_hdr_off_from_frag, via
oracle/refgen.c), in every kernel variant and addressing mode; the 64-byte
records written beside them must stay the golden records."""
import numpy as np
import pytest

from conftest import load_golden
from pptk_amd.records import FRAG_DTYPE, REC32_DTYPE, diff_records, to_rec32

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
FRAG_SETS = ("frag", "edge", "fuzz", "cmix")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _want_frag(name):
    zf = load_golden("frag")
    return np.ascontiguousarray(zf["frag" if name == "frag" else f"{name}_frag"]).reshape(-1) \
        .view(FRAG_DTYPE)


def _ctx(z):
    from pptk_amd.rx import RxContext
    b4, b6, hs = (int(x) for x in z["iphash"])
    return RxContext(0, z["key"].tobytes(), b4, b6, hs, max_frame=65535)


def _run(ctx, z, dev, compact=False, mixed=False, shift=0):
    n = len(z["off"])
    big = torch.zeros(z["buf"].size + shift + 64, dtype=torch.uint8, device=dev)
    big[shift:shift + z["buf"].size] = torch.from_numpy(z["buf"]).to(dev)
    frames = big[shift:]
    off = torch.from_numpy(z["off"].view(np.int64)).to(dev)
    lens = torch.from_numpy(z["len"].view(np.int16)).to(dev)
    frag = torch.full((n, 16), 0xA5, dtype=torch.uint8, device=dev)
    if mixed:
        recs = ctx.batch_device_mixed(frames, n, off, lens, max_len=int(z["len"].max()),
                                      frag_out=frag)
    else:
        recs = ctx.batch_device(frames, n, off=off, lens=lens, max_len=int(z["len"].max()),
                                compact=compact, frag_out=frag)
    torch.cuda.synchronize()
    return recs.cpu().numpy().reshape(-1), frag.cpu().numpy().reshape(-1).view(FRAG_DTYPE)


@pytest.mark.parametrize("name", FRAG_SETS)
def test_frag_side_records_equal_golden(dev, name):
    z = load_golden(name)
    recs, frag = _run(_ctx(z), z, dev)
    d = diff_records(frag, _want_frag(name), dtype=FRAG_DTYPE)
    assert not d, d
    d = diff_records(recs, z["recs"])
    assert not d, d


@pytest.mark.parametrize("name", ["frag", "fuzz"])
def test_frag_every_variant(dev, name):
    """Every team kernel shape (forced) and two alignments write the same
    side records; the lane kernel is never chosen when d_frag is set."""
    from pptk_amd.rx import RX_L4, VARIANTS
    z = load_golden(name)
    want = _want_frag(name)
    ctx = _ctx(z)
    for v in range(len(VARIANTS)):
        ctx.set_tuning(v, -1)
        for shift in (0, 5):
            recs, frag = _run(ctx, z, dev, shift=shift)
            assert ctx.last_variant() != RX_L4
            d = diff_records(frag, want, dtype=FRAG_DTYPE)
            assert not d, f"{VARIANTS[v]} shift {shift}: {d}"
            d = diff_records(recs, z["recs"])
            assert not d, f"{VARIANTS[v]} shift {shift}: {d}"


@pytest.mark.parametrize("name", FRAG_SETS)
def test_frag_binned_mixed_path(dev, name):
    """pptk_rx_batch_device_mixed (binned order, one launch per length
    group): side records still land at the frame's own index."""
    z = load_golden(name)
    recs, frag = _run(_ctx(z), z, dev, mixed=True)
    d = diff_records(frag, _want_frag(name), dtype=FRAG_DTYPE)
    assert not d, d
    d = diff_records(recs, z["recs"])
    assert not d, d


def test_frag_with_compact_records(dev):
    z = load_golden("frag")
    recs, frag = _run(_ctx(z), z, dev, compact=True)
    d = diff_records(frag, _want_frag("frag"), dtype=FRAG_DTYPE)
    assert not d, d
    d = diff_records(recs.view(np.uint8), to_rec32(z["recs"]), dtype=REC32_DTYPE)
    assert not d, d


@pytest.mark.parametrize("name,stride", [("c64", 64), ("c1500", 1500)])
def test_frag_fixed_stride(dev, oracle_lib_frag, name, stride):
    """Fixed-stride batches (C64 would take the lane kernel without d_frag):
    IPv4 side records of every frame, against the CPU oracle."""
    z = load_golden(name)
    n = len(z["off"])
    ctx = _ctx(z)
    frames = torch.from_numpy(z["buf"]).to(dev)
    frag = torch.zeros((n, 16), dtype=torch.uint8, device=dev)
    recs = ctx.batch_device(frames, n, stride=stride, fixed_len=stride, frag_out=frag)
    torch.cuda.synchronize()
    want = oracle_lib_frag.frag_batch(z["buf"], z["off"], z["len"])
    d = diff_records(frag.cpu().numpy().reshape(-1).view(FRAG_DTYPE), want, dtype=FRAG_DTYPE)
    assert not d, d
    d = diff_records(recs.cpu().numpy().reshape(-1), z["recs"])
    assert not d, d


@pytest.fixture(scope="module")
def oracle_lib_frag():
    from oracle.oracle import Oracle
    return Oracle()
