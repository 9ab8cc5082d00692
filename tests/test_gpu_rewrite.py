"""Header rewrite with incremental checksum updates on the GPU
(pptk_tx_rewrite_device) against the reference's ip_decr_ttl_cksum_update /
ip_set_src/dst_cksum_update / tcp/udp_set_src/dst_port_cksum_update
(tests/golden/rewrite.npz), byte for byte with the per-frame status, in
both layouts and misaligned; and, on a large batch, the size-independent
property that a rewrite keeps every checksum verdict of the receive
transform while the records show the new addresses and ports.  Needs an
MI355X."""
import numpy as np
import pytest

from test_oracle import REWRITE_CASES, rewrite_case

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _ctx():
    from pptk_amd.rx import RxContext
    return RxContext(0, bytes(range(1, 17)))


def _rewrite(ctx, z, buf, rw, dev, shift, stride=None):
    big = torch.zeros(buf.size + shift + 64, dtype=torch.uint8, device=dev)
    big[shift:shift + buf.size] = torch.from_numpy(buf).to(dev)
    frames = big[shift:]
    n = len(z["off"])
    rw_t = torch.from_numpy(rw.view(np.uint8).copy()).to(dev)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    if stride is None:
        ctx.tx_rewrite_device(frames, n, rw_t, off=torch.from_numpy(z["off"].view(np.int64)).to(dev),
                              lens=torch.from_numpy(z["len"].view(np.int16)).to(dev), status=st)
    else:
        ctx.tx_rewrite_device(frames, n, rw_t, stride=stride, fixed_len=int(z["len"][0]), status=st)
    torch.cuda.synchronize()
    return big, frames, st.cpu().numpy()


@pytest.mark.parametrize("tag,name", REWRITE_CASES)
@pytest.mark.parametrize("shift", [0, 5, 64])
def test_rewrite_matches_reference(tag, name, shift, dev):
    z, buf_in, buf_out, rw, status = rewrite_case(tag, name)
    big, frames, st = _rewrite(_ctx(), z, buf_in, rw, dev, shift)
    got = frames[:buf_in.size].cpu().numpy()
    assert np.array_equal(st, status)
    assert np.array_equal(got, buf_out), int((got != buf_out).sum())
    # nothing outside the frames' buffer was touched
    assert int(big[:shift].sum()) == 0 and int(big[shift + buf_in.size:].sum()) == 0


@pytest.mark.parametrize("tag", ["c64", "c64_one"])
def test_rewrite_fixed_stride(tag, dev):
    z, buf_in, buf_out, rw, status = rewrite_case(tag, "c64")
    _, frames, st = _rewrite(_ctx(), z, buf_in, rw, dev, 3, stride=64)
    assert np.array_equal(st, status)
    assert np.array_equal(frames[:buf_in.size].cpu().numpy(), buf_out)


def test_rewrite_keeps_verdicts_large(dev):
    """1 M C64 + 128 K C1500 frames: after a NAT rewrite (new source and
    destination, new ports, TTL decrement) of every frame, the receive
    transform still verifies exactly the frames it verified before (but for
    UDP checksums of 0), and its records carry the new addresses and ports."""
    from pptk_amd.records import F_IP_OK, F_L4_OK, F_UDP_ZERO, REWRITE_DTYPE, as_records
    from harness.synth import make_batch
    ctx = _ctx()
    for cfg, n in (("c64", 1 << 20), ("c1500", 1 << 17)):
        b = make_batch(cfg, n, dev)
        before = as_records(ctx.batch_device(b["frames"], n, stride=b["stride"],
                                             fixed_len=b["fixed_len"]).cpu().numpy().reshape(-1))
        rw = np.zeros(1, REWRITE_DTYPE)
        rw["ops"], rw["src"], rw["dst"] = 0x1F, 0xC0A80A01, 0x0A000002
        rw["sport"], rw["dport"] = 4242, 443
        st = torch.zeros(n, dtype=torch.uint8, device=dev)
        ctx.tx_rewrite_device(b["frames"], n, torch.from_numpy(rw.view(np.uint8).copy()).to(dev),
                              stride=b["stride"], fixed_len=b["fixed_len"], status=st)
        after = as_records(ctx.batch_device(b["frames"], n, stride=b["stride"],
                                            fixed_len=b["fixed_len"]).cpu().numpy().reshape(-1))
        torch.cuda.synchronize()
        assert (st.cpu().numpy() == 3).all()          # IP + L4 applied, TTL 64 -> 63
        # a transmitted UDP checksum of 0 means "none" and stays 0, also when
        # one of the updates produced it (as in the reference, which re-reads
        # the field before each update), so those frames (a few in 10^5) may
        # change verdict
        keep = ((before["flags"] | after["flags"]) & F_UDP_ZERO) == 0
        assert keep.mean() > 0.999
        for flag in (F_IP_OK, F_L4_OK):
            assert np.array_equal(before["flags"][keep] & flag, after["flags"][keep] & flag), \
                (cfg, flag)
        assert (after["src"][:, :4] == np.array([192, 168, 10, 1], np.uint8)).all()
        assert (after["dst"][:, :4] == np.array([10, 0, 0, 2], np.uint8)).all()
        assert (after["sport"] == 4242).all() and (after["dport"] == 443).all()
        assert np.array_equal(before["l4_len"], after["l4_len"])


def test_rewrite_rejects_bad_args(dev):
    from pptk_amd.records import REWRITE_DTYPE
    ctx = _ctx()
    frames = torch.zeros(640, dtype=torch.uint8, device=dev)
    rw = torch.zeros((3, 16), dtype=torch.uint8, device=dev)   # neither 1 nor n entries
    with pytest.raises(OSError):
        ctx.tx_rewrite_device(frames, 10, rw, stride=64, fixed_len=64)
    ctx.tx_rewrite_device(frames, 0, rw, stride=64, fixed_len=64)   # n = 0: no-op
    assert REWRITE_DTYPE.itemsize == 16
