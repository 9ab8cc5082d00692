"""A registered-ring host batch checked against the CPU oracle (used by
tests/test_gpu_parity.py::test_registered_ring_span_dma, in-process and as
a child process with PPTK_RX_RING_DMA_PCT set).  Needs an MI355X.

    python tests/ringcase.py GAP"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def run(gap, n=70_000, L=1500):
    """70 000 C1500 frames `gap` bytes apart in a pageable ring at an odd
    address: staged, then registered (twice), every record against the
    oracle."""
    import torch
    from oracle.oracle import Oracle, make_opts
    from pptk_amd.rx import RxContext, ldp_packets
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    b = make_batch("c1500", n, dev)
    src = b["frames"][: n * L].cpu().numpy().reshape(n, L)
    step = L + gap
    ring = np.zeros(n * step + 4096 + 3, dtype=np.uint8)[3:]   # odd base address
    np.lib.stride_tricks.as_strided(ring, (n, L), (step, 1))[:] = src
    off = np.arange(n, dtype=np.uint64) * step
    lens = np.full(n, L, np.uint16)
    want = Oracle().rx_batch(ring, off, lens, opts=make_opts(bytes(range(1, 17))), nthreads=8)
    want = want.view(np.uint8).reshape(n, 64)
    ctx = RxContext(0, bytes(range(1, 17)), max_batch=65536, max_frame=1518, gather_threads=8)
    pkts = ldp_packets(ring, off, lens)
    assert np.array_equal(ctx.batch_host(pkts).view(np.uint8).reshape(n, 64), want), "staged"
    ctx.register_ring(ring)
    for k in range(2):
        got = ctx.batch_host(pkts).view(np.uint8).reshape(n, 64)
        assert np.array_equal(got, want), f"ring, pass {k}"
    ctx.unregister_ring(ring)
    ctx.close()


if __name__ == "__main__":
    run(int(sys.argv[1]))
    print("ok")
