"""pptk_tx_cksum_device against the reference's setters (tests/golden/tx.npz)
for the golden sets, offsets and fixed-stride layouts -- run as a child
process by tests/test_gpu_tx.py::test_tx_in_place_mode with PPTK_TX_TWO_PASS=0
(the env switch is read once per process).  Needs an MI355X.

    python tests/txcase.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def run():
    import torch
    from conftest import load_golden
    from pptk_amd.rx import RxContext
    dev = torch.device("cuda", 0)
    t = load_golden("tx")
    ctx = RxContext(0, bytes(range(1, 17)))
    for name in ("edge", "fuzz", "cmix", "c64"):
        z = load_golden(name)
        pos = t[f"{name}_pos"].astype(np.int64)
        buf_in = z["buf"].copy()
        buf_in[pos] = t[f"{name}_in"]
        want = buf_in.copy()
        want[pos] = t[f"{name}_out"]
        n = len(z["off"])
        for shift in (0, 3):
            big = torch.zeros(buf_in.size + shift + 64, dtype=torch.uint8, device=dev)
            big[shift:shift + buf_in.size] = torch.from_numpy(buf_in).to(dev)
            frames = big[shift:]
            ctx.tx_cksum_device(frames, n, off=torch.from_numpy(z["off"].view(np.int64)).to(dev),
                                lens=torch.from_numpy(z["len"].view(np.int16)).to(dev),
                                max_len=int(z["len"].max()))
            torch.cuda.synchronize()
            got = frames[:buf_in.size].cpu().numpy()
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, f"{name} shift {shift}: {bad.size} bytes differ, first {bad[:8]}"
            if name == "c64":   # fixed stride: the in-place stores of the streaming pass
                fr = torch.from_numpy(buf_in).to(dev)
                ctx.tx_cksum_device(fr, n, stride=64, fixed_len=64)
                torch.cuda.synchronize()
                assert np.array_equal(fr.cpu().numpy(), want), "c64 fixed stride"


if __name__ == "__main__":
    run()
    print("ok")
