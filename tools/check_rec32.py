"""BENCH TOOLING: compare compact records with the projection of the full
records on a large synthetic batch (both from the GPU), report mismatches by
position.  python tools/check_rec32.py c1500 [n]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pptk_amd.records import REC32_DTYPE, to_rec32
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    cfg = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16 * 1024 * 1024
    dev = torch.device("cuda", 0)
    b = make_batch(cfg, n, dev)
    kw = (dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]) if "off" in b
          else dict(stride=b["stride"], fixed_len=b["fixed_len"]))
    ctx = RxContext(0, bytes(range(1, 17)))
    full = ctx.batch_device(b["frames"], n, **kw)
    c32 = ctx.batch_device(b["frames"], n, compact=True, **kw)
    torch.cuda.synchronize()
    chunk = 1 << 20
    bad = []
    for s in range(0, n, chunk):
        w = to_rec32(full[s:s + chunk].cpu().numpy())
        g = c32[s:s + chunk].cpu().numpy().reshape(-1).view(REC32_DTYPE)
        d = np.nonzero((g.view(np.uint8).reshape(-1, 32) != w.view(np.uint8).reshape(-1, 32)).any(1))[0]
        bad += list(d + s)
    print("mismatches", len(bad), "first", bad[:20])
    if bad:
        i = bad[0]
        print("got ", c32[i].cpu().numpy())
        print("want", to_rec32(full[i:i + 1].cpu().numpy()).view(np.uint8))
        t = np.array(bad) // 64
        print("tiles", np.unique(t)[:20], "lanes", np.unique(np.array(bad) % 64)[:64])


if __name__ == "__main__":
    main()
