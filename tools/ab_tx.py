"""BENCH TOOLING: in-process A/B of tx-side (pptk_tx_cksum_device) settings
on one batch.  python tools/ab_tx.py c1500 3:32 3:33 3:544 ...
(variant:flags; flag 512 = diagnostics, no checksum writes)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pptk_amd.rx import RxContext
    from tools.synth import make_batch
    cfg = sys.argv[1]
    settings = [tuple(int(x) for x in a.split(":")) for a in sys.argv[2:]]
    n = int(os.environ.get("AB_FRAMES", 16 * 1024 * 1024))
    dev = torch.device("cuda", 0)
    b = make_batch(cfg, n, dev)
    kw = (dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]) if "off" in b
          else dict(stride=b["stride"], fixed_len=b["fixed_len"]))
    ctx = RxContext(0, bytes(range(1, 17)))
    times = {s: [] for s in settings}
    for _ in range(5):
        for s in settings:
            ctx.set_tuning(*s)
            ctx.tx_cksum_device(b["frames"], n, **kw)
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ctx.tx_cksum_device(b["frames"], n, **kw)
                e1.record()
                torch.cuda.synchronize()
                times[s].append(e0.elapsed_time(e1))
    out = {"cfg": cfg, "frames": n}
    for s, t in times.items():
        ms = float(np.median(t))
        out[f"{s[0]}:{s[1]}"] = {"ms": round(ms, 4), "gbs": round(b["bytes"] / ms / 1e6, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
