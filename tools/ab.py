"""BENCH TOOLING: in-process A/B of kernel variants / flags on one batch.

    python tools/ab.py c1500 3:1 3:0 6:1 7:1 ...   (variant:flags pairs)

Generates the batch once, then times every setting in interleaved rounds
(A B C A B C ...) so that clock and thermal drift hit all settings alike;
prints one JSON line with the median kernel ms and GB/s per setting."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pptk_amd.rx import RxContext
    from tools.membench import measure
    from tools.synth import make_batch
    cfg = sys.argv[1]
    settings = [tuple(int(x) for x in a.split(":")) for a in sys.argv[2:]]
    n = int(os.environ.get("AB_FRAMES", 16 * 1024 * 1024))
    rounds = int(os.environ.get("AB_ROUNDS", 5))
    reps = int(os.environ.get("AB_REPS", 5))
    dev = torch.device("cuda", 0)
    b = make_batch(cfg, n, dev)
    kw = (dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]) if "off" in b
          else dict(stride=b["stride"], fixed_len=b["fixed_len"]))
    recs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    ctx = RxContext(0, bytes(range(1, 17)))
    times = {s: [] for s in settings}
    for _ in range(rounds):
        for s in settings:
            ctx.set_tuning(*s)
            ctx.batch_device(b["frames"], n, recs=recs, **kw)
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ctx.batch_device(b["frames"], n, recs=recs, **kw)
                e1.record()
                torch.cuda.synchronize()
                times[s].append(e0.elapsed_time(e1))
    out = {"cfg": cfg, "frames": n, "box": measure(b["frames"])}
    for s, t in times.items():
        ms = float(np.median(t))
        out[f"{s[0]}:{s[1]}"] = {"ms": round(ms, 4), "gbs": round(b["bytes"] / ms / 1e6, 1),
                                 "mpkts": round(n / ms / 1e3, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
