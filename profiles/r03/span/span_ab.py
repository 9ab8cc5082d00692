"""BENCH TOOLING: the span kernel (RX_SPAN) against the automatic team
variant on the same batch and record buffer, interleaved launches, medians.

    python tools/span_ab.py [--cfgs cmix,imix,c1500,c64] [--reps 10]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pptk_amd.rx import VARIANTS, RxContext
    from harness.synth import make_batch
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="cmix,imix,c1500")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--n", type=int, default=16 * 1024 * 1024)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = RxContext(0, bytes(range(1, 17)))
    out = {}
    for cfg in args.cfgs.split(","):
        b = make_batch(cfg, args.n, dev)
        kw = (dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]) if "off" in b
              else dict(stride=b["stride"], fixed_len=b["fixed_len"]))
        recs = torch.empty((args.n, 64), dtype=torch.uint8, device=dev)
        ref = None
        t = {}
        for rep in range(args.reps + 2):
            for v in ("auto", "SPAN"):
                ctx.set_tuning(-1 if v == "auto" else VARIANTS.index(v), -1)
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                ctx.batch_device(b["frames"], args.n, recs=recs, **kw)
                z.record()
                torch.cuda.synchronize()
                if rep >= 2:
                    t.setdefault(v, []).append(a.elapsed_time(z))
                if rep == 0:
                    h = recs.view(torch.int64)[:, :8].sum(dim=0).cpu()   # whole-batch checksum
                    if ref is None:
                        ref = h
                    t.setdefault("identical", []).append(bool(torch.equal(ref, h)))
                if rep == 2 and v == "auto":
                    t["auto_variant"] = VARIANTS[ctx.last_variant()]
        res = {k: (round(sorted(x)[len(x) // 2], 4) if k in ("auto", "SPAN") else x)
               for k, x in t.items()}
        res["bytes"] = b["bytes"]
        res["span_read_frac"] = round(b["bytes"] / (res["SPAN"] * 1e-3) / 8e12, 4)
        out[cfg] = res
        print(json.dumps({cfg: res}), flush=True)
        del b, recs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
