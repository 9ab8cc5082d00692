"""BENCH TOOLING: in-process A/B of kernel variants / flags / library builds
on one batch.

    python tools/ab.py c1500 3:1 3:0 6:1 ...        (variant:flags pairs)
    AB_LIBS=old=build/ab_old/libpptkrx.so python tools/ab.py cmix 3:33 old:3:33

A setting is [lib:]variant:flags[:c][:m][:h]; variant or flags -1 = automatic
choice; a trailing :h also writes the dense flow-hash array (the multi-GPU
all-gather's send slice, into one buffer allocated after the records);
a trailing :c writes compact 32-byte records, :m runs that setting
through pptk_rx_batch_device_mixed (mixed batches; as AB_MIXED=1 does for all);
lib names come from AB_LIBS (name=path,...), default = pptk_amd/libpptkrx.so.
Generates the batch once, then times every setting in interleaved rounds
(A B C A B C ...) so that clock and thermal drift hit all settings alike;
prints one JSON line with the median kernel ms and GB/s per setting.
AB_PLACE=1 times on placed frame and record buffers (bench.placed_buffers);
AB_SOL=1 adds the speed of light of the launch's traffic (bench.mix_sol).
AB_BIN=1 processes mixed batches in length-binned order (pptk_rx_bin_device,
timed inside each launch's window); AB_MIXED=1 through
pptk_rx_batch_device_mixed (binning + one launch per length group)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_setting(a):
    """[lib:]variant:flags[:c][:m][:h] -> (lib, variant, flags, compact, mixed, hash)."""
    p = a.split(":")
    hsh = p[-1] == "h"
    if hsh:
        p = p[:-1]
    mixed = p[-1] == "m"
    if mixed:
        p = p[:-1]
    compact = p[-1] == "c"
    if compact:
        p = p[:-1]
    if len(p) == 2:
        return ("", int(p[0]), int(p[1]), compact, mixed, hsh)
    return (p[0], int(p[1]), int(p[2]), compact, mixed, hsh)


def main():
    import torch
    from pptk_amd.rx import RxContext
    from harness.membench import measure
    from harness.synth import make_batch
    cfg = sys.argv[1]
    settings = [parse_setting(a) for a in sys.argv[2:]]
    libs = {"": None}
    for kv in filter(None, os.environ.get("AB_LIBS", "").split(",")):
        k, v = kv.split("=", 1)
        libs[k] = os.path.join(ROOT, v) if not os.path.isabs(v) else v
    n = int(os.environ.get("AB_FRAMES", 16 * 1024 * 1024))
    rounds = int(os.environ.get("AB_ROUNDS", 5))
    reps = int(os.environ.get("AB_REPS", 5))
    binned = bool(os.environ.get("AB_BIN"))
    dev = torch.device("cuda", 0)
    b = make_batch(cfg, n, dev)
    kw = (dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]) if "off" in b
          else dict(stride=b["stride"], fixed_len=b["fixed_len"]))
    ctxs = {k: RxContext(0, bytes(range(1, 17)), lib_path=v) for k, v in libs.items()}
    placement = None
    if os.environ.get("AB_PLACE"):
        # well-placed frame and record buffers (bench.placed_buffers), as
        # bench.py uses
        import bench
        recs64, placement = bench.placed_buffers(ctxs[""], b, n, dev, False, kw)
        recs32, _ = bench.placed_buffers(ctxs[""], b, n, dev, True, kw, frames=False)
    else:
        recs64 = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        recs32 = torch.empty((n, 32), dtype=torch.uint8, device=dev)

    mixed = bool(os.environ.get("AB_MIXED")) and "off" in b
    if (mixed or any(st[4] for st in settings)) and "off" in b:
        perm = torch.empty(n, dtype=torch.int32, device=dev)
        scratch = torch.empty(ctxs[""]._L.pptk_rx_bin_scratch_bytes(n), dtype=torch.uint8,
                              device=dev)

    hbuf = (torch.empty(n, dtype=torch.int64, device=dev) if any(st[5] for st in settings)
            else None)

    def launch(ctx, compact, mix=False, hsh=False):
        recs = recs32 if compact else recs64
        if (mixed or mix) and "off" in b:
            ctx.batch_device_mixed(b["frames"], n, b["off"], b["lens"], recs=recs64,
                                   max_len=b["max_len"], perm=perm, scratch=scratch)
        elif binned and "off" in b:
            ctx.batch_device(b["frames"], n, recs=recs, perm=ctx.bin_device(b["lens"], n),
                             compact=compact, **kw)
        else:
            ctx.batch_device(b["frames"], n, recs=recs, compact=compact,
                             hash_out=hbuf if hsh else None, **kw)

    ref = {}
    times = {s: [] for s in settings}
    same = {}
    for _ in range(rounds):
        for s in settings:
            ctx = ctxs[s[0]]
            ctx.set_tuning(s[1], s[2])
            launch(ctx, s[3], s[4], s[5])
            torch.cuda.synchronize()
            if s not in same:       # every setting must give the same records
                r = recs32 if s[3] else recs64
                if s[3] not in ref:
                    ref[s[3]] = r.clone()
                same[s] = bool(torch.equal(r, ref[s[3]]))
                if s[5] and not s[3]:     # the dense hashes equal the records' flow_hash
                    same[s] = same[s] and bool(torch.equal(hbuf, r.view(torch.int64)[:, 0]))
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                launch(ctx, s[3], s[4], s[5])
                e1.record()
                torch.cuda.synchronize()
                times[s].append(e0.elapsed_time(e1))
    out = {"cfg": cfg, "frames": n, "binned": binned, "mixed": mixed,
           "box": measure(b["frames"]), "placement": placement}
    if os.environ.get("AB_SOL"):
        # the speed of light of this launch's traffic on these buffers
        # (tools/rwmix.py sol_ms, as bench.mix_sol)
        import bench
        sol = bench.mix_sol(b, recs64, n)
        if sol:
            out["sol_ms"], out["sol_desc"] = round(sol[0], 4), sol[1]
    for s, t in times.items():
        ms = float(np.median(t))
        key = ":".join(str(x) for x in s[:3] if x != "") + (":c" if s[3] else "") + \
            (":m" if s[4] else "") + (":h" if s[5] else "")
        out[key] = {"ms": round(ms, 4), "gbs": round(b["bytes"] / ms / 1e6, 1),
                    "mpkts": round(n / ms / 1e3, 1), "same_records": same[s]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
