"""BENCH TOOLING: run bench.py's rate-limiter workload once (for rocprofv3
wrapping): python tools/permit_run.py [runs] [--ab] [--lib=NAME=PATH ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stamps():
    """The fused rate limiter's phase timestamps (every workgroup, 100 MHz
    clock, PermitFused::stamps: 12 x 256 words after the 2 KB of barrier
    words and 256 B of flags at the start of the scratch) on 16 M dense keys,
    2^16 buckets, as bench's keys / keys_denying runs: microseconds from the
    earliest workgroup start, min / median / max over the 256 workgroups;
    rows 9-11 are phase-3 durations of wave 0 (ordered walk: list building /
    walk; hash tables: partition / ranking / passes)."""
    import numpy as np
    import torch
    from pptk_amd.rx import RxContext
    dev = torch.device("cuda", 0)
    n, hs, nblk = 16 * 1024 * 1024, 1 << 16, 256
    ctx = RxContext(0, bytes(range(1, 17)), 24, 0, hs)
    keys = torch.randint(0, hs, (n,), dtype=torch.int32, device=dev)
    scratch = torch.zeros(ctx._L.pptk_rx_permit_scratch_bytes(n, hs), dtype=torch.uint8, device=dev)
    labels = ["start", "histogram", "row written", "barrier 1", "phase 2", "barrier 2", "verdicts",
              "codes staged", "boundaries found"]
    off, nrow = 2048 + 256, 12
    out = {}
    for name, t in (("keys", 1 << 20), ("keys_denying", 128)):
        runs = []
        for _ in range(8):
            tok = torch.full((hs,), t, dtype=torch.int32, device=dev)
            ctx.permit_keys_device(keys, 4, tok, scratch=scratch)
            torch.cuda.synchronize()
            w = scratch[off:off + nrow * nblk * 4].view(torch.int32).cpu().numpy()
            runs.append(w.view(np.uint32).astype(np.int64).reshape(nrow, nblk))
        st = runs[len(runs) // 2]
        t0 = st[0].min()
        r = (st - t0) / 100.0
        out[name] = {lab: [round(float(r[k].min()), 2), round(float(np.median(r[k])), 2),
                           round(float(r[k].max()), 2)] for k, lab in enumerate(labels)}
        out[name]["slowest_phase1_blocks"] = [int(x) for x in np.argsort(r[2] - r[0])[-8:]]
        out[name]["slowest_phase2_blocks"] = [int(x) for x in np.argsort(r[4] - r[3])[-8:]]
        hb = int(np.argmax(r[8] - r[7])) if name == "keys_denying" else 0
        out[name + "_phase3_heaviest"] = {"block": hb, "part_or_list_us": st[9, hb] / 100.0,
                                          "rank_or_walk_us": st[10, hb] / 100.0,
                                          "hash_passes": int(st[11, hb])}
    out["unit"] = "us from the earliest workgroup start: [min, median, max] over workgroups"
    print(json.dumps(out), flush=True)


def main():
    import torch
    import bench
    if "--stamps" in sys.argv:
        return stamps()
    dev = torch.device("cuda", 0)
    runs = tuple(sys.argv[1].split(",")) if len(sys.argv) > 1 else ("records", "keys",
                                                                     "keys_denying")
    ab = "--ab" in sys.argv
    print(json.dumps({"fused": bench.permit_bench(16 * 1024 * 1024, dev, 1, 0, 20, 3, runs=runs)}),
          flush=True)
    if ab:   # the four-launch path on the same workload
        print(json.dumps({"passes": bench.permit_bench(16 * 1024 * 1024, dev, 1, 0, 20, 3, runs=runs,
                                                       tune=0x400)}), flush=True)
    for a in sys.argv[1:]:   # --lib NAME=PATH: the fused path of another build
        if a.startswith("--lib="):
            name, path = a[6:].split("=", 1)
            print(json.dumps({name: bench.permit_bench(16 * 1024 * 1024, dev, 1, 0, 20, 3, runs=runs,
                                                       lib_path=os.path.join(ROOT, path))}),
                  flush=True)


if __name__ == "__main__":
    main()
