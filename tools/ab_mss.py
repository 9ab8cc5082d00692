"""BENCH TOOLING: in-process A/B of library builds on the MSS-clamping bench
workload (bench.py mss_bench), interleaved rounds.

    AB_LIBS=bytes=build/ab_mssbytes/libpptkrx.so python tools/ab_mss.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pptk_amd.rx import RxContext
    dev = torch.device("cuda", 0)
    libs = {"": None}
    for kv in filter(None, os.environ.get("AB_LIBS", "").split(",")):
        k, v = kv.split("=", 1)
        libs[k] = os.path.join(ROOT, v)
    n = int(os.environ.get("AB_FRAMES", 16 * 1024 * 1024))
    res = {k: [] for k in libs}
    for _ in range(int(os.environ.get("AB_ROUNDS", 4))):
        for k, p in libs.items():
            ctx = RxContext(0, bench.KEY, lib_path=p)
            r = bench.mss_bench(ctx, n, dev, 10, 2)
            assert r["clamped_every_frame"] or k.startswith("d")   # d*: diagnostic builds
            res[k].append(r["kernel_ms"])
            ctx.close()
    print(json.dumps({k or "current": sorted(v)[len(v) // 2] for k, v in res.items()}))


if __name__ == "__main__":
    main()
