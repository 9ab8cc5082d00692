"""BENCH TOOLING: the ceilings under the end-to-end host path (DESIGN.md
section 7, "End-to-end"): pinned host-to-device and device-to-host copy
rates over PCIe, on one stream and on two, and the host memcpy rate of the
gather (pageable frames into pinned staging) on 1 and 8 threads.

    python tools/pcie_probe.py [MB per copy]

One JSON line, GB/s."""
import json
import sys
import threading
import time

import numpy as np


def rate(fn, nbytes, reps=20):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return round(nbytes * reps / (time.perf_counter() - t0) / 1e9, 2)


def main():
    import torch
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    nb = mb << 20
    dev = torch.device("cuda", 0)
    h = [torch.empty(nb, dtype=torch.uint8).pin_memory() for _ in range(2)]
    d = [torch.empty(nb, dtype=torch.uint8, device=dev) for _ in range(2)]
    s = [torch.cuda.Stream(dev) for _ in range(2)]
    out = {"copy_mb": mb}

    def h2d1():
        d[0].copy_(h[0], non_blocking=True)
        torch.cuda.synchronize(dev)

    def h2d2():
        for k in range(2):
            with torch.cuda.stream(s[k]):
                d[k].copy_(h[k], non_blocking=True)
        torch.cuda.synchronize(dev)

    def d2h1():
        h[0].copy_(d[0], non_blocking=True)
        torch.cuda.synchronize(dev)

    def bidir():
        with torch.cuda.stream(s[0]):
            d[0].copy_(h[0], non_blocking=True)
        with torch.cuda.stream(s[1]):
            h[1].copy_(d[1], non_blocking=True)
        torch.cuda.synchronize(dev)

    out["h2d_1stream_gbs"] = rate(h2d1, nb)
    out["h2d_2streams_gbs"] = rate(h2d2, 2 * nb)
    out["d2h_1stream_gbs"] = rate(d2h1, nb)
    out["bidir_gbs_each_way"] = rate(bidir, nb)

    src = np.random.default_rng(0).integers(0, 255, nb, dtype=np.uint8)   # pageable
    dst = h[0].numpy()

    def gather(nth):
        def run():
            parts = np.array_split(np.arange(nb // 1500) * 1500, nth)
            def work(p):
                for o in p[::64]:     # 64-frame runs: ~96 KB memcpy per call
                    e = min(nb, o + 64 * 1500)
                    dst[o:e] = src[o:e]
            ts = [threading.Thread(target=work, args=(p,)) for p in parts]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        return run

    out["host_copy_1thread_gbs"] = rate(gather(1), nb, reps=5)
    out["host_copy_8threads_gbs"] = rate(gather(8), nb, reps=5)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
