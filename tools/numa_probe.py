"""PROBE: where the GPU sits (NUMA node), which CPUs this job may use per
node, and bench's e2e (host to host) with the process pinned to the GPU's
node against unpinned.  Prints JSON."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.init()
    info = bench.gpu_numa(dev)
    out = {"numa": info, "affinity_n": len(os.sched_getaffinity(0))}
    print(json.dumps(out), flush=True)
    for mode in ("pinned", "unpinned", "pinned"):
        t0 = time.time()
        r = bench.e2e_bench(dev, numa_local=(mode == "pinned"),
                            cfgs=(("c64", "c64", 1 << 22, True, False),
                                  ("c64_rec32", "c64", 1 << 22, True, True)))
        out[mode] = r
        print(json.dumps({mode: r, "s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
