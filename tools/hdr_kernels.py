"""BENCH TOOLING: run the header kernels' bench workloads once each (for
rocprofv3 wrapping): MSS clamping of 16 M SYNs and the C64 header rewrite.

    rocprofv3 --kernel-trace --stats -- python tools/hdr_kernels.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pptk_amd.rx import RxContext
    dev = torch.device("cuda", 0)
    ctx = RxContext(0, bench.KEY)
    n = int(os.environ.get("HDR_FRAMES", 16 * 1024 * 1024))
    steps = int(os.environ.get("HDR_STEPS", 5))
    print("mss", bench.mss_bench(ctx, n, dev, steps, 1), flush=True)
    print("rewrite", bench.rewrite_bench(ctx, n, dev, 0, steps, 1), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
