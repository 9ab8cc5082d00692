"""BENCH TOOLING: run bench.py's rate-limiter workload once (for rocprofv3
wrapping): python tools/permit_run.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    print(bench.permit_bench(16 * 1024 * 1024, dev, 1, 0, 5, 1), flush=True)


if __name__ == "__main__":
    main()
