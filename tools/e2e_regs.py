"""BENCH TOOLING: host-to-host C64 with the record array registered (the
kernel stores records over PCIe) or not (records land in device memory and
a DMA copies them back, overlapping the next chunk's frames going down), for
64- and 32-byte records, staged and ring paths -- bench.e2e_bench's
measurement with other settings.  One JSON line.

    python tools/e2e_regs.py [seconds]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
    dev = torch.device("cuda", 0)
    cfgs = (("c64_reg", "c64", 1 << 22, True, False),
            ("c64_noreg", "c64", 1 << 22, False, False),
            ("c64_rec32_reg", "c64", 1 << 22, True, True),
            ("c64_rec32_noreg", "c64", 1 << 22, False, True))
    print(json.dumps(bench.e2e_bench(dev, secs, cfgs)), flush=True)


if __name__ == "__main__":
    main()
