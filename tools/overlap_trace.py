"""PROBE TOOLING: from a rocprofv3 kernel trace (kernel_trace.csv), how much
of each RCCL stand-in kernel (tools/standin.hip) ran while an rx kernel was
running, and how long the rx kernels beside it took.  One JSON line.

    python tools/overlap_trace.py TRACE_DIR
"""
import csv
import glob
import json
import os
import sys


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    name = next(k for k in rows[0] if k.lower() in ("kernel_name", "kernel-name"))
    rx = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                if "rx_kernel" in r[name])
    st = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                if "standin" in r[name])
    st = st[len(st) // 2:]   # the later half: past the settle and the alone runs
    fr, waits = [], []
    for s0, s1 in st:
        ov = sum(max(0, min(s1, r1) - max(s0, r0)) for r0, r1 in rx)
        fr.append(ov / max(1, s1 - s0))
        prev_end = max((r1 for r0, r1 in rx if r1 <= s0 + 1000), default=None)
        if prev_end is not None:
            waits.append((s0 - prev_end) / 1e3)
    rx_ms = sorted((r1 - r0) / 1e6 for r0, r1 in rx)
    print(json.dumps({
        "trace": os.path.relpath(f), "rx_kernels": len(rx), "standin_kernels": len(st),
        "standin_ms_median": sorted((s1 - s0) / 1e6 for s0, s1 in st)[len(st) // 2],
        "standin_overlap_with_rx_median": sorted(fr)[len(fr) // 2],
        "standin_start_after_batch_us_median": sorted(waits)[len(waits) // 2] if waits else None,
        "rx_ms_median": rx_ms[len(rx_ms) // 2]}))


if __name__ == "__main__":
    main()
