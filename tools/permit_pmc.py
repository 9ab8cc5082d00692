"""BENCH TOOLING: per-launch HBM traffic of the rate limiter's kernels from
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of tools/permit_run.py.

    python tools/permit_pmc.py DIR [run ...]   (DIR/pmc_<run>_<COUNTER>/)

FETCH_SIZE x 2 for the 16-byte-per-lane reads (MI355X_MICROARCH.md, HBM
section, as tools/pmc_summary.py); both counters in KiB.  Prints JSON: per
run, per kernel, the median per launch in MB, and the total per call."""
import csv
import glob
import json
import os
import re
import statistics
import sys


def per_kernel(d, cname):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        acc = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != cname or "permit" not in r["Kernel_Name"]:
                continue
            k = re.search(r"permit_\w+", r["Kernel_Name"]).group(0)
            acc.setdefault((k, r["Dispatch_Id"]), 0.0)
            acc[(k, r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, _), v in acc.items():
            out.setdefault(k, []).append(v)
    return {k: statistics.median(v) * 1024 / 1e6 for k, v in out.items()}


def main():
    d = sys.argv[1]
    runs = sys.argv[2:] or ["keys", "keys_denying"]
    res = {}
    for run in runs:
        fe = per_kernel(os.path.join(d, f"pmc_{run}_FETCH_SIZE"), "FETCH_SIZE")
        wr = per_kernel(os.path.join(d, f"pmc_{run}_WRITE_SIZE"), "WRITE_SIZE")
        ks = sorted(set(fe) | set(wr))
        res[run] = {k: {"read_mb": round(2 * fe.get(k, 0.0), 2), "written_mb": round(wr.get(k, 0.0), 2)}
                    for k in ks}
        res[run]["total_mb"] = round(sum(2 * fe.get(k, 0.0) + wr.get(k, 0.0) for k in ks), 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
