"""BENCH TOOLING: per-tile SQ counters (instructions per 64-frame tile) of
the last rx dispatch in each rocprofv3 --pmc output directory given.

    python tools/sq_summary.py gpurun_out/sq_cmix_32 gpurun_out/sq_cmix_48 ..."""
import collections
import csv
import glob
import json
import os
import sys


def summarize(d, frames=16 * 1024 * 1024):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    by = collections.defaultdict(dict)
    name = {}
    for r in csv.DictReader(open(f)):
        by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        name[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    last = max(by)
    tiles = frames / 64
    return {"dir": d, "kernel": name[last][:80],
            "per_tile": {k: round(v / tiles, 1) for k, v in sorted(by[last].items())}}


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(json.dumps(summarize(d)))
