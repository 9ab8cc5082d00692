"""BENCH TOOLING: summarize rocprofv3 runs into profiles/<round>/pmc_summary.json.

    python tools/pmc_summary.py OUT.json cfg=DIR_FETCH,DIR_WRITE[,DIR_STATS] ...
                                         op:NAME:REGEX:CHANGED=DIR_FETCH,DIR_WRITE ...

Per config: average rx_kernel duration from the kernel trace, FETCH_SIZE and
WRITE_SIZE per launch, and HBM traffic per launch corrected as
MI355X_MICROARCH.md (HBM section) prescribes for gfx950: FETCH_SIZE counts
half of the bytes of wide (16 B/lane) coalesced streaming reads -> x2;
WRITE_SIZE is exact for 16 B/lane streaming stores; both are in KiB."""
import csv
import glob
import json
import os
import sys


def rows(d, name):
    out = []
    for f in glob.glob(os.path.join(d, "**", name), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def counter(d, cname):
    """Per-launch values of the dominant rx kernel variant (the one the run's
    autotune chose: its settle + timed launches outnumber the 9 trial
    launches of every other shape)."""
    by = {}
    for r in rows(d, "*counter_collection.csv"):
        if "rx_kernel" in r["Kernel_Name"] and r["Counter_Name"] == cname:
            v, t = by.setdefault(r["Kernel_Name"], ([], []))
            v.append(float(r["Counter_Value"]))
            t.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    name = max(by, key=lambda k: len(by[k][0]))
    return by[name][0], by[name][1], name


def timed_launches(d, name, steps, gap_ms=20.0):
    """From the kernel trace of the traced bench command: the launches of
    kernel `name` split into runs (consecutive launches less than gap_ms
    apart); the first run at least half as long as the longest one is the
    config's settle + warmup + timed steps (the placement probe's and the
    autotune's runs are far shorter than the 1.5 s settle), and its last
    `steps` launches are the ones bench.py timed.
    Their mean / median duration is the same-run counterpart of the bench
    line's kernel_ms."""
    tr = [r for r in rows(d, "*kernel_trace.csv") if r["Kernel_Name"] == name]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    runs, cur, last_end = [], [], None
    for r in tr:
        s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and (s0 - last_end) / 1e6 > gap_ms:
            runs.append(cur)
            cur = []
        cur.append((e0 - s0) / 1e6)
        last_end = e0
    if cur:
        runs.append(cur)
    longest = max((len(r) for r in runs), default=0)
    run = next((r for r in runs if 2 * len(r) >= longest), [])
    if len(run) < steps:
        return {}
    t = sorted(run[-steps:])
    ks = [r for r in rows(d, "*kernel_stats.csv") if r["Name"] == name]
    out = {"kernel_name": name, "trace_timed_launches": steps,
           "trace_timed_mean_ms": sum(t) / len(t), "trace_timed_median_ms": t[len(t) // 2],
           "trace_run_launches": len(run)}
    if ks:
        out["kernel_stats_avg_ms_all_launches"] = float(ks[0]["AverageNs"]) / 1e6
        out["kernel_stats_calls"] = int(ks[0]["Calls"])
    return out


def timed_range(d, cfg):
    """The bench's timed launches of `cfg` as the traced run reports them
    when run with PPTK_BENCH_ROCTX=1 under `rocprofv3 --marker-trace
    --kernel-rename`: the kernels inside bench.py's ROCTx range
    "timed_<cfg>" are renamed to it, so kernel_stats.csv has a row of
    exactly the timed steps (no probe, autotune or settle launches)."""
    ks = [r for r in rows(d, "*kernel_stats.csv") if r["Name"] == f"timed_{cfg}"]
    if not ks:
        return {}
    return {"timed_range_calls": int(ks[0]["Calls"]),
            "timed_range_avg_ms": float(ks[0]["AverageNs"]) / 1e6,
            "timed_range_min_ms": float(ks[0]["MinNs"]) / 1e6,
            "timed_range_max_ms": float(ks[0]["MaxNs"]) / 1e6}


def op_counter(d, cname, regex):
    """Per-launch values of the kernels matching `regex` (all of them: an
    op's launches), and their durations."""
    import re
    v, t, names = [], [], set()
    for r in rows(d, "*counter_collection.csv"):
        if re.search(regex, r["Kernel_Name"]) and r["Counter_Name"] == cname:
            v.append(float(r["Counter_Value"]))
            t.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
            names.add(r["Kernel_Name"])
    return v, t, sorted(names)


def op_entry(spec):
    """op:NAME:REGEX:CHANGED_BYTES[:CALLS]=DIR_FETCH,DIR_WRITE -- a secondary
    op's HBM traffic per launch and its write amplification (WRITE_SIZE
    bytes / bytes the op must change).  With CALLS (the op calls the run
    made: an op may be several kernels), also the traffic per call."""
    head, dirs = spec.rsplit("=", 1)
    parts = head.split(":")
    calls = int(parts[4]) if len(parts) > 4 else 0
    changed, regex = parts[3], parts[2]
    dirs = dirs.split(",")
    f, fd, names = op_counter(dirs[0], "FETCH_SIZE", regex)
    w, wd, _ = op_counter(dirs[1], "WRITE_SIZE", regex)
    if not f or not w:
        return {"error": "no matching launches", "regex": regex}
    e = {"launches": len(f), "kernels": names,
         "hbm_read_bytes": sum(f) / len(f) * 1024 * 2,
         "hbm_write_bytes": sum(w) / len(w) * 1024,
         "pmc_pass_kernel_ms": sum(fd + wd) / len(fd + wd)}
    e["traffic_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
    # per kernel (an op made of several launches, e.g. the binned path)
    import re
    per = {}
    for cname, key in (("FETCH_SIZE", 0), ("WRITE_SIZE", 1)):
        for r in rows(dirs[key], "*counter_collection.csv"):
            if re.search(regex, r["Kernel_Name"]) and r["Counter_Name"] == cname:
                k = r["Kernel_Name"][:80]
                p = per.setdefault(k, {"launches": 0, "read": 0.0, "write": 0.0})
                if key == 0:
                    p["launches"] += 1
                    p["read"] += float(r["Counter_Value"]) * 1024 * 2
                else:
                    p["write"] += float(r["Counter_Value"]) * 1024
    e["per_kernel"] = {k: {"launches": v["launches"],
                           "read_bytes_per_launch": v["read"] / max(1, v["launches"]),
                           "write_bytes_per_launch": v["write"] / max(1, v["launches"])}
                       for k, v in per.items()}
    if calls:
        e["calls"] = calls
        e["traffic_bytes_per_call"] = (sum(f) * 2 + sum(w)) * 1024 / calls
    e["changed_bytes"] = int(changed)
    e["write_amplification"] = round(e["hbm_write_bytes"] / int(changed), 2)
    return e


def main():
    out = {}
    for arg in sys.argv[2:]:
        if arg.startswith("op:"):
            out["op_" + arg.split(":")[1]] = op_entry(arg)
            continue
        cfg, dirs = arg.split("=")
        dirs = dirs.split(",")
        fetch, fd, fname = counter(dirs[0], "FETCH_SIZE")
        write, wd, wname = counter(dirs[1], "WRITE_SIZE")
        e = {"launches": len(fetch), "pmc_kernel": fname, "pmc_kernel_write": wname,
             "fetch_size_kib": sum(fetch) / len(fetch), "write_size_kib": sum(write) / len(write)}
        e["hbm_read_bytes"] = e["fetch_size_kib"] * 1024 * 2
        e["hbm_write_bytes"] = e["write_size_kib"] * 1024
        e["traffic_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        e["pmc_pass_kernel_ms"] = sum(fd + wd) / len(fd + wd)
        if len(dirs) > 2:
            e.update(timed_launches(dirs[2], fname, int(os.environ.get("PMC_STEPS", "20"))))
            e.update(timed_range(dirs[2], cfg))
        out[cfg] = e
    json.dump(out, open(sys.argv[1], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
