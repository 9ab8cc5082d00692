"""BENCH TOOLING: does the same launch on the same placed buffers drift with
the GPU's clocks, power or temperature?  (a placed
pair alternated between 4.23 and 4.48 ms within one process.)

    python tools/clock_probe.py [--seconds S] [--group G]

Places a C1500 batch as bench.py does, then runs back-to-back launches for
S seconds; every G launches it records the group's median launch time
(HIP events) and one read-only amdsmi sample of this GPU's metrics (clocks,
socket power, temperatures, throttle status).  One JSON object per line:
first the placement report, then one line per group."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEYS = ("clk", "power", "temperature", "throttle", "energy", "activity")


def smi_handle(dev_index):
    """The amdsmi handle of torch device `dev_index` (matched by PCI bus),
    or None when amdsmi is unavailable."""
    try:
        import amdsmi
        import torch
        amdsmi.amdsmi_init()
        p = torch.cuda.get_device_properties(dev_index)
        want = int(getattr(p, "pci_bus_id", -1))
        for h in amdsmi.amdsmi_get_processor_handles():
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)      # "0000:bb:dd.f"
            if int(bdf.split(":")[1], 16) == want:
                return amdsmi, h
    except Exception as e:   # noqa: BLE001 (diagnostic tool)
        print(json.dumps({"amdsmi": f"unavailable: {e!r}"}), flush=True)
    return None, None


def sample(amdsmi, h):
    if h is None:
        return {}
    out = {}
    try:
        m = amdsmi.amdsmi_get_gpu_metrics_info(h)
        for k, v in m.items():
            if any(s in k for s in KEYS) and not isinstance(v, (list, tuple, dict)):
                out[k] = v
            elif any(s in k for s in ("gfxclk", "fclk", "uclk")) and isinstance(v, (list, tuple)):
                vals = [x for x in v if isinstance(x, int) and x < 65535]
                if vals:
                    out[k] = [min(vals), max(vals)]
    except Exception as e:   # noqa: BLE001
        out["error"] = repr(e)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--group", type=int, default=50)
    ap.add_argument("--n", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--free-gb", type=str, default="",
                    help="comma list: after the run, allocate and free this many GB, "
                         "then run again for --seconds (does freeing memory slow the "
                         "launches that follow?)")
    args = ap.parse_args()
    import torch
    import bench
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    amdsmi, h = smi_handle(0)
    print(json.dumps({"idle": sample(amdsmi, h)}, default=str), flush=True)
    n = args.n
    ctx = RxContext(0, bench.KEY)
    b = make_batch("c1500", n, dev)
    kw = dict(stride=1500, fixed_len=1500)
    recs, rep = bench.placed_buffers(ctx, b, n, dev, False, kw)
    print(json.dumps({"placement": {k: rep[k] for k in ("chosen", "chosen_ms",
                                                          "as_allocated_ms")}}), flush=True)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.group)]

    def series(tag):
        t0 = time.perf_counter()
        g = 0
        while time.perf_counter() - t0 < args.seconds:
            for a, z in ev:
                a.record()
                ctx.batch_device(b["frames"], n, recs=recs, **kw)
                z.record()
            s = sample(amdsmi, h)          # while the group's tail is running
            torch.cuda.synchronize(dev)
            ts = sorted(a.elapsed_time(z) for a, z in ev)
            print(json.dumps({"phase": tag, "g": g, "t": round(time.perf_counter() - t0, 2),
                              "ms_median": round(ts[len(ts) // 2], 4),
                              "ms_min": round(ts[0], 4), "ms_max": round(ts[-1], 4),
                              "smi": s}, default=str), flush=True)
            g += 1

    series("after_placement")
    for gb in [float(x) for x in args.free_gb.split(",") if x]:
        blk = [torch.empty(1 << 30, dtype=torch.uint8, device=dev) for _ in range(int(gb))]
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        del blk
        torch.cuda.empty_cache()
        print(json.dumps({"freed_gb": gb, "free_call_s": round(time.perf_counter() - t, 3)}),
              flush=True)
        series(f"after_free_{gb:g}gb")


if __name__ == "__main__":
    main()
