"""PROBE TOOLING: C1500-shaped tiles read with the record run written right
after each tile, or held until a chip-wide clock period begins (global write
phases, tools/epoch_probe.hip), on the library's placed rings (the bench's
allocation), beside the rx kernel on the same frames.  Interleaved in one
process; prints JSON (median ms per setting).

    python tools/epoch_probe.py [--rounds 4] [--out FILE]
    EPOCH_SWEEP=stagger|depth|writer (default stagger)
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    import bench
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    L = ctypes.CDLL(os.path.join(HERE, "libepoch_probe.so"))
    vp = ctypes.c_void_p
    L.epoch_probe_run.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_int,
                                  ctypes.c_uint64, ctypes.c_int, vp, vp]
    dev = torch.device("cuda", 0)
    n = 16 * 1024 * 1024
    ctx = RxContext(0, bytes(range(1, 17)))
    b = make_batch("c1500", n, dev)
    recs, report = bench.ring_buffers(ctx, b, n, dev, False)
    # past the driver's scrub of what the placement probe freed (bench.py's
    # settle rule), then warm
    import time
    wait = report["_freed_at"] + report["freed_bytes"] / bench.SCRUB_BYTES_PER_S - time.perf_counter()
    if wait > 0:
        time.sleep(wait)
    frames = b["frames"]
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    sink = torch.zeros(64, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    ntiles = n // 64
    settings = [("rx", None, 0, 0)]
    sweep = os.environ.get("EPOCH_SWEEP", "stagger")
    if sweep == "writer":   # a fifth wave per workgroup writes the runs
        for bpc in (2, 3):
            settings.append((f"tile_end_b{bpc}", 0, 1, bpc))
            settings.append((f"phase30us_b{bpc}", 1, 3000, bpc))
            settings.append((f"writer_b{bpc}", 5, 1, bpc))
            for per in (2000, 3000, 4000):
                settings.append((f"writer_phase{per // 100}us_b{bpc}", 6, per, bpc))
    elif sweep == "depth":
        for bpc in (2, 3):
            settings.append((f"tile_end_b{bpc}", 0, 1, bpc))
            for per in (2000, 3000, 4000, 6000):
                settings.append((f"phase{per // 100}us_b{bpc}", 1, per, bpc))
        for per in (3000, 4000, 6000, 8000, 12000):   # two tiles' runs held (2 blocks per CU)
            settings.append((f"phase2x{per // 100}us_b2", 2, per, 2))
    else:   # all waves at once vs the XCDs (or two halves) in turn, 3 blocks per CU
        settings.append(("tile_end_b3", 0, 1, 3))
        for per in (3000, 4000):
            settings.append((f"phase{per // 100}us_b3", 1, per, 3))
            settings.append((f"phase{per // 100}us_xcd8_b3", 3, per, 3))
            settings.append((f"phase{per // 100}us_half2_b3", 4, per, 3))

    def run(mode, per, bpc):
        if mode is None:
            ctx.batch_device(frames, n, recs=recs, stride=1500, fixed_len=1500)
            return
        rc = L.epoch_probe_run(frames.data_ptr(), ntiles, 96000, recs.data_ptr(), mode, per,
                               ncu * bpc, sink.data_ptr(), vp(s.cuda_stream))
        if rc:
            raise SystemExit(f"epoch_probe_run {mode} {per} {bpc}: {rc}")

    for _, mode, per, bpc in settings:
        run(mode, per, bpc)
    torch.cuda.synchronize()
    times = {}
    for r in range(args.rounds):
        for name, mode, per, bpc in settings:
            run(mode, per, bpc)
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(mode, per, bpc)
                e1.record()
                torch.cuda.synchronize()
                times.setdefault(name, []).append(e0.elapsed_time(e1))
        print(f"round {r} done", file=sys.stderr, flush=True)
    res = {"frames": n, "placement": {k: v for k, v in report.items() if not k.startswith("_")},
           "rx_variant": ctx.last_variant()}
    for k, ts in times.items():
        ts.sort()
        res[k] = round(ts[len(ts) // 2], 4)
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
