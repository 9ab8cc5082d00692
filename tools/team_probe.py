"""PROBE TOOLING: the rx kernel's team-round load pattern on a CMIX batch,
nothing computed (tools/team_probe.hip), plain vs non-temporal loads and
what the lanes past a frame's end load; beside the SOL kernel's linear
spans (tools/rwmix.py sol_ms).  Interleaved in one process; prints JSON.

    python tools/team_probe.py [cmix] [--rounds 3] [--out FILE]
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

SETTINGS = [("rx_T16S6", 0, -1), ("plain_clamp", 0, 0), ("nt_clamp", 1, 0), ("plain_pred", 0, 1), ("nt_pred", 1, 1),
            ("nt_clamp_tail", 1, 2), ("plain_buf", 0, 3), ("nt_buf", 1, 3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg", nargs="?", default="cmix")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    from harness.synth import make_batch
    L = ctypes.CDLL(os.path.join(HERE, "libteam_probe.so"))
    vp = ctypes.c_void_p
    L.team_probe_run.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, vp, vp]
    dev = torch.device("cuda", 0)
    n = 16 * 1024 * 1024
    b = make_batch(args.cfg, n, dev)
    assert "off" in b, "an offset-described config"
    recs = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    sink = torch.zeros(64, dtype=torch.int32, device=dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    s = torch.cuda.current_stream(dev)

    from pptk_amd.rx import RxContext
    ctx = RxContext(0, bytes(range(1, 17)))
    ctx.set_tuning(3, 32)                 # the rx kernel itself: T16S6, plain loads, NT stores
    recs_rx = recs.view(n, 64)

    def run(nt, mode):
        if mode < 0:
            ctx.batch_device(b["frames"], n, recs=recs_rx, off=b["off"], lens=b["lens"],
                             max_len=b["max_len"])
            return
        rc = L.team_probe_run(b["frames"].data_ptr(), b["off"].data_ptr(), b["lens"].data_ptr(), n,
                              recs.data_ptr(), nt, mode, ncu * 2, sink.data_ptr(), vp(s.cuda_stream))
        if rc:
            raise SystemExit(f"team_probe_run {nt} {mode}: {rc}")

    for _, nt, mode in SETTINGS:
        run(nt, mode)
    torch.cuda.synchronize()
    times = {}
    for r in range(args.rounds):
        for name, nt, mode in SETTINGS:
            run(nt, mode)
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(nt, mode)
                e1.record()
                torch.cuda.synchronize()
                times.setdefault(name, []).append(e0.elapsed_time(e1))
        print(f"round {r} done", file=sys.stderr, flush=True)
    res = {"cfg": args.cfg, "frames": n, "frame_bytes": b["bytes"]}
    for k, ts in times.items():
        ts.sort()
        res[k] = round(ts[len(ts) // 2], 4)
    os.environ["RWMIX_SOL_SHAPES"] = "1"
    from harness.rwmix import sol_ms
    ms, how = sol_ms(b["frames"], n, recs.view(n, 64), 4096, off=b["off"], lens=b["lens"])
    res["sol_ms"], res["sol_shapes"] = round(ms, 4), how.get("shapes")
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
