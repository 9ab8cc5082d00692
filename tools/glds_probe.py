"""PROBE TOOLING: HBM read rate of direct global->LDS loads against vector
loads on C1500-shaped tiles (tools/glds_probe.hip), interleaved in one
process on one buffer.  Prints one JSON object (GB/s of frame bytes read,
median per variant).

    python tools/glds_probe.py [--rounds 3] [--reps 5] [--out FILE]
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

# (name, mode, depth, aux, blocks per CU)
VARIANTS = [
    ("vec_nt_d8_b2", 0, 8, 1, 2), ("vec_nt_d8_b4", 0, 8, 1, 4), ("vec_nt_d8_b8", 0, 8, 1, 8),
    ("vec_d8_b4", 0, 8, 0, 4), ("vec_nt_d16_b2", 0, 16, 1, 2), ("vec_nt_d16_b4", 0, 16, 1, 4),
    ("vec_nt_d24_b2", 0, 24, 1, 2),
    ("glds_d8_b4", 1, 8, 0, 4), ("glds_nt_d8_b2", 1, 8, 2, 2), ("glds_nt_d8_b4", 1, 8, 2, 4),
    ("glds_d16_b2", 1, 16, 0, 2), ("glds_nt_d16_b2", 1, 16, 2, 2), ("glds_nt_d32_b1", 1, 32, 2, 1),
    ("gldsrd_nt_d8_b4", 2, 8, 2, 4), ("gldsrd_nt_d16_b2", 2, 16, 2, 2),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ins", type=int, default=96, help="KB per tile (1 KB per wave-instruction)")
    ap.add_argument("--gib", type=int, default=24)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    L = ctypes.CDLL(os.path.join(HERE, "libglds_probe.so"))
    vp = ctypes.c_void_p
    L.glds_probe_run.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint32, vp, vp, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    ntiles = (args.gib << 30) // (args.ins * 1024)
    buf = torch.empty(ntiles * args.ins * 1024, dtype=torch.uint8, device=dev)
    buf.fill_(0x5a)
    recs = torch.empty(ntiles * 4096, dtype=torch.uint8, device=dev)
    recs.zero_()
    out = torch.zeros(1024, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()
    nbytes = ntiles * args.ins * 1024

    def run(v, with_recs):
        _, mode, depth, aux, bpc = v
        rc = L.glds_probe_run(buf.data_ptr(), ntiles, args.ins, recs.data_ptr() if with_recs else None,
                              out.data_ptr(), mode, depth, aux, ncu * bpc, vp(s.cuda_stream))
        if rc:
            raise SystemExit(f"glds_probe_run {v}: {rc}")

    # warm the clocks and the code objects
    for v in VARIANTS:
        run(v, False)
    torch.cuda.synchronize()
    times = {}
    for r in range(args.rounds):
        for v in VARIANTS:
            for wr in (False, True):
                key = v[0] + ("+recs" if wr else "")
                run(v, wr)
                for _ in range(args.reps):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    run(v, wr)
                    b.record()
                    torch.cuda.synchronize()
                    times.setdefault(key, []).append(a.elapsed_time(b))
        print(f"round {r} done", file=sys.stderr, flush=True)
    res = {"tile_bytes": args.ins * 1024, "ntiles": ntiles, "read_bytes": nbytes, "results": {}}
    for k, ts in times.items():
        ts.sort()
        ms = ts[len(ts) // 2]
        res["results"][k] = {"ms": round(ms, 4), "read_gbs": round(nbytes / ms / 1e6, 1),
                             "min_ms": round(ts[0], 4)}
    line = json.dumps(res)
    print(line)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
