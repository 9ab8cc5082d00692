"""BENCH TOOLING: read/write mix microbenchmark (tools/rwmix.hip).

    python tools/rwmix.py            -> one JSON line: ms per setting

Reads 24 GiB worth of tiles (a 6 GiB buffer read 4 times over would hit
the caches differently, so the buffer is the full 24 GiB) and writes 1/24
of that, in bursts of wb bytes per rb-byte tile, for several burst sizes at
the same read:write ratio; plus a read-only reference.  Store modes (the
`nt` key, see rwmix.hip): 1 = non-temporal loads and stores (the rx
kernel's policy), 3 = stores independent of the loads, 5 = stores into a
reused 32 MiB window, 9 = ordinary (write-back) stores, 13 = ordinary stores
into a reused 1 MiB window (they never leave L2)."""
import ctypes
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def _lib():
    L = ctypes.CDLL(os.path.join(HERE, "librwmix.so"))
    vp = ctypes.c_void_p
    L.rwmix_run.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                            ctypes.c_int, ctypes.c_int, vp, vp]
    L.sol_run.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint64, ctypes.c_uint32,
                          ctypes.c_uint32, ctypes.c_int, ctypes.c_int, vp, vp]
    L.sol_run.restype = ctypes.c_int
    L.sol_run_phased.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint64,
                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, vp,
                                 ctypes.c_uint32, vp]
    L.sol_run_phased.restype = ctypes.c_int
    L.rwdefer_run.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                              ctypes.c_int, ctypes.c_int, vp, vp]
    L.rwdefer_run.restype = ctypes.c_int
    L.rwstage_run.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                              ctypes.c_int, ctypes.c_uint32, ctypes.c_int, vp, vp]
    L.rwstage_run.restype = ctypes.c_int
    return L


def sol_ms(inp, n, out, wb, rb=0, off=None, lens=None, reps=6):
    """Speed of light of an rx launch's traffic on this GPU: the fastest of
    several trivial kernels (tools/rwmix.hip sol_kernel: plain / non-
    temporal, 4 or 16 loads per lane in flight, 2 / 4 / 8 blocks per CU)
    reading the launch's frame bytes in 64-frame tiles -- fixed tiles of rb
    bytes, or (off/lens given: frames packed in batch order) each tile's
    actual span after its descriptors -- and writing wb record bytes per
    tile; the non-temporal shapes also with the rx kernel's global write
    phases (period ~0.75 of a tile's duration at 5.5 TB/s, as
    rx_capi.hip phase_ticks_for sets it).  The grids go past what fits at
    once (32 and 128 blocks per CU: ~8 and ~2 tiles per wave for 16 M
    frames), as the rx kernels' oversubscribed grids do (DESIGN.md §7
    "Round 6: grids"); their phase period follows the 8 blocks per CU that
    are resident.  Returns (ms, setting)."""
    import torch
    L = _lib()
    dev = inp.device
    ntiles = n // 64
    assert ntiles > 0 and out.numel() >= ntiles * wb and wb % 16 == 0
    gather = off is not None
    if not gather:
        assert inp.numel() >= ntiles * rb
    sink = torch.zeros(64, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    best = (float("inf"), None)
    shapes = {}
    if gather:   # the tiles' mean span
        tile_bytes = (int(off[ntiles * 64 - 1].item()) + int(lens[ntiles * 64 - 1].item() & 0xFFFF)
                      - int(off[0].item())) / ntiles
    else:
        tile_bytes = rb
    for mode in (0, 1, 4, 5, 9, 13):
        m = (mode & 7) | (2 if gather else 0)
        phased = bool(mode & 8)
        for mult in (2, 4, 8, 32, 128):
            period = max(100, int(tile_bytes * ncu * min(mult, 8) * 4 * 3 / 4 / 55000))
            ts = []
            for k in range(reps + 2):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                args = (inp.data_ptr(), off.data_ptr() if gather else None,
                        lens.data_ptr() if gather else None, n, out.data_ptr(), ntiles, rb, wb, m,
                        ncu * mult, sink.data_ptr())
                if phased:
                    rc = L.sol_run_phased(*args, period, ctypes.c_void_p(s.cuda_stream))
                else:
                    rc = L.sol_run(*args, ctypes.c_void_p(s.cuda_stream))
                b.record()
                torch.cuda.synchronize(dev)
                assert rc == 0
                if k >= 2:
                    ts.append(a.elapsed_time(b))
            ts.sort()
            med = ts[len(ts) // 2]
            shapes[f"{'nt' if mode & 1 else 'plain'}_l{4 if mode & 4 else 16}_b{mult}"
                   + ("_phased" if phased else "")] = round(med, 4)
            if med < best[0]:
                best = (med, {"nt": bool(mode & 1), "loads_in_flight": 4 if mode & 4 else 16,
                              "blocks_per_cu": mult * 1, "write_phases": phased})
    if os.environ.get("RWMIX_SOL_SHAPES"):   # every shape's median (A/B probes)
        best[1]["shapes"] = shapes
    return best


def mix_ms(inp, rb, ntiles, out, wb, nt=1, reps=8):
    """Median ms of the trivial stream over the same bytes as an rx launch:
    ntiles tiles of rb bytes read from torch uint8 CUDA tensor `inp` (only
    read), wb bytes written per tile into `out` -- the speed of light of
    that read/write mix on this GPU (no parsing, no hashing, no sums)."""
    import torch
    assert rb % 16 == 0 and wb % 16 == 0
    assert inp.numel() >= ntiles * rb and out.numel() >= ntiles * wb
    L = _lib()
    dev = inp.device
    sink = torch.zeros(64, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    grid = torch.cuda.get_device_properties(dev).multi_processor_count * 2
    ts = []
    for k in range(reps + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        L.rwmix_run(inp.data_ptr(), out.data_ptr(), ntiles, rb, wb, nt, grid, sink.data_ptr(),
                    ctypes.c_void_p(s.cuda_stream))
        b.record()
        torch.cuda.synchronize(dev)
        if k >= 2:
            ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    import torch
    L = _lib()
    vp = ctypes.c_void_p
    dev = torch.device("cuda", 0)
    total = 24 * 1024 ** 3
    inp = torch.empty(total, dtype=torch.uint8, device=dev)
    inp.fill_(1)
    out = torch.empty(total // 24 + (1 << 20), dtype=torch.uint8, device=dev)
    sink = torch.zeros(64, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    settings = [(96 << 10, 0), (96 << 10, 4 << 10), (1536 << 10, 64 << 10)]
    res = {}
    for rounds in range(2):
        for nt in (1, 5, 9, 13):
            for grid_mult in (2,):
                for rb, wb in settings:
                    ntiles = total // rb
                    key = f"rb{rb >> 10}k_wb{wb >> 10}k_nt{nt}_g{grid_mult}"
                    ts = []
                    for k in range(4):
                        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        a.record()
                        L.rwmix_run(inp.data_ptr(), out.data_ptr(), ntiles, rb, wb, nt,
                                    ncu * grid_mult, sink.data_ptr(), vp(s.cuda_stream))
                        b.record()
                        torch.cuda.synchronize()
                        if k:
                            ts.append(a.elapsed_time(b))
                    res.setdefault(key, []).extend(ts)
    out_ = {k: round(sorted(v)[len(v) // 2], 4) for k, v in res.items()}
    print(json.dumps(out_))


if __name__ == "__main__":
    main()
