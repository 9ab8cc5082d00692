"""PROBE TOOLING: when does each wave of the rx grid (persistent or
oversubscribed) start and finish?
Needs the probe build (`make abvariant NAME=wt DEFS=-DPPTK_RX_WAVE_TIMES`,
copied to tools/ab_libs/wt.so, run with PPTK_RX_LIB=tools/ab_libs/wt.so):
every wave writes its start and end clock (s_memrealtime, 100 MHz).  For
C1500 and CMIX on the library's rings, after the settle launches: the
launch span, the spread of the waves' starts and ends, the end percentiles,
and the mean end per XCD group (block % 8).  One JSON line per config.

    PPTK_RX_LIB=tools/ab_libs/wt.so python tools/wave_times.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from pptk_amd.rx import RxContext, VARIANTS
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = bench.N_PER_GPU
    ctx = RxContext(0, bench.KEY)
    L = ctx._L
    L.pptk_rx_wave_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.pptk_rx_wave_times.restype = ctypes.c_int
    for cfg in sys.argv[1:] or ["c1500", "cmix"]:
        b = make_batch(cfg, n, dev)
        kw = (dict(stride=b["stride"], fixed_len=b["fixed_len"]) if "off" not in b else
              dict(off=b["off"], lens=b["lens"], max_len=b["max_len"]))
        recs, rep = bench.ring_buffers(ctx, b, n, dev, False)
        time.sleep(max(0.0, rep["_freed_at"] + rep["freed_bytes"] / bench.SCRUB_BYTES_PER_S
                       - time.perf_counter()))
        ctx.autotune(b["frames"], n, recs=recs, reps=5, **kw)
        out = []
        for rep_i in range(5):
            for _ in range(30):
                ctx.batch_device(b["frames"], n, recs=recs, **kw)
            torch.cuda.synchronize()
            buf = np.zeros(2 * 65536, dtype=np.uint64)
            nw = L.pptk_rx_wave_times(buf.ctypes.data, 65536)
            assert nw > 0, nw
            t = buf[:2 * nw].reshape(nw, 2).astype(np.int64)
            t0 = t[:, 0].min()
            st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0     # us
            grp = (np.arange(nw) // 4) % 8
            # concurrency over time: how many waves run at once, and how
            # long the launch runs with fewer than 90 % of the peak
            ev = np.concatenate([np.stack([st, np.ones(nw)], 1), np.stack([en, -np.ones(nw)], 1)])
            ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
            act = np.cumsum(ev[:, 1])
            peak = float(act.max())
            hi = ev[act >= 0.9 * peak, 0]
            out.append({
                "waves": int(nw), "peak_active": peak,
                "util": float((en - st).sum() / (peak * en.max())),
                "tail_below90_us": float(en.max() - hi.max()) if len(hi) else None,
                "span_us": float(en.max()), "start_spread_us": float(st.max()),
                "end_pct_us": {p: float(np.percentile(en, p)) for p in (0, 10, 50, 90, 99, 100)},
                "tail_frac": float((en.max() - np.median(en)) / en.max()),
                "busy_frac": float((en - st).sum() / (nw * en.max())),
                "end_by_group_us": [float(en[grp == k].mean()) for k in range(8)]})
            del buf
        del recs
        torch.cuda.empty_cache()
        print(json.dumps({"config": cfg, "waves": nw,
                          "variant": VARIANTS[L.pptk_rx_last_variant(ctx._ctx)],
                          "runs": out}), flush=True)


if __name__ == "__main__":
    main()
