"""BENCH TOOLING: end-to-end host-to-host rate of pptk_rx_batch (the LDP rx
loop's view: borrowed frames in host memory -> records in host memory),
for the staged path (pinned gather + H2D) and the zero-copy registered-ring
path (GPU reads the frames in place over PCIe).

    python tools/e2e.py [frames] [chunk]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pptk_amd.records import REC_DTYPE, diff_records
    from pptk_amd.rx import RxContext, ldp_packets
    from harness.synth import make_batch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    dev = torch.device("cuda", 0)
    out = {"frames": n, "chunk": chunk}
    for cfg in os.environ.get("E2E_CFGS", "c1500,c64").split(","):
        b = make_batch(cfg, n, dev)
        stride = b["stride"]
        ring = b["frames"][: n * stride + 64].cpu().numpy()     # pageable host "ring"
        slot = int(os.environ.get("E2E_SLOT", "0"))
        if slot > stride:
            # netmap-style fixed slots: frame i at i * slot (E2E_SLOT bytes)
            packed = ring
            ring = np.zeros(n * slot + 64, np.uint8)
            np.lib.stride_tricks.as_strided(ring, (n, stride), (slot, 1))[:] = \
                packed[: n * stride].reshape(n, stride)
            out["slot"] = slot
        ref = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        gt = int(os.environ.get("E2E_GATHER_THREADS", "8"))
        lib = os.environ.get("E2E_LIB")     # A/B: another build of the library
        ctx = RxContext(0, bytes(range(1, 17)), max_batch=chunk, max_frame=1518,
                        gather_threads=gt, lib_path=lib)
        out["gather_threads"] = gt
        out["lib"] = lib
        ctx.batch_device(b["frames"], n, stride=stride, fixed_len=b["fixed_len"], recs=ref)
        want = ref.cpu().numpy()
        pkts = ldp_packets(ring, np.arange(n, dtype=np.uint64) * max(stride, slot),
                           np.full(n, b["fixed_len"], np.uint16))
        res = {}
        # the records land in one array reused by every call, as in an rx
        # loop (a fresh 64 MB array per call faulted its pages in inside the
        # call's copy-out: E2E_FRESH_OUT=1 measures that way)
        fresh_out = bool(os.environ.get("E2E_FRESH_OUT"))
        outbuf = None if fresh_out else np.zeros(n, dtype=REC_DTYPE)
        out["fresh_out"] = fresh_out
        # E2E_REG_OUT=1: the record array registered with the context, so the
        # kernel writes the records into it in place (no copy back)
        reg_out = bool(os.environ.get("E2E_REG_OUT")) and outbuf is not None
        out["registered_out"] = reg_out
        if reg_out:
            ctx.register_ring(outbuf)
        for mode in os.environ.get("E2E_MODES", "staged,ring").split(","):
            if os.environ.get("E2E_FRESH") and res:    # one context per mode
                ctx.close()
                ctx = RxContext(0, bytes(range(1, 17)), max_batch=chunk, max_frame=1518,
                                gather_threads=gt, lib_path=lib)
                if reg_out:
                    ctx.register_ring(outbuf)
            if mode == "ring":
                ctx.register_ring(ring)
            got = ctx.batch_host(pkts, out=outbuf)          # warm-up (allocations)
            assert not diff_records(got, want), f"{cfg} {mode} parity"
            reps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < 3.0:
                ctx.batch_host(pkts, out=outbuf)
                reps += 1
            el = (time.perf_counter() - t0) / reps
            res[mode] = {"mpkts": round(n / el / 1e6, 2),
                         "frame_gbs": round(n * b["fixed_len"] / el / 1e9, 2),
                         "ms_per_batch": round(el * 1e3, 2)}
            if mode == "ring":
                ctx.unregister_ring(ring)
        out[cfg] = res
        if reg_out:
            ctx.unregister_ring(outbuf)
        ctx.close()
        del b, ref
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
