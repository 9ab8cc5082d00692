"""BENCH TOOLING: would a two-pass tx (compute the checksums while streaming
into a small side array, then scatter the 2-byte fields into the frames in
a second pass without the read stream beside it) beat the in-place tx?

    python tools/tx_split_probe.py

Times, on one C1500 batch: the in-place tx kernel; a strided torch write
of the two checksum fields of every frame (bytes 24-25 and 50-51) alone;
and a plain 64 MB side-array write.  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps=10):
    import torch
    ts = []
    for k in range(reps + 2):
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        z.record()
        torch.cuda.synchronize()
        if k >= 2:
            ts.append(a.elapsed_time(z))
    ts.sort()
    return round(ts[len(ts) // 2], 4)


def main():
    import torch
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    dev = torch.device("cuda", 0)
    n = 16 * 1024 * 1024
    ctx = RxContext(0, bytes(range(1, 17)))
    b = make_batch("c1500", n, dev)
    fr = b["frames"][: n * 1500].view(n, 1500)
    vals = torch.randint(0, 255, (n, 2), dtype=torch.uint8, device=dev)
    side = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    out = {
        "tx_inplace_ms": timed(lambda: ctx.tx_cksum_device(b["frames"], n, stride=1500,
                                                           fixed_len=1500)),
        "scatter_one_field_ms": timed(lambda: fr[:, 24:26].copy_(vals)),
        "scatter_two_fields_ms": timed(lambda: (fr[:, 24:26].copy_(vals), fr[:, 50:52].copy_(vals))),
        "side_array_write_ms": timed(lambda: side.fill_(7)),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
