"""BENCH TOOLING: the rate limiter's denying regime alone (dense keys of a
C64 batch, 128 tokens per bucket before each batch), for rocprofv3 passes on
its kernels.

    python tools/permit_probe.py [--reps R] [--tokens T] [--records]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pptk_amd.rx import RxContext
    from harness.synth import make_batch
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tokens", type=int, default=128)
    ap.add_argument("--records", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, hs = 1 << 24, 1 << 16
    b = make_batch("c64", n, dev)
    ctx = RxContext(0, bytes(range(1, 17)), 24, 0, hs)
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    recs = ctx.batch_device(b["frames"], n, stride=b["stride"], fixed_len=b["fixed_len"],
                            key_out=keys)
    del b
    tok = torch.empty(hs, dtype=torch.int32, device=dev)
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    scratch = torch.empty(ctx._L.pptk_rx_permit_scratch_bytes(n, hs), dtype=torch.uint8,
                          device=dev)
    for _ in range(args.reps):
        tok.fill_(args.tokens)
        if args.records:
            ctx.permit_device(recs, 4, tok, verdict=verdict, scratch=scratch)
        else:
            ctx.permit_keys_device(keys, 4, tok, verdict=verdict, scratch=scratch)
    torch.cuda.synchronize()
    v = verdict.cpu()
    print({"permitted": int((v == 1).sum()), "denied": int((v == 0).sum())})


if __name__ == "__main__":
    main()
