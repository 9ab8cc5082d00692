"""Generate the golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists).

Inputs are the deterministic frames of tests/framegen.py.  Expected records
come from oracle/_ref/libpptkref.so: the reference's iphdr/ipcksum.c,
iphdr/iphdr.c, misc/siphash.h, iphash/iphash.c compiled unmodified, composed
by oracle/refgen.c.  Nothing from the reference is stored here: each .npz
holds only frames (inputs) and the 64-byte records (outputs).

    python tests/golden/gen_golden.py [set ...]     (default: every set)

permit.npz additionally holds rate-limiter cases: token arrays before/after
and per-frame verdicts of the reference's ip_permitted / ipv6_permitted
called once per subject frame in frame order (oracle/refgen.c
ref_permit_batch), and refills by the reference's own timer function
(ref_tokens_refill).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import framegen  # noqa: E402
from oracle.oracle import Reference, build, make_opts  # noqa: E402

KEY = bytes(range(1, 17))          # iphash/iphashtest5.c:59 key {1..16}
BITS4, BITS6, HASH_SIZE = 24, 48, 4096

SETS = {
    "edge": lambda: framegen.gen_edge(),
    "fuzz": lambda: framegen.gen_fuzz(2000),
    "c64": lambda: framegen.gen_c64(4096),
    "c1500": lambda: framegen.gen_c1500(1024),
    "cmix": lambda: framegen.gen_cmix(2048),
}


PERMIT_HASH = 64                   # few buckets: long token runs, collisions
PERMIT_INIT = (3, 300, 70000)      # tiny / small / full entries (iphash.h:53-61)


def gen_permit(ref):
    buf, off, lens = framegen.gen_permit()
    opts = make_opts(KEY, BITS4, BITS6, PERMIT_HASH)
    recs = ref.rx_batch(buf, off, lens, opts=opts, with_bucket=True)
    rng = np.random.default_rng(0x7E57)
    out = dict(buf=buf, off=off, len=lens, recs=recs.view(np.uint8).reshape(-1, 64),
               key=np.frombuffer(KEY, dtype=np.uint8),
               iphash=np.array([BITS4, BITS6, PERMIT_HASH], dtype=np.uint32))
    cases = []
    for fam, bits in ((4, BITS4), (6, BITS6)):
        for init in PERMIT_INIT:
            for sub in (None, "rand"):
                tok = rng.integers(0, init + 1, PERMIT_HASH).astype(np.uint32)
                subj = None if sub is None else (rng.random(len(off)) < 0.7).astype(np.uint8)
                v, t2 = ref.permit_batch(KEY, recs, fam, bits, subj, PERMIT_HASH, init, tok)
                cases.append((fam, init, tok, subj, v, t2))
    out["case_meta"] = np.array([[c[0], c[1], c[3] is not None] for c in cases], dtype=np.uint32)
    out["case_tok_in"] = np.stack([c[2] for c in cases])
    out["case_subject"] = np.stack([c[3] if c[3] is not None else np.ones(len(off), np.uint8)
                                    for c in cases])
    out["case_verdict"] = np.stack([c[4] for c in cases])
    out["case_tok_out"] = np.stack([c[5] for c in cases])
    refills = []
    for init, add in ((250, 7), (1000, 300), (100000, 99999), (5, 200)):
        for k in range(PERMIT_HASH // 16):
            tok = rng.integers(0, init + 1, PERMIT_HASH).astype(np.uint32)
            refills.append((init, add, k, tok, ref.tokens_refill(PERMIT_HASH, 16, init, add, k,
                                                                 tok)))
    out["refill_meta"] = np.array([[r[0], r[1], r[2] * 16, r[2] * 16 + 16] for r in refills],
                                  dtype=np.uint32)
    out["refill_in"] = np.stack([r[3] for r in refills])
    out["refill_out"] = np.stack([r[4] for r in refills])
    return out


def main():
    build()
    ref = Reference()
    opts = make_opts(KEY, BITS4, BITS6, HASH_SIZE)
    want = set(sys.argv[1:]) or set(SETS) | {"permit"}
    if "permit" in want:
        path = os.path.join(HERE, "permit.npz")
        np.savez_compressed(path, **gen_permit(ref))
        print(f"permit -> {os.path.getsize(path)} B")
    for name, fn in SETS.items():
        if name not in want:
            continue
        buf, off, lens = fn()
        recs = ref.rx_batch(buf, off, lens, opts=opts, with_bucket=True)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, buf=buf, off=off, len=lens,
                            recs=recs.view(np.uint8).reshape(-1, 64),
                            key=np.frombuffer(KEY, dtype=np.uint8),
                            iphash=np.array([BITS4, BITS6, HASH_SIZE], dtype=np.uint32))
        print(f"{name}: {len(off)} frames, {buf.nbytes} B -> {os.path.getsize(path)} B")


if __name__ == "__main__":
    main()
