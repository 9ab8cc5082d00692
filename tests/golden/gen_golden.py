"""Generate the golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists).

Inputs are the deterministic frames of tests/framegen.py.  Expected records
come from oracle/_ref/libpptkref.so: the reference's iphdr/ipcksum.c,
iphdr/iphdr.c, misc/siphash.h, iphash/iphash.c compiled unmodified, composed
by oracle/refgen.c.  Nothing from the reference is stored here: each .npz
holds only frames (inputs) and the 64-byte records (outputs).

    python tests/golden/gen_golden.py
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


def main():
    build()
    ref = Reference()
    opts = make_opts(KEY, BITS4, BITS6, HASH_SIZE)
    for name, fn in SETS.items():
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
