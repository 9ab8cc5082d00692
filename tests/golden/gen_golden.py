"""Generate the golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists).

Inputs are the deterministic frames of tests/framegen.py.  Expected records
come from oracle/_ref/libpptkref.so: the reference's iphdr/ipcksum.c,
iphdr/iphdr.c, misc/siphash.h, iphash/iphash.c compiled unmodified, composed
by oracle/refgen.c.  Nothing from the reference is stored here: each .npz
holds only frames (inputs) and the 64-byte records (outputs).

    python tests/golden/gen_golden.py [set ...]     (default: every set)

tx.npz holds tx-side cases: frames with scrambled checksum fields and the
same frames after the reference's ip_set_hdr_cksum_calc /
tcp/udp(6)_set_cksum_calc (oracle/refgen.c ref_tx_batch).

rewrite.npz holds header-rewrite cases (pptk_tx_rewrite_device): per
golden set, frames with some IPv4 TTLs set to 0 or 1 and some UDP checksums
to 0 (inputs), random per-frame rewrite entries (ops, new addresses and
ports), and the frames after the reference's ip_decr_ttl_cksum_update /
ip_set_src/dst_cksum_update / tcp/udp_set_src/dst_port_cksum_update
(oracle/refgen.c ref_rewrite_batch) with the per-frame status.

mss.npz holds TCP MSS-clamping cases (pptk_tcp_mss_clamp_device): the
framegen.gen_mss frames and, per (mss, flags) case, the changed bytes and
per-frame status after the reference's tcp_parse_options +
tcp_set_mss_cksum_update (oracle/refgen.c ref_mss_clamp_batch).

tcpopt.npz holds kept-API cases for the TCP option functions: TCP headers
(framegen.tcp_headers), the reference's tcp_parse_options /
tcp_find_sack_ts_headers / tcp_find_sack_header results on them, and each
header after one option rewrite (tcp_set_mss / disable_sack /
adjust_sack_2 / adjust_tsval / adjust_tsecho / set_ack_off / seq / ack /
window *_cksum_update; oracle/refgen.c ref_tcp_opt_op).  Inputs on which
the reference never returns are marked and not run.

frag.npz holds fragment side records (struct pptk_rx_frag) made by the
reference's ip_id / ip_frag_off / ip_more_frags / ip_dont_frag and
ipv6_const_proto_hdr_2 (oracle/refgen.c ref_frag_batch): a dedicated
fragment set (framegen.gen_frag) with its 64-byte records, and the side
records of the edge, fuzz and cmix sets.

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
    "icmp": lambda: framegen.gen_icmp(1500),
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


def scramble_cksums(z, rng):
    """Copy of z's buffer with random bytes in the IPv4 header and TCP/UDP
    checksum fields of every frame the record composition parses."""
    from pptk_amd.records import F_IPV6, F_L4, F_MALFORMED, F_PARSED, as_records
    buf = z["buf"].copy()
    rec = as_records(z["recs"])
    for i, o in enumerate(z["off"]):
        r, f = rec[i], int(o)
        fl = int(r["flags"])
        if not fl & F_PARSED or fl & F_MALFORMED:
            continue
        if not fl & F_IPV6:
            p = f + int(r["l3_off"]) + 10
            buf[p:p + 2] = rng.integers(0, 256, 2)
        if fl & F_L4:
            p = f + int(r["l4_off"]) + (16 if int(r["proto"]) == 6 else 6)
            buf[p:p + 2] = rng.integers(0, 256, 2)
    return buf


def gen_tx(ref):
    """Tx-side fixtures over the golden sets: random bytes in every parsed
    frame's checksum fields (inputs), and the reference's
    *_set_cksum_calc result.  Stored as byte positions into the set's buffer
    with the scrambled and the expected bytes (the setters change nothing
    else, which the tests check)."""
    rng = np.random.default_rng(0x7C)
    out = {}
    for name in ("edge", "fuzz", "cmix", "c64"):
        z = dict(np.load(os.path.join(HERE, f"{name}.npz")))
        buf_in = scramble_cksums(z, rng)
        buf_out = ref.tx_batch(buf_in, z["off"], z["len"])
        pos = np.nonzero((buf_in != z["buf"]) | (buf_out != buf_in))[0]
        out[f"{name}_pos"] = pos.astype(np.uint64)
        out[f"{name}_in"] = buf_in[pos]
        out[f"{name}_out"] = buf_out[pos]
    return out


def rewrite_inputs(z, rng):
    """Copy of z's buffer with the TTL of ~1/4 of the parsed IPv4 frames set
    to 0 or 1 and the checksum of ~1/4 of the UDP frames set to 0."""
    from pptk_amd.records import F_IPV6, F_L4, F_MALFORMED, F_PARSED, as_records
    buf = z["buf"].copy()
    rec = as_records(z["recs"])
    for i, o in enumerate(z["off"]):
        r, f = rec[i], int(o)
        fl = int(r["flags"])
        if not fl & F_PARSED or fl & (F_MALFORMED | F_IPV6):
            continue
        if rng.random() < 0.25:
            buf[f + int(r["l3_off"]) + 8] = rng.integers(0, 2)
        if fl & F_L4 and int(r["proto"]) == 17 and rng.random() < 0.25:
            p = f + int(r["l4_off"]) + 6
            buf[p:p + 2] = 0
    return buf


def random_rewrites(n, rng, nops=32):
    from pptk_amd.records import REWRITE_DTYPE
    rw = np.zeros(n, REWRITE_DTYPE)
    rw["ops"] = rng.integers(0, nops, n)
    rw["src"] = rng.integers(0, 2 ** 32, n, dtype=np.uint64)
    rw["dst"] = rng.integers(0, 2 ** 32, n, dtype=np.uint64)
    rw["sport"] = rng.integers(0, 65536, n)
    rw["dport"] = rng.integers(0, 65536, n)
    return rw


def gen_rewrite(ref):
    """Header-rewrite fixtures over the golden sets (positions into the set's
    buffer with input and expected bytes, the rewrite entries, the status);
    for c64 also one shared rewrite entry for every frame ("c64_one")."""
    rng = np.random.default_rng(0x5E7)
    out = {}
    # (the ICMP case comes last, with the identifier op among the random
    # ops, so the earlier cases' random streams are unchanged)
    cases = [("edge", "edge", None), ("fuzz", "fuzz", None), ("cmix", "cmix", None),
             ("c64", "c64", None), ("c64_one", "c64", 1), ("icmp", "icmp", None)]
    for tag, name, count in cases:
        z = dict(np.load(os.path.join(HERE, f"{name}.npz")))
        buf_in = rewrite_inputs(z, rng)
        rw = random_rewrites(count or len(z["off"]), rng, 64 if tag == "icmp" else 32)
        if count == 1:
            rw["ops"] = 0x1F
        buf_out, status = ref.rewrite_batch(buf_in, rw, z["off"], z["len"])
        pos = np.nonzero((buf_in != z["buf"]) | (buf_out != buf_in))[0]
        out[f"{tag}_pos"] = pos.astype(np.uint64)
        out[f"{tag}_in"] = buf_in[pos]
        out[f"{tag}_out"] = buf_out[pos]
        out[f"{tag}_rw"] = rw.view(np.uint8).reshape(-1, 16)
        out[f"{tag}_status"] = status
    return out


MSS_CASES = ((1200, 0), (1460, 1), (536, 0), (0, 1))


def gen_mss(ref):
    frames = framegen.gen_mss()
    buf, off, lens = framegen.pack(frames)
    out = {"buf": buf, "off": off, "len": lens, "cases": np.array(MSS_CASES, np.uint32)}
    for k, (mss, flags) in enumerate(MSS_CASES):
        b, st = ref.mss_clamp_batch(buf, mss, flags, off=off, lens=lens)
        pos = np.nonzero(b != buf)[0]
        out[f"c{k}_pos"] = pos.astype(np.uint64)
        out[f"c{k}_out"] = b[pos]
        out[f"c{k}_status"] = st
    return out


def gen_tcpopt(ref):
    import ctypes
    hdrs = framegen.tcp_headers()
    n, w = hdrs.shape
    rng = np.random.default_rng(0x0F7)
    parse = np.zeros((n, 4), np.uint32)         # packed flags, mss, ts, tsecho
    sackts = np.zeros((n, 2), np.uint32)        # packed (sackoff, sacklen, tsoff), ok
    sack = np.zeros((n, 3), np.int64)           # offset or -1, length, 16-bit aligned
    ops = np.zeros((n, 3), np.uint32)           # op, value, ran
    after = hdrs.copy()
    L = ref.lib
    for i in range(n):
        h = np.ascontiguousarray(hdrs[i]).copy()
        p = h.ctypes.data_as(ctypes.c_void_p)
        mss, ts, te = ctypes.c_uint16(), ctypes.c_uint32(), ctypes.c_uint32()
        parse[i, 0] = L.ref_tcp_parse_options(p, ctypes.byref(mss), ctypes.byref(ts),
                                              ctypes.byref(te))
        parse[i, 1:] = (mss.value, ts.value, te.value)
        term, so, sl, to = framegen.sack_ts_walk(h)
        if term:
            sackts[i] = (L.ref_tcp_find_sack_ts(p), 1)
        sl_, al = ctypes.c_uint32(), ctypes.c_int()
        sack[i] = (L.ref_tcp_find_sack(p, ctypes.byref(sl_), ctypes.byref(al)), sl_.value,
                   al.value)
        op, val = i % 9, int(rng.integers(0, 2 ** 32))
        if op in (0, 8):
            val &= 0xFFFF
        ok = True
        if op in (2, 3, 4):
            ok = term and not (op == 2 and so % 2 == 1 and sl >= 10)
        ops[i] = (op, val, ok)
        if ok:
            L.ref_tcp_opt_op(p, op, val)
        after[i] = h
    return {"hdrs": hdrs, "parse": parse, "sackts": sackts, "sack": sack, "ops": ops,
            "after": after}


def gen_frag(ref):
    """Fragment side records (struct pptk_rx_frag) from the reference's own
    getters and IPv6 walk (oracle/refgen.c ref_frag_batch): a dedicated
    fragment set (framegen.gen_frag, with its 64-byte records too) and the
    side records of the edge / fuzz / cmix sets."""
    opts = make_opts(KEY, BITS4, BITS6, HASH_SIZE)
    buf, off, lens = framegen.gen_frag()
    out = dict(buf=buf, off=off, len=lens,
               recs=ref.rx_batch(buf, off, lens, opts=opts, with_bucket=True)
               .view(np.uint8).reshape(-1, 64),
               frag=ref.frag_batch(buf, off, lens).view(np.uint8).reshape(-1, 16),
               key=np.frombuffer(KEY, dtype=np.uint8),
               iphash=np.array([BITS4, BITS6, HASH_SIZE], dtype=np.uint32))
    for name in ("edge", "fuzz", "cmix"):
        z = dict(np.load(os.path.join(HERE, f"{name}.npz")))
        out[f"{name}_frag"] = ref.frag_batch(z["buf"], z["off"], z["len"]).view(np.uint8) \
            .reshape(-1, 16)
    return out


def main():
    build()
    ref = Reference()
    opts = make_opts(KEY, BITS4, BITS6, HASH_SIZE)
    want = set(sys.argv[1:]) or set(SETS) | {"permit", "tx", "rewrite", "mss", "tcpopt", "frag"}
    if "mss" in want:
        path = os.path.join(HERE, "mss.npz")
        np.savez_compressed(path, **gen_mss(ref))
        print(f"mss -> {os.path.getsize(path)} B")
    if "tcpopt" in want:
        path = os.path.join(HERE, "tcpopt.npz")
        np.savez_compressed(path, **gen_tcpopt(ref))
        print(f"tcpopt -> {os.path.getsize(path)} B")
    if "rewrite" in want:
        path = os.path.join(HERE, "rewrite.npz")
        np.savez_compressed(path, **gen_rewrite(ref))
        print(f"rewrite -> {os.path.getsize(path)} B")
    if "tx" in want:
        path = os.path.join(HERE, "tx.npz")
        np.savez_compressed(path, **gen_tx(ref))
        print(f"tx -> {os.path.getsize(path)} B")
    if "frag" in want:
        path = os.path.join(HERE, "frag.npz")
        np.savez_compressed(path, **gen_frag(ref))
        print(f"frag -> {os.path.getsize(path)} B")
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
