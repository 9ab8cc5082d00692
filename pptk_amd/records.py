"""Record formats of the rx transform: numpy views of ``struct pptk_rx_rec``
(64 bytes per frame) and ``struct pptk_rx_rec32`` (32 bytes), little-endian
(include/pptk_rx.h)."""
import numpy as np

REC_DTYPE = np.dtype([
    ("flow_hash", "<u8"),
    ("src", "u1", 16),
    ("dst", "u1", 16),
    ("sport", "<u2"),
    ("dport", "<u2"),
    ("ip_cksum", "<u2"),
    ("l4_cksum", "<u2"),
    ("l4_off", "<u2"),
    ("l4_len", "<u2"),
    ("l3_off", "u1"),
    ("proto", "u1"),
    ("flags", "<u2"),
    ("src_bucket", "<u4"),
    ("ethertype", "<u2"),
    ("ip_version", "u1"),
    ("reserved", "u1"),
])
assert REC_DTYPE.itemsize == 64

# struct pptk_rewrite (pptk_tx_rewrite_device): ops, new src/dst (host
# order), new ports (host order)
REWRITE_DTYPE = np.dtype([("ops", "<u4"), ("src", "<u4"), ("dst", "<u4"),
                          ("sport", "<u2"), ("dport", "<u2")])
assert REWRITE_DTYPE.itemsize == 16
RW_DECR_TTL, RW_SRC, RW_DST, RW_SPORT, RW_DPORT = 0x1, 0x2, 0x4, 0x8, 0x10
RW_ST_IP, RW_ST_L4, RW_ST_TTL_ZERO, RW_ST_EXPIRED, RW_ST_ICMP = 0x1, 0x2, 0x4, 0x8, 0x10
RW_ICMP_ID = 0x20
MSS_SYN_ONLY = 0x1
MSS_ST_TCP, MSS_ST_FOUND, MSS_ST_CLAMPED, MSS_ST_BADOPT = 0x1, 0x2, 0x4, 0x8

REC32_DTYPE = np.dtype([
    ("flow_hash", "<u8"),
    ("src4", "u1", 4),
    ("dst4", "u1", 4),
    ("sport", "<u2"),
    ("dport", "<u2"),
    ("flags", "<u2"),
    ("proto", "u1"),
    ("l3_off", "u1"),
    ("l4_off", "<u2"),
    ("l4_len", "<u2"),
    ("src_bucket", "<u4"),
])
assert REC32_DTYPE.itemsize == 32

# struct pptk_rx_frag: the fragment side record (pptk_rx_dev_batch.d_frag)
FRAG_DTYPE = np.dtype([
    ("ident", "<u4"),
    ("frag_off", "<u2"),
    ("data_len", "<u2"),
    ("frag_hdr_off", "<u2"),
    ("proto_hdr_off_from_frag", "<u2"),
    ("next_hdr", "u1"),
    ("flags", "u1"),
    ("reserved", "<u2"),
])
assert FRAG_DTYPE.itemsize == 16
FRAG_IS, FRAG_MF, FRAG_DF, FRAG_V6 = 0x01, 0x02, 0x04, 0x08

F_PARSED = 0x0001
F_IP_OK = 0x0002
F_L4_OK = 0x0004
F_L4 = 0x0008
F_IPV6 = 0x0010
F_VLAN = 0x0020
F_FRAGMENT = 0x0040
F_UDP_ZERO = 0x0080
F_MALFORMED = 0x0100
F_V6_EXT = 0x0200


def as_records(raw):
    """View a uint8 buffer (n*64 bytes) as records."""
    raw = np.ascontiguousarray(raw)
    return raw.view(np.uint8).reshape(-1).view(REC_DTYPE)


def to_rec32(recs):
    """The compact record the kernel writes for each full record: the same
    values, IPv6 addresses left out (src4/dst4 = 0)."""
    r = as_records(recs)
    out = np.zeros(len(r), dtype=REC32_DTYPE)
    v4 = (r["flags"] & F_IPV6) == 0
    for f in ("flow_hash", "sport", "dport", "flags", "proto", "l3_off", "l4_off", "l4_len",
              "src_bucket"):
        out[f] = r[f]
    out["src4"] = np.where(v4[:, None], r["src"][:, :4], 0)
    out["dst4"] = np.where(v4[:, None], r["dst"][:, :4], 0)
    return out


def diff_records(got, want, limit=5, dtype=REC_DTYPE):
    """Return a human-readable description of the first mismatching records
    (empty string when identical byte for byte)."""
    rb = dtype.itemsize
    g = np.ascontiguousarray(got).view(np.uint8).reshape(-1, rb)
    w = np.ascontiguousarray(want).view(np.uint8).reshape(-1, rb)
    if g.shape != w.shape:
        return f"shape mismatch {g.shape} vs {w.shape}"
    bad = np.nonzero((g != w).any(axis=1))[0]
    if bad.size == 0:
        return ""
    lines = [f"{bad.size} of {g.shape[0]} records differ"]
    gr, wr = g.view(dtype).reshape(-1), w.view(dtype).reshape(-1)
    for i in bad[:limit]:
        fields = [n for n in dtype.names
                  if not np.array_equal(gr[i][n], wr[i][n])]
        lines.append(f"  rec {i}: fields {fields}: got "
                     + ", ".join(f"{n}={gr[i][n]}" for n in fields)
                     + " want " + ", ".join(f"{n}={wr[i][n]}" for n in fields))
    return "\n".join(lines)
