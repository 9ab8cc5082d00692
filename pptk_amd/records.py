"""Record format of the rx transform: numpy view of ``struct pptk_rx_rec``
(include/pptk_rx.h).  64 bytes per frame, little-endian."""
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


def diff_records(got, want, limit=5):
    """Return a human-readable description of the first mismatching records
    (empty string when identical byte for byte)."""
    g = np.ascontiguousarray(got).view(np.uint8).reshape(-1, 64)
    w = np.ascontiguousarray(want).view(np.uint8).reshape(-1, 64)
    if g.shape != w.shape:
        return f"shape mismatch {g.shape} vs {w.shape}"
    bad = np.nonzero((g != w).any(axis=1))[0]
    if bad.size == 0:
        return ""
    lines = [f"{bad.size} of {g.shape[0]} records differ"]
    gr, wr = g.view(REC_DTYPE).reshape(-1), w.view(REC_DTYPE).reshape(-1)
    for i in bad[:limit]:
        fields = [n for n in REC_DTYPE.names
                  if not np.array_equal(gr[i][n], wr[i][n])]
        lines.append(f"  rec {i}: fields {fields}: got "
                     + ", ".join(f"{n}={gr[i][n]}" for n in fields)
                     + " want " + ", ".join(f"{n}={wr[i][n]}" for n in fields))
    return "\n".join(lines)
