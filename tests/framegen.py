"""Deterministic synthetic Ethernet frames for the rx-transform tests.

Recipes follow SURVEY.md section 8(d) (C64 / C1500 / CMIX) and the
reference's frame recipe ldp/ldpsend.c:141-168 (Eth + IPv4 DF TTL 64 +
UDP, checksums filled).  Checksums are filled by a small independent
Python one's-complement sum, not by the oracle.

Every generator returns ``(buf, off, lens)``: frames packed back to back in
one uint8 buffer (so frame starts are generally NOT aligned), u64 offsets
and u16 lengths.
"""
import struct

import numpy as np

ETH_IP, ETH_IP6, ETH_VLAN = 0x0800, 0x86DD, 0x8100


# ---------------------------------------------------------------- checksums
def ones_sum(data, start=0):
    """Sum of big-endian 16-bit words (RFC 1071), odd tail padded."""
    b = bytes(data)
    if len(b) & 1:
        b += b"\0"
    a = np.frombuffer(b, dtype=">u2").astype(np.uint64)
    s = int(a.sum()) + start
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def csum(data, start=0):
    return (~ones_sum(data, start)) & 0xFFFF


def eth(etype, vlan=None, dst=b"\x02\0\0\0\0\x01", src=b"\x02\0\0\0\0\x02"):
    h = dst + src
    if vlan is not None:
        h += struct.pack(">HH", ETH_VLAN, vlan & 0x0FFF)
    return h + struct.pack(">H", etype)


def ipv4_hdr(src, dst, proto, payload_len, opts=b"", df=True, mf=False,
             frag_off=0, ttl=64, ident=0, fix=True):
    assert len(opts) % 4 == 0
    ihl = 5 + len(opts) // 4
    flags = (0x4000 if df else 0) | (0x2000 if mf else 0) | (frag_off & 0x1FFF)
    h = bytearray(struct.pack(">BBHHHBBH4s4s", 0x40 | ihl, 0, ihl * 4 + payload_len,
                              ident, flags, ttl, proto, 0, src, dst) + opts)
    if fix:
        struct.pack_into(">H", h, 10, csum(h))
    return bytes(h)


def ipv6_hdr(src, dst, nexthdr, payload_len, hlim=64):
    return struct.pack(">IHBB16s16s", 0x60000000, payload_len, nexthdr, hlim, src, dst)


def tcp_hdr(sport, dport, seq=0, ack=0, flags=0x18, win=8192, opts=b""):
    doff = 5 + len(opts) // 4
    return struct.pack(">HHIIBBHHH", sport, dport, seq, ack, doff << 4, flags,
                       win, 0, 0) + opts


def udp_hdr(sport, dport, length):
    return struct.pack(">HHHH", sport, dport, length, 0)


def pseudo4(src, dst, proto, l4len):
    return src + dst + struct.pack(">BBH", 0, proto, l4len)


def pseudo6(src, dst, proto, l4len):
    return src + dst + struct.pack(">II", l4len, proto)


def fill_l4(seg, proto, pseudo, udp_zero=False):
    seg = bytearray(seg)
    off = 16 if proto == 6 else 6
    seg[off:off + 2] = b"\0\0"
    if proto == 17 and udp_zero:
        return bytes(seg)
    c = csum(bytes(pseudo) + bytes(seg))
    if proto == 17 and c == 0:
        c = 0xFFFF
    struct.pack_into(">H", seg, off, c)
    return bytes(seg)


# ------------------------------------------------------------ frame builders
def frame_v4(rng, proto, total, vlan=None, ihl_words=5, corrupt=None,
             src=None, dst=None, udp_zero=False, mf=False, frag_off=0):
    """IPv4 frame of exactly `total` bytes (>= minimum)."""
    l2 = eth(ETH_IP, vlan)
    opts = bytes(rng.integers(0, 256, (ihl_words - 5) * 4, dtype=np.uint8))
    l4min = 20 if proto == 6 else 8
    l4len = total - len(l2) - 20 - len(opts)
    assert l4len >= l4min, (total, l4len)
    src = src if src is not None else bytes([10]) + bytes(rng.integers(0, 256, 3, dtype=np.uint8))
    dst = dst if dst is not None else bytes([192, 168]) + bytes(rng.integers(0, 256, 2, dtype=np.uint8))
    sp, dp = (int(x) for x in rng.integers(0, 65536, 2))
    payload = bytes(rng.integers(0, 256, l4len - l4min, dtype=np.uint8))
    if proto == 6:
        seg = tcp_hdr(sp, dp, int(rng.integers(0, 2**32)), 0) + payload
    else:
        seg = udp_hdr(sp, dp, l4len) + payload
    seg = fill_l4(seg, proto, pseudo4(src, dst, proto, l4len), udp_zero)
    ip = ipv4_hdr(src, dst, proto, l4len, opts, mf=mf, frag_off=frag_off,
                  ident=int(rng.integers(0, 65536)))
    f = bytearray(l2 + ip + seg)
    corrupt_frame(f, rng, corrupt, len(l2), len(ip))
    return bytes(f)


def frame_v6(rng, proto, total, vlan=None, ext=None, corrupt=None, src=None):
    """IPv6 frame; ext = list of (type, bytes) extension headers."""
    l2 = eth(ETH_IP6, vlan)
    ext = ext or []
    exth = b""
    types = [t for t, _ in ext] + [proto]
    for i, (t, body) in enumerate(ext):
        exth += bytes([types[i + 1]]) + body[1:]
    l4min = 20 if proto == 6 else 8
    l4len = total - len(l2) - 40 - len(exth)
    assert l4len >= l4min
    if src is None:
        src = bytes([0x20, 0x01, 0x0d, 0xb8]) + bytes(rng.integers(0, 256, 12, dtype=np.uint8))
    dst = bytes([0xfd]) + bytes(rng.integers(0, 256, 15, dtype=np.uint8))
    sp, dp = (int(x) for x in rng.integers(0, 65536, 2))
    payload = bytes(rng.integers(0, 256, l4len - l4min, dtype=np.uint8))
    seg = (tcp_hdr(sp, dp) if proto == 6 else udp_hdr(sp, dp, l4len)) + payload
    seg = fill_l4(seg, proto, pseudo6(src, dst, proto, l4len))
    ip = ipv6_hdr(src, dst, types[0], len(exth) + l4len)
    f = bytearray(l2 + ip + exth + seg)
    corrupt_frame(f, rng, corrupt, len(l2), 40 + len(exth))
    return bytes(f)


def hbh(n8=1):
    """Hop-by-hop / destination-options header of n8*8 bytes (PadN)."""
    body = bytearray(8 * n8)
    body[1] = n8 - 1
    body[2] = 1          # PadN
    body[3] = 8 * n8 - 4
    return bytes(body)


def corrupt_frame(f, rng, how, l3, l3len):
    if how is None:
        return
    if how == "ip":        # flip a bit of the IPv4 identification field
        f[l3 + 4] ^= 0x01
    elif how == "l4":      # flip a payload/L4 byte
        pos = int(rng.integers(l3 + l3len, len(f)))
        f[pos] ^= 0xFF if f[pos] != 0xFF else 0x01


def pack(frames, align=1):
    """Pack frames back to back (each start rounded up to `align`)."""
    offs, lens, pos = [], [], 0
    for fr in frames:
        pos = (pos + align - 1) // align * align
        offs.append(pos)
        lens.append(len(fr))
        pos += len(fr)
    buf = np.zeros(pos + 64, dtype=np.uint8)
    for o, fr in zip(offs, frames):
        buf[o:o + len(fr)] = np.frombuffer(fr, dtype=np.uint8)
    return buf, np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint16)


def _corrupt_choice(rng, rate=0.01):
    u = rng.random()
    return "ip" if u < rate / 2 else ("l4" if u < rate else None)


# ----------------------------------------------------------------- configs
def gen_c64(n, seed=0x5EED + 1):
    rng = np.random.default_rng(seed)
    return pack([frame_v4(rng, 17, 64, corrupt=_corrupt_choice(rng)) for _ in range(n)])


def gen_c1500(n, seed=0x5EED + 2):
    rng = np.random.default_rng(seed)
    return pack([frame_v4(rng, 6, 1500, corrupt=_corrupt_choice(rng)) for _ in range(n)])


def gen_cmix(n, seed=0x5EED + 3):
    """64..1500 B, 70 % IPv4 / 30 % IPv6, 50/50 TCP/UDP, 25 % VLAN, 5 % IPv4
    with IHL > 5, 2 % IPv6 with one hop-by-hop header."""
    rng = np.random.default_rng(seed)
    frames = []
    for _ in range(n):
        proto = 6 if rng.random() < 0.5 else 17
        vlan = int(rng.integers(1, 4095)) if rng.random() < 0.25 else None
        size = int(rng.integers(64, 1501))
        corrupt = _corrupt_choice(rng)
        if rng.random() < 0.7:
            ihl = int(rng.integers(6, 16)) if rng.random() < 0.05 else 5
            minsz = 14 + (4 if vlan is not None else 0) + ihl * 4 + (20 if proto == 6 else 8)
            frames.append(frame_v4(rng, proto, max(size, minsz), vlan, ihl, corrupt))
        else:
            ext = [(0, hbh(1))] if rng.random() < 0.02 else None
            minsz = 14 + (4 if vlan is not None else 0) + 40 + (8 if ext else 0) + (20 if proto == 6 else 8)
            frames.append(frame_v6(rng, proto, max(size, minsz), vlan, ext,
                                   "l4" if corrupt else None))
    return pack(frames)


# ------------------------------------------------------- reference KAT frames
# Raw IP packets of iphdr/ipcksumtest.c:14-18 and iphdr/iphdrtest.c:5-8
# (fixture data, each must verify to 0 / walk as the reference tests assert).
KAT_IP = {
    "iptcp6hdr": bytes.fromhex(
        "6000000000170640" + "00" * 15 + "01" + "00" * 15 + "01"
        + "00140050000000000000000050022000ba0a0000666f6f"),
    "ipudp6hdr": bytes.fromhex(
        "60000000000b1140" + "00" * 15 + "01" + "00" * 15 + "01"
        + "00350035000b29fd666f6f"),
    "iphdr": bytes.fromhex("450000140001000040007ce77f0000017f000001"),
    "iptcphdr": bytes.fromhex(
        "4500002b0001000040067cca7f0000017f000001"
        "00140050000000000000000050022000bc090000666f6f"),
    "ipudphdr": bytes.fromhex(
        "4500001f0001000040117ccb7f0000017f000001"
        "00350035000b2bfc666f6f"),
    "tcp6frag": bytes.fromhex(
        "60000000001f2c40" + "00" * 15 + "01" + "00" * 15 + "01"
        + "0600000000000000" + "00140050000000000000000050022000ba0a0000666f6f"),
    "tcp6hop": bytes.fromhex(
        "60000000001f0040" + "00" * 15 + "01" + "00" * 15 + "01"
        + "0600010400000000" + "00140050000000000000000050022000ba0a0000666f6f"),
    "tcp6subsequentfrag": bytes.fromhex(
        "60000000001f2c40" + "00" * 15 + "01" + "00" * 15 + "01"
        + "0600000800000000" + "00140050000000000000000050022000ba0a0000666f6f"),
}


def kat_frames():
    out = []
    for name, ip in KAT_IP.items():
        et = ETH_IP6 if ip[0] >> 4 == 6 else ETH_IP
        out.append(eth(et) + ip)
        out.append(eth(et, vlan=7) + ip)
    return out


# ------------------------------------------------------------- edge frames
def edge_frames(seed=0xED6E):
    rng = np.random.default_rng(seed)
    F = []
    base4 = frame_v4(rng, 6, 100)
    base6 = frame_v6(rng, 17, 120)
    F += kat_frames()
    # runts and truncations of valid frames at every length up to 80
    for cut in list(range(0, 80)) + [99]:
        F.append(base4[:cut])
    for cut in (0, 13, 14, 17, 18, 40, 53, 54, 55, 61, 62, 119):
        F.append(base6[:cut])
        F.append(eth(ETH_IP6, 5)[:min(cut, 18)] + base6[14:cut])
    F.append(eth(ETH_VLAN)[:14] + b"\x00")                       # VLAN runt
    F.append(b"\x02" * 12 + b"\x81\x00\x00\x05")                 # VLAN, len 16
    # IHL / total-length / version corner cases
    for ihl_nib in range(0, 16):
        f = bytearray(frame_v4(rng, 17, 90))
        f[14] = 0x40 | ihl_nib
        F.append(bytes(f))
    for tl in (0, 19, 20, 27, 28, 29, 39, 40, 41, 75, 76, 77, 1000):
        f = bytearray(frame_v4(rng, 17, 90))
        struct.pack_into(">H", f, 16, tl)
        F.append(bytes(f))
    for ver in (0, 5, 6, 15):
        f = bytearray(frame_v4(rng, 6, 90))
        f[14] = (ver << 4) | 5
        F.append(bytes(f))
        g = bytearray(frame_v6(rng, 6, 100))
        g[14] = (ver << 4) | (g[14] & 0xF)
        F.append(bytes(g))
    # Ethernet padding beyond ip_total_len (excluded from the L4 sum)
    for pad in (1, 2, 3, 6, 17):
        F.append(frame_v4(rng, 17, 60) + bytes(rng.integers(0, 256, pad, dtype=np.uint8)))
    # odd and tiny L4 lengths
    for total in range(42, 80):
        F.append(frame_v4(rng, 17, total))
    for total in range(54, 90):
        F.append(frame_v4(rng, 6, total))
    for total in range(62, 100):
        F.append(frame_v6(rng, 17, total))
        F.append(frame_v6(rng, 6, total + 12))
    # runt L4 (UDP < 8, TCP < 20) via total length
    for proto, l4 in ((17, 0), (17, 4), (17, 7), (6, 0), (6, 8), (6, 19)):
        ip = ipv4_hdr(b"\x0a\0\0\x01", b"\x0a\0\0\x02", proto, l4)
        F.append(eth(ETH_IP) + ip + bytes(rng.integers(0, 256, l4, dtype=np.uint8)))
    # UDP transmitted checksum zero (v4) and one that sums to 0xffff
    F.append(frame_v4(rng, 17, 80, udp_zero=True))
    F.append(frame_v4(rng, 17, 64, udp_zero=True, vlan=100))
    # fragments: MF, offset, both, DF only
    F.append(frame_v4(rng, 6, 200, mf=True))
    F.append(frame_v4(rng, 17, 200, frag_off=185))
    F.append(frame_v4(rng, 17, 200, mf=True, frag_off=3))
    # IHL up to 15 with options
    for ihl in range(5, 16):
        F.append(frame_v4(rng, 6, 200, ihl_words=ihl))
        F.append(frame_v4(rng, 17, 120, vlan=9, ihl_words=ihl))
    # IPv6 extension chains
    for chain in ([(0, hbh(1))], [(0, hbh(2))], [(60, hbh(1))], [(43, hbh(1))],
                  [(0, hbh(1)), (60, hbh(3))], [(60, hbh(1)), (43, hbh(2)), (60, hbh(1))],
                  [(51, bytes([0, 1]) + bytes(6))], [(51, bytes([0, 4]) + bytes(22))],
                  [(44, bytes(8))], [(0, hbh(1)), (44, bytes(8))],
                  [(0, hbh(3)), (44, bytes(8))],           # extlen-from-next-header quirk
                  [(44, bytes([0, 0, 0, 8]) + bytes(4))],   # subsequent fragment
                  [(44, bytes([0, 0, 0, 1]) + bytes(4))],   # first fragment, M=1
                  [(60, hbh(1))] * 6,
                  [(60, hbh(1))] * 20):
        for proto in (6, 17):
            try:
                F.append(frame_v6(rng, proto, 64 + 8 * sum(len(b) // 8 for _, b in chain) + 80, ext=chain))
            except AssertionError:
                pass
    # IPv6 chain overrunning the payload length -> NULL in the reference
    g = bytearray(frame_v6(rng, 6, 120, ext=[(0, hbh(1))]))
    g[14 + 40 + 1] = 30
    F.append(bytes(g))
    g = bytearray(frame_v6(rng, 6, 120, ext=[(60, hbh(1))]))
    struct.pack_into(">H", g, 18, 7)                             # plen 7 < 8
    F.append(bytes(g[:14 + 47]))
    # non-IP ethertypes, QinQ
    F.append(eth(0x0806) + bytes(28))
    F.append(eth(0x88A8) + bytes(46))
    F.append(eth(0x0800, vlan=1)[:12] + b"\x81\x00\x00\x01\x86\xdd" + bytes(60))
    # jumbo frames
    F.append(frame_v4(rng, 6, 9014))
    F.append(frame_v4(rng, 17, 9018, vlan=3))
    F.append(frame_v6(rng, 6, 9000))
    F.append(frame_v6(rng, 17, 65535))
    F.append(frame_v4(rng, 6, 65535))
    return F


def gen_edge(seed=0xED6E):
    return pack(edge_frames(seed))


def gen_fuzz(n, seed=0xF022):
    """Valid frames of every kind with random header mutations/truncations."""
    rng = np.random.default_rng(seed)
    frames = []
    for i in range(n):
        kind = int(rng.integers(0, 4))
        if kind == 0:
            ihl = int(rng.integers(5, 16)) if rng.random() < 0.3 else 5
            f = frame_v4(rng, 6 if rng.random() < 0.5 else 17,
                         max(int(rng.integers(64, 400)), 18 + 4 * ihl + 20),
                         vlan=5 if rng.random() < 0.3 else None, ihl_words=ihl)
        elif kind == 1:
            ext = [(int(rng.choice([0, 43, 44, 51, 60])), hbh(1))] if rng.random() < 0.5 else None
            f = frame_v6(rng, 6 if rng.random() < 0.5 else 17, int(rng.integers(100, 400)),
                         vlan=5 if rng.random() < 0.3 else None, ext=ext)
        elif kind == 2:
            f = frame_v4(rng, 17, int(rng.integers(42, 200)))
        else:
            f = frame_v6(rng, 17, int(rng.integers(80, 200)),
                         ext=[(int(rng.choice([0, 44, 60])), hbh(int(rng.integers(1, 3))))])
        f = bytearray(f)
        for _ in range(int(rng.integers(1, 4))):
            pos = int(rng.integers(0, min(len(f), 96)))
            f[pos] = int(rng.integers(0, 256))
        if rng.random() < 0.2:
            f = f[:int(rng.integers(0, len(f) + 1))]
        frames.append(bytes(f))
    return pack(frames)


def frag6(off_bytes=0, m=0, ident=0, reserved=0):
    """IPv6 fragment header body (next header filled in by frame_v6):
    reserved byte, offset (bytes, multiple of 8) | M, 32-bit Identification."""
    return bytes([0, reserved & 0xFF]) + struct.pack(">HI", (off_bytes & 0xFFF8) | (m & 1),
                                                      ident & 0xFFFFFFFF)


def gen_frag(n=1500, seed=0xF7A6):
    """Fragment workload for the fragment side record (pptk_rx_frag): IPv4
    fragments (MF / offset / DF / ident, IHL > 5, VLAN) and non-fragments,
    IPv6 fragment headers first / subsequent / atomic, behind hop-by-hop,
    destination and routing headers (some long enough to put the fragment
    header past the first 128 bytes), two fragment headers in one chain, a
    non-zero reserved byte (the reference's extlen-from-next-header quirk),
    and random header mutations."""
    rng = np.random.default_rng(seed)
    frames = []
    for i in range(n):
        vlan = int(rng.integers(1, 4095)) if rng.random() < 0.25 else None
        proto = int(rng.choice([6, 17]))
        kind = int(rng.integers(0, 3))
        if kind == 0:
            ihl = int(rng.integers(6, 16)) if rng.random() < 0.1 else 5
            mf = bool(rng.random() < 0.5)
            fo = int(rng.integers(0, 0x2000)) if rng.random() < 0.6 else 0
            minsz = 14 + (4 if vlan else 0) + 4 * ihl + (20 if proto == 6 else 8)
            f = bytearray(frame_v4(rng, proto, max(int(rng.integers(64, 1500)), minsz), vlan,
                                   ihl, mf=mf, frag_off=fo))
            if rng.random() < 0.3:                      # DF cleared on some
                f[14 + (4 if vlan else 0) + 6] &= 0xBF
        else:
            ext = []
            for _ in range(int(rng.integers(0, 3))):
                t = int(rng.choice([0, 60, 43]))
                ext.append((t, hbh(int(rng.integers(1, 18)))))
            m = int(rng.integers(0, 2))
            off = int(rng.integers(1, 8000)) * 8 if rng.random() < 0.5 else 0
            res = int(rng.integers(1, 3)) if rng.random() < 0.05 else 0
            ext.append((44, frag6(off, m, int(rng.integers(0, 2 ** 32)), res)))
            if rng.random() < 0.1:                      # a second fragment header
                ext.append((44, frag6(0, int(rng.integers(0, 2)), int(rng.integers(0, 2 ** 32)))))
            if rng.random() < 0.1:
                ext.append((60, hbh(1)))
            hdrs = sum(len(b) for _, b in ext)
            minsz = 14 + (4 if vlan else 0) + 40 + hdrs + (20 if proto == 6 else 8)
            f = bytearray(frame_v6(rng, proto, max(int(rng.integers(80, 1500)), minsz), vlan, ext))
        if rng.random() < 0.1:
            for _ in range(int(rng.integers(1, 3))):
                pos = int(rng.integers(0, min(len(f), 200)))
                f[pos] = int(rng.integers(0, 256))
        frames.append(bytes(f))
    return pack(frames)


def gen_permit(n=3000, seed=0x9E7):
    """Rate-limiter workload: frames from few source prefixes (20 IPv4 /24s,
    8 IPv6 /48s) so that token buckets see long runs, in random order, with a
    few non-IP and malformed frames mixed in."""
    rng = np.random.default_rng(seed)
    v4_nets = [bytes([10, int(a), int(b)]) for a, b in rng.integers(0, 256, (20, 2))]
    v6_nets = [bytes([0x20, 0x01, 0x0d, 0xb8]) + bytes(rng.integers(0, 256, 2, dtype=np.uint8))
               for _ in range(8)]
    weights = rng.random(20) ** 3
    weights /= weights.sum()
    frames = []
    for _ in range(n):
        u = rng.random()
        proto = 6 if rng.random() < 0.5 else 17
        if u < 0.65:
            net = v4_nets[int(rng.choice(20, p=weights))]
            src = net + bytes([int(rng.integers(0, 256))])
            frames.append(frame_v4(rng, proto, int(rng.integers(64, 200)), src=src))
        elif u < 0.95:
            net = v6_nets[int(rng.integers(0, 8))]
            src = net + bytes(rng.integers(0, 256, 10, dtype=np.uint8))
            frames.append(frame_v6(rng, proto, int(rng.integers(90, 200)), src=src))
        elif u < 0.98:
            frames.append(eth(0x0806) + bytes(46))     # ARP: not IP
        else:
            frames.append(frame_v4(rng, 17, 64)[:30])  # runt: malformed
    return pack(frames)


# ------------------------------------------------------------ TCP options
def tcp_options(rng, syn=True):
    """A random TCP option list (bytes, padded to a multiple of 4, <= 40):
    well-formed lists most of the time, plus the malformed shapes the
    reference's walks distinguish (length bytes 0/1, lengths past the end,
    a length byte past the options, unknown kinds, EOL before the end)."""
    out = bytearray()
    for _ in range(int(rng.integers(0, 7))):
        c = int(rng.integers(0, 100))
        if c < 20:
            out += b"\x01"                                   # NOP (shifts parity)
        elif c < 45:
            out += struct.pack(">BBH", 2, 4, int(rng.choice([536, 1200, 1380, 1400, 1440,
                                                              1460, 8960, 65535,
                                                              int(rng.integers(0, 65536))])))
        elif c < 55:
            out += bytes([3, 3, int(rng.integers(0, 15))])     # window scale
        elif c < 62:
            out += b"\x04\x02"                               # SACK permitted
        elif c < 72:
            out += struct.pack(">BBII", 8, 10, *(int(x) for x in rng.integers(0, 2**32, 2)))
        elif c < 80:
            k = int(rng.integers(1, 4))                      # SACK blocks
            out += bytes([5, 2 + 8 * k]) + bytes(rng.integers(0, 256, 8 * k, dtype=np.uint8))
        elif c < 85:
            out += bytes([int(rng.choice([2, 3, 8, 5, 30])), int(rng.integers(0, 2))])  # len 0/1
        elif c < 90:
            out += bytes([int(rng.choice([2, 3, 4, 8, 30])), int(rng.integers(2, 60))])  # odd len
        elif c < 95:
            out += bytes([int(rng.integers(9, 256)), 2 + int(rng.integers(0, 5))])  # unknown
        else:
            out += b"\x00"                                   # EOL
    out = out[:40]
    while len(out) % 4:
        out += bytes([int(rng.choice([0, 1]))])
    return bytes(out)


def frame_tcp_opts(rng, v6=False, vlan=None, ihl_words=5, syn=True, opts=None, payload=None,
                   doff_override=None):
    """A TCP frame (valid checksums) carrying `opts` (random if None)."""
    opts = tcp_options(rng) if opts is None else opts
    payload = bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8)) \
        if payload is None else payload
    sp, dp = (int(x) for x in rng.integers(0, 65536, 2))
    flags = 0x02 if syn else 0x10
    seg = bytearray(tcp_hdr(sp, dp, int(rng.integers(0, 2**32)), 0, flags=flags, opts=opts)
                    + payload)
    if doff_override is not None:
        seg[12] = (doff_override << 4) | (seg[12] & 0x0f)
    l4len = len(seg)
    if v6:
        src = bytes([0x20, 0x01]) + bytes(rng.integers(0, 256, 14, dtype=np.uint8))
        dst = bytes([0xfd]) + bytes(rng.integers(0, 256, 15, dtype=np.uint8))
        seg = fill_l4(seg, 6, pseudo6(src, dst, 6, l4len))
        return eth(ETH_IP6, vlan) + ipv6_hdr(src, dst, 6, l4len) + seg
    src = bytes([10]) + bytes(rng.integers(0, 256, 3, dtype=np.uint8))
    dst = bytes([192, 168]) + bytes(rng.integers(0, 256, 2, dtype=np.uint8))
    seg = fill_l4(seg, 6, pseudo4(src, dst, 6, l4len))
    ipo = bytes(rng.integers(0, 256, (ihl_words - 5) * 4, dtype=np.uint8))
    return eth(ETH_IP, vlan) + ipv4_hdr(src, dst, 6, l4len, ipo) + seg


def gen_mss(n=4000, seed=0x355):
    """MSS-clamping fixture frames: TCP over IPv4 (IHL 5-15) / IPv6, with and
    without a VLAN tag, SYN and non-SYN, random option lists incl. malformed
    ones, data offsets past the segment, plus UDP / non-IP frames that must
    stay untouched."""
    rng = np.random.default_rng(seed)
    frames = []
    for i in range(n):
        c = int(rng.integers(0, 100))
        vlan = int(rng.integers(1, 4095)) if rng.random() < 0.25 else None
        if c < 85:
            v6 = rng.random() < 0.3
            ihl = 5 if v6 or rng.random() < 0.7 else int(rng.integers(6, 16))
            frames.append(frame_tcp_opts(rng, v6=v6, vlan=vlan, ihl_words=ihl,
                                         syn=rng.random() < 0.7))
        elif c < 92:
            # data offset past the segment end (options overrun): BADOPT
            frames.append(frame_tcp_opts(rng, vlan=vlan, opts=b"\x02\x04\x05\xb4",
                                         payload=b"", doff_override=int(rng.integers(7, 16))))
        elif c < 96:
            frames.append(frame_v4(rng, 17, int(rng.integers(60, 200)), vlan=vlan))
        else:
            frames.append(bytes(rng.integers(0, 256, int(rng.integers(14, 120)), dtype=np.uint8)))
    return frames


def sack_ts_walk(t):
    """The reference's tcp_find_sack_ts_headers (iphdr/iphdr.c:134-199) on
    TCP header bytes t, simulated: (terminates, sackoff, sacklen, tsoff).
    A SACK or timestamp option whose length byte is 0 makes the reference
    loop forever (terminates False) -- test inputs for the reference must
    avoid those."""
    end = (t[12] >> 4) * 4
    off, sackoff, sacklen, tsoff = 20, 0, 0, 0
    while off < end:
        k = t[off]
        if k == 0:
            break
        if k == 1:
            off += 1
            continue
        ln = end - off
        if off + 1 < end and t[off + 1] < ln:
            ln = t[off + 1]
        if k == 5:
            sackoff, sacklen = off, ln
        elif k == 8:
            if ln == 10:
                tsoff = off
        elif ln < 2:
            break
        if ln == 0:
            return False, sackoff, sacklen, tsoff
        off += ln
    return True, sackoff, sacklen, tsoff


def tcp_headers(n=3000, seed=0x7C9, width=80):
    """n TCP headers (width bytes each: the header with its options, then
    payload bytes) for the kept option API: random option lists, odd
    offsets, data offsets 0-15."""
    rng = np.random.default_rng(seed)
    out = np.zeros((n, width), np.uint8)
    for i in range(n):
        opts = tcp_options(rng)
        h = bytearray(tcp_hdr(*(int(x) for x in rng.integers(0, 65536, 2)),
                              int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)),
                              flags=int(rng.integers(0, 256)), win=int(rng.integers(0, 65536)),
                              opts=opts))
        h[16:18] = bytes(rng.integers(0, 256, 2, dtype=np.uint8))
        if rng.random() < 0.1:
            h[12] = (int(rng.integers(0, 16)) << 4) | (h[12] & 0x0F)
        h += bytes(rng.integers(0, 256, width - len(h), dtype=np.uint8))
        out[i] = np.frombuffer(bytes(h[:width]), np.uint8)
    return out


# ------------------------------------------------------------ ICMP
def frame_icmp4(rng, icmp_type=8, payload_len=None, vlan=None, ihl_words=5, mf=False,
                frag_off=0, l4_len=None):
    """IPv4/ICMP frame (valid checksums): echo request/reply by default,
    identifier and sequence random; l4_len truncates the ICMP message
    (< 8 bytes: a short header)."""
    pl = int(rng.integers(0, 64)) if payload_len is None else payload_len
    ident, seq = (int(x) for x in rng.integers(0, 65536, 2))
    msg = bytearray(struct.pack(">BBHHH", icmp_type, 0, 0, ident, seq) +
                    bytes(rng.integers(0, 256, pl, dtype=np.uint8)))
    if l4_len is not None:
        msg = msg[:l4_len]
    if len(msg) >= 4:
        msg[2:4] = b"\0\0"
        struct.pack_into(">H", msg, 2, csum(bytes(msg)))
    src = bytes([10]) + bytes(rng.integers(0, 256, 3, dtype=np.uint8))
    dst = bytes([192, 168]) + bytes(rng.integers(0, 256, 2, dtype=np.uint8))
    opts = bytes(rng.integers(0, 256, (ihl_words - 5) * 4, dtype=np.uint8))
    ip = ipv4_hdr(src, dst, 1, len(msg), opts, mf=mf, frag_off=frag_off,
                  ident=int(rng.integers(0, 65536)))
    return eth(ETH_IP, vlan) + ip + bytes(msg)


def gen_icmp(n=1500, seed=0x1C3):
    """ICMP fixture frames: echo request / reply (most), other types (3, 11,
    13), short messages (< 8 bytes), fragments, IP options, VLAN tags, some
    Ethernet padding, and TCP/UDP frames in between."""
    rng = np.random.default_rng(seed)
    frames = []
    for _ in range(n):
        c = int(rng.integers(0, 100))
        vlan = int(rng.integers(1, 4095)) if rng.random() < 0.2 else None
        ihl = 5 if rng.random() < 0.8 else int(rng.integers(6, 16))
        if c < 60:
            f = frame_icmp4(rng, int(rng.choice([0, 8])), vlan=vlan, ihl_words=ihl)
        elif c < 70:
            f = frame_icmp4(rng, int(rng.choice([3, 11, 13, 5])), vlan=vlan, ihl_words=ihl)
        elif c < 76:
            f = frame_icmp4(rng, 8, vlan=vlan, l4_len=int(rng.integers(0, 8)))
        elif c < 82:
            f = frame_icmp4(rng, 8, vlan=vlan, mf=rng.random() < 0.5,
                            frag_off=int(rng.integers(0, 4)))
        else:
            f = frame_v4(rng, int(rng.choice([6, 17])), int(rng.integers(64, 200)), vlan=vlan)
        if rng.random() < 0.1:
            f = f + bytes(int(rng.integers(1, 20)))          # Ethernet padding
        frames.append(f)
    return pack(frames)
