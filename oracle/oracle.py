"""TEST INFRASTRUCTURE ONLY -- ctypes front-end of the CPU oracle.

Two checkers live under oracle/:
  * ``Oracle``    -- liboracle.so, the C restatement (rx_oracle.c), built
                     everywhere (here and on the GPU box).
  * ``Reference`` -- _ref/libpptkref.so, the reference's own sources compiled
                     in place plus refgen.c; present where it was built in
                     this container (it travels to the GPU box untracked).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product (pptk_amd/) never does.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libpptkref.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p


class Opts(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint8 * 16), ("bits4", ctypes.c_uint8),
                ("bits6", ctypes.c_uint8), ("pad", ctypes.c_uint16),
                ("hash_size", ctypes.c_uint32)]


def make_opts(key, bits4=0, bits6=0, hash_size=1):
    o = Opts()
    kb = bytes(key)
    assert len(kb) == 16
    for i in range(16):
        o.key[i] = kb[i]
    o.bits4, o.bits6, o.hash_size = bits4, bits6, hash_size
    return o


def _ptr(a, t=_vp):
    if a is None:
        return None
    return ctypes.cast(a.ctypes.data, t)


def _tx(fn, buf, off, lens, stride, fixed_len, n):
    out = np.array(buf, dtype=np.uint8, copy=True)
    off = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    lens = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
    if n is None:
        n = len(off) if off is not None else len(buf) // stride
    fn(_ptr(out), _ptr(off), _ptr(lens), ctypes.c_uint64(stride), ctypes.c_uint32(fixed_len),
       ctypes.c_size_t(n))
    return out


def _rewrite(fn, buf, rw, off, lens, stride, fixed_len, n):
    from pptk_amd.records import REWRITE_DTYPE
    out = np.array(buf, dtype=np.uint8, copy=True)
    rw = np.ascontiguousarray(rw, dtype=REWRITE_DTYPE)
    off = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    lens = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
    if n is None:
        n = len(off) if off is not None else len(buf) // stride
    status = np.zeros(n, dtype=np.uint8)
    fn(_ptr(out), _ptr(off), _ptr(lens), ctypes.c_uint64(stride), ctypes.c_uint32(fixed_len),
       ctypes.c_size_t(n), _ptr(rw), ctypes.c_uint64(len(rw)), _ptr(status))
    return out, status


_RW_ARGS = [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t, _vp,
            ctypes.c_uint64, _vp]
_MSS_ARGS = [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_uint16,
             ctypes.c_uint32, _vp]


def _mss(fn, buf, mss, flags, off, lens, stride, fixed_len, n):
    out = np.array(buf, dtype=np.uint8, copy=True)
    off = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    lens = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
    if n is None:
        n = len(off) if off is not None else len(buf) // stride
    status = np.zeros(n, dtype=np.uint8)
    fn(_ptr(out), _ptr(off), _ptr(lens), ctypes.c_uint64(stride), ctypes.c_uint32(fixed_len),
       ctypes.c_size_t(n), ctypes.c_uint16(mss), ctypes.c_uint32(flags), _ptr(status))
    return out, status


def _frag(fn, buf, off, lens, stride, fixed_len, n):
    from pptk_amd.records import FRAG_DTYPE
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    lens = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
    if n is None:
        n = len(off) if off is not None else len(buf) // stride
    out = np.zeros(n, dtype=FRAG_DTYPE)
    fn(_ptr(buf), _ptr(off), _ptr(lens), ctypes.c_uint64(stride), ctypes.c_uint32(fixed_len),
       ctypes.c_size_t(n), _ptr(out))
    return out


_FRAG_ARGS = [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t, _vp]


class _Lib:
    prefix = ""

    def __init__(self, path):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.path = path
        self.lib = ctypes.CDLL(path)

    def _batch(self, fn, buf, off, lens, stride, fixed_len, n, opts, nthreads,
               *extra):
        from pptk_amd.records import REC_DTYPE
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
        lens = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
        recs = np.zeros(n, dtype=REC_DTYPE)
        rc = fn(_ptr(buf), _ptr(off), _ptr(lens), ctypes.c_uint64(stride),
                ctypes.c_uint32(fixed_len), ctypes.c_size_t(n),
                ctypes.byref(opts), _ptr(recs), ctypes.c_int(nthreads), *extra)
        if rc != 0:
            raise RuntimeError(f"{fn.__name__} failed: {rc}")
        return recs


class Oracle(_Lib):
    """The C restatement (oracle/rx_oracle.c)."""

    def __init__(self, path=ORACLE_SO):
        super().__init__(path)
        L = self.lib
        L.orc_cksum_buf.restype = ctypes.c_uint16
        L.orc_cksum_buf.argtypes = [_vp, ctypes.c_size_t]
        L.orc_siphash.restype = ctypes.c_uint64
        L.orc_siphash.argtypes = [_vp, _vp, ctypes.c_size_t]
        L.orc_siphash64.restype = ctypes.c_uint64
        L.orc_siphash64.argtypes = [_vp, ctypes.c_uint64]
        L.orc_ip_hdr_cksum.restype = ctypes.c_uint16
        L.orc_ip_hdr_cksum.argtypes = [_vp]
        for f in ("orc_l4_cksum_v4", "orc_l4_cksum_v6"):
            getattr(L, f).restype = ctypes.c_uint16
            getattr(L, f).argtypes = [_vp, _vp, ctypes.c_uint16, ctypes.c_uint8]
        L.orc_v6_walk.restype = ctypes.c_int
        L.orc_v6_walk.argtypes = [_vp, _u8p, ctypes.POINTER(ctypes.c_int),
                                  _u16p, ctypes.POINTER(ctypes.c_int)]
        L.orc_ip_bucket.restype = ctypes.c_uint32
        L.orc_ip_bucket.argtypes = [_vp, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_uint32]
        L.orc_ipv6_bucket.restype = ctypes.c_uint32
        L.orc_ipv6_bucket.argtypes = [_vp, _vp, ctypes.c_uint8, ctypes.c_uint32]
        L.orc_rx_batch.restype = ctypes.c_int
        L.orc_rx_batch.argtypes = [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_size_t, ctypes.POINTER(Opts), _vp,
                                   ctypes.c_int]
        L.orc_cksum_loop.restype = ctypes.c_uint32
        L.orc_cksum_loop.argtypes = [_vp, ctypes.c_size_t, ctypes.c_uint64]
        L.orc_tx_batch.restype = None
        L.orc_rewrite_batch.restype = None
        L.orc_rewrite_batch.argtypes = _RW_ARGS
        L.orc_mss_clamp_batch.restype = None
        L.orc_mss_clamp_batch.argtypes = _MSS_ARGS
        L.orc_update_cksum16.restype = ctypes.c_uint16
        L.orc_update_cksum16.argtypes = [ctypes.c_uint16] * 3
        L.orc_update_cksum32.restype = ctypes.c_uint16
        L.orc_update_cksum32.argtypes = [ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_tx_batch.argtypes = [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_size_t]
        L.orc_frag_batch.restype = None
        L.orc_frag_batch.argtypes = _FRAG_ARGS
        L.orc_permit_batch.restype = None
        L.orc_permit_batch.argtypes = [_vp, ctypes.c_size_t, ctypes.c_int, _vp, _vp, _vp]
        L.orc_tokens_refill.restype = None
        L.orc_tokens_refill.argtypes = [_vp, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.c_uint32]

    def permit_batch(self, recs, family, subject, tokens):
        """Sequential ip(v6)_permitted over records; returns (verdict,
        tokens after)."""
        recs = np.ascontiguousarray(recs)
        tok = np.array(tokens, dtype=np.uint32)
        subj = None if subject is None else np.ascontiguousarray(subject, dtype=np.uint8)
        v = np.zeros(len(recs), dtype=np.uint8)
        self.lib.orc_permit_batch(_ptr(recs), len(recs), family, _ptr(subj), _ptr(tok), _ptr(v))
        return v, tok

    def tokens_refill(self, tokens, start, end, add, initial):
        tok = np.array(tokens, dtype=np.uint32)
        self.lib.orc_tokens_refill(_ptr(tok), start, end, add, initial)
        return tok

    def frag_batch(self, buf, off=None, lens=None, stride=0, fixed_len=0, n=None):
        """struct pptk_rx_frag side records (records.FRAG_DTYPE) of a batch."""
        return _frag(self.lib.orc_frag_batch, buf, off, lens, stride, fixed_len, n)

    def tx_batch(self, buf, off=None, lens=None, stride=0, fixed_len=0, n=None):
        """Tx-side checksum setting; returns an updated copy of buf."""
        return _tx(self.lib.orc_tx_batch, buf, off, lens, stride, fixed_len, n)

    def rewrite_batch(self, buf, rw, off=None, lens=None, stride=0, fixed_len=0, n=None):
        """Header rewrite with incremental checksum updates (REWRITE_DTYPE
        entries, 1 or n); returns (updated copy of buf, status per frame)."""
        return _rewrite(self.lib.orc_rewrite_batch, buf, rw, off, lens, stride, fixed_len, n)

    def mss_clamp_batch(self, buf, mss, flags=0, off=None, lens=None, stride=0, fixed_len=0,
                        n=None):
        """TCP MSS clamping; returns (updated copy of buf, status per frame)."""
        return _mss(self.lib.orc_mss_clamp_batch, buf, mss, flags, off, lens, stride, fixed_len,
                    n)

    def update_cksum16(self, c, old, new):
        return self.lib.orc_update_cksum16(c, old, new)

    def update_cksum32(self, c, old, new):
        return self.lib.orc_update_cksum32(c, old, new)

    def cksum(self, data):
        b = bytes(data)
        return self.lib.orc_cksum_buf(b, len(b))

    def siphash(self, key, data):
        b = bytes(data)
        return self.lib.orc_siphash(bytes(key), b, len(b))

    def siphash64(self, key, v):
        return self.lib.orc_siphash64(bytes(key), v)

    def v6_walk(self, ip6):
        proto, frag, off, walked = ctypes.c_uint8(), ctypes.c_int(), ctypes.c_uint16(), ctypes.c_int()
        rc = self.lib.orc_v6_walk(bytes(ip6), ctypes.byref(proto), ctypes.byref(frag),
                                  ctypes.byref(off), ctypes.byref(walked))
        if rc != 0:
            return None
        return proto.value, frag.value, off.value

    def rx_batch(self, buf, off=None, lens=None, stride=0, fixed_len=0, n=None,
                 opts=None, nthreads=1):
        if n is None:
            n = len(off) if off is not None else len(buf) // stride
        return self._batch(self.lib.orc_rx_batch, buf, off, lens, stride,
                           fixed_len, n, opts, nthreads)

    def cksum_loop(self, buf, iters):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        return self.lib.orc_cksum_loop(_ptr(buf), buf.size, iters)


class Reference(_Lib):
    """The reference's own functions (oracle/_ref/libpptkref.so)."""

    def __init__(self, path=REF_SO):
        super().__init__(path)
        L = self.lib
        L.ref_cksum_buf.restype = ctypes.c_uint16
        L.ref_cksum_buf.argtypes = [_vp, ctypes.c_size_t]
        for f in ("ref_tcp_cksum_calc", "ref_udp_cksum_calc",
                  "ref_tcp6_cksum_calc", "ref_udp6_cksum_calc"):
            getattr(L, f).restype = ctypes.c_uint16
            getattr(L, f).argtypes = [_vp, ctypes.c_uint16, _vp, ctypes.c_uint16]
        L.ref_ip_hdr_cksum_calc.restype = ctypes.c_uint16
        L.ref_ip_hdr_cksum_calc.argtypes = [_vp, ctypes.c_uint16]
        L.ref_siphash_buf.restype = ctypes.c_uint64
        L.ref_siphash_buf.argtypes = [_vp, _vp, ctypes.c_size_t]
        L.ref_siphash64.restype = ctypes.c_uint64
        L.ref_siphash64.argtypes = [_vp, ctypes.c_uint64]
        L.ref_ipv6_proto_hdr.restype = ctypes.c_int
        L.ref_ipv6_proto_hdr.argtypes = [_vp, _u8p, ctypes.POINTER(ctypes.c_int), _u16p]
        L.ref_ip_bucket.restype = ctypes.c_uint32
        L.ref_ip_bucket.argtypes = [_vp, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_uint32]
        L.ref_ipv6_bucket.restype = ctypes.c_uint32
        L.ref_ipv6_bucket.argtypes = [_vp, _vp, ctypes.c_uint8, ctypes.c_uint32]
        L.ref_rx_batch.restype = ctypes.c_int
        L.ref_rx_batch.argtypes = [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_size_t, ctypes.POINTER(Opts), _vp,
                                   ctypes.c_int, ctypes.c_int]
        L.ref_cksum_loop.restype = ctypes.c_uint32
        L.ref_cksum_loop.argtypes = [_vp, ctypes.c_size_t, ctypes.c_uint64]
        L.ref_tx_batch.restype = None
        L.ref_rewrite_batch.restype = None
        L.ref_rewrite_batch.argtypes = _RW_ARGS
        L.ref_mss_clamp_batch.restype = None
        L.ref_mss_clamp_batch.argtypes = _MSS_ARGS
        L.ref_tcp_parse_options.restype = ctypes.c_uint32
        L.ref_tcp_parse_options.argtypes = [_vp, _vp, _vp, _vp]
        L.ref_tcp_find_sack_ts.restype = ctypes.c_uint32
        L.ref_tcp_find_sack_ts.argtypes = [_vp]
        L.ref_tcp_find_sack.restype = ctypes.c_int64
        L.ref_tcp_find_sack.argtypes = [_vp, _vp, _vp]
        L.ref_tcp_opt_op.restype = None
        L.ref_tcp_opt_op.argtypes = [_vp, ctypes.c_int, ctypes.c_uint32]
        L.ref_update_cksum16.restype = ctypes.c_uint16
        L.ref_update_cksum16.argtypes = [ctypes.c_uint16] * 3
        L.ref_update_cksum32.restype = ctypes.c_uint16
        L.ref_update_cksum32.argtypes = [ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint32]
        L.ref_tx_batch.argtypes = [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_size_t]
        L.ref_frag_batch.restype = None
        L.ref_frag_batch.argtypes = _FRAG_ARGS
        L.ref_permit_batch.restype = None
        L.ref_permit_batch.argtypes = [_vp, _vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint8,
                                       _vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]
        L.ref_tokens_refill.restype = None
        L.ref_tokens_refill.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.c_uint32, _vp]

    def permit_batch(self, key, recs, family, bits, subject, hash_size, initial, tokens):
        """The reference's ip_permitted / ipv6_permitted, once per subject
        frame in frame order; returns (verdict, tokens after)."""
        recs = np.ascontiguousarray(recs)
        tok = np.array(tokens, dtype=np.uint32)
        subj = None if subject is None else np.ascontiguousarray(subject, dtype=np.uint8)
        v = np.zeros(len(recs), dtype=np.uint8)
        self.lib.ref_permit_batch(bytes(key), _ptr(recs), len(recs), family, bits, _ptr(subj),
                                  hash_size, initial, _ptr(tok), _ptr(v))
        return v, tok

    def frag_batch(self, buf, off=None, lens=None, stride=0, fixed_len=0, n=None):
        """Fragment side records from the reference's own getters and walk."""
        return _frag(self.lib.ref_frag_batch, buf, off, lens, stride, fixed_len, n)

    def tx_batch(self, buf, off=None, lens=None, stride=0, fixed_len=0, n=None):
        """The reference's *_set_cksum_calc on every parsed frame; returns an
        updated copy of buf."""
        return _tx(self.lib.ref_tx_batch, buf, off, lens, stride, fixed_len, n)

    def rewrite_batch(self, buf, rw, off=None, lens=None, stride=0, fixed_len=0, n=None):
        """The reference's incremental-update functions (iphdr/ipcksum.h:
        213-393) as pptk_tx_rewrite_device composes them."""
        return _rewrite(self.lib.ref_rewrite_batch, buf, rw, off, lens, stride, fixed_len, n)

    def mss_clamp_batch(self, buf, mss, flags=0, off=None, lens=None, stride=0, fixed_len=0,
                        n=None):
        """The reference's tcp_parse_options + tcp_set_mss_cksum_update as
        pptk_tcp_mss_clamp_device composes them."""
        return _mss(self.lib.ref_mss_clamp_batch, buf, mss, flags, off, lens, stride, fixed_len,
                    n)

    def update_cksum16(self, c, old, new):
        return self.lib.ref_update_cksum16(c, old, new)

    def update_cksum32(self, c, old, new):
        return self.lib.ref_update_cksum32(c, old, new)

    def tokens_refill(self, hash_size, batch_size, initial, add, k, tokens):
        """The reference's batch_timer_fn for timer k (buckets
        [k*batch_size, (k+1)*batch_size))."""
        tok = np.array(tokens, dtype=np.uint32)
        self.lib.ref_tokens_refill(hash_size, batch_size, initial, add, k, _ptr(tok))
        return tok

    def cksum(self, data):
        b = bytes(data)
        return self.lib.ref_cksum_buf(b, len(b))

    def siphash(self, key, data):
        b = bytes(data)
        return self.lib.ref_siphash_buf(bytes(key), b, len(b))

    def siphash64(self, key, v):
        return self.lib.ref_siphash64(bytes(key), v)

    def v6_walk(self, ip6):
        proto, frag = ctypes.c_uint8(), ctypes.c_int()
        off = self.lib.ref_ipv6_proto_hdr(bytes(ip6), ctypes.byref(proto),
                                          ctypes.byref(frag), None)
        if off < 0:
            return None
        return proto.value, frag.value, off

    def rx_batch(self, buf, off=None, lens=None, stride=0, fixed_len=0, n=None,
                 opts=None, nthreads=1, with_bucket=True):
        if n is None:
            n = len(off) if off is not None else len(buf) // stride
        return self._batch(self.lib.ref_rx_batch, buf, off, lens, stride,
                           fixed_len, n, opts, nthreads,
                           ctypes.c_int(1 if with_bucket else 0))

    def cksum_loop(self, buf, iters):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        return self.lib.ref_cksum_loop(_ptr(buf), buf.size, iters)


def build():
    """Compile liboracle.so (+ _ref when the reference tree is present)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE], stdout=subprocess.DEVNULL)
