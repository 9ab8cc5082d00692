"""ctypes front-end of libpptkrx.so (include/pptk_rx.h) for tests and bench.

The product is the C-ABI library; this module only marshals torch/numpy
buffers into it.  There is no Python or CPU fallback: if the library is
missing, importing this module raises.
"""
import collections
import ctypes
import os

import numpy as np

from .records import REC32_DTYPE, REC_DTYPE

LIB_PATH = os.environ.get("PPTK_RX_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libpptkrx.so")   # env: A/B builds


class RxOpts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("key", ctypes.c_uint8 * 16),
                ("iphash_bits4", ctypes.c_uint8), ("iphash_bits6", ctypes.c_uint8),
                ("gather_threads", ctypes.c_uint16), ("iphash_size", ctypes.c_uint32),
                ("max_batch", ctypes.c_uint32), ("max_frame", ctypes.c_uint32),
                ("comm_timeout_ms", ctypes.c_uint32)]


class RxDevBatch(ctypes.Structure):
    _fields_ = [("d_frames", ctypes.c_void_p), ("d_off", ctypes.c_void_p),
                ("d_len", ctypes.c_void_p), ("d_perm", ctypes.c_void_p),
                ("stride", ctypes.c_uint64), ("fixed_len", ctypes.c_uint32),
                ("max_len", ctypes.c_uint32), ("n", ctypes.c_uint64),
                ("d_recs", ctypes.c_void_p), ("d_hash", ctypes.c_void_p),
                ("d_recs32", ctypes.c_void_p), ("d_frag", ctypes.c_void_p),
                ("d_key", ctypes.c_void_p)]


class RxRingSpec(ctypes.Structure):
    """struct pptk_rx_ring_spec (include/pptk_rx.h "Device rings")."""
    _fields_ = [("frame_bytes", ctypes.c_uint64), ("nrec", ctypes.c_uint64),
                ("rec_bytes", ctypes.c_uint32), ("probe_len", ctypes.c_uint32),
                ("frame_cands", ctypes.c_uint32), ("rec_cands", ctypes.c_uint32),
                ("reps", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("budget_bytes", ctypes.c_uint64), ("reserved", ctypes.c_uint64)]


class RxGatherSpec(ctypes.Structure):
    """struct pptk_rx_gather_spec (include/pptk_rx.h)."""
    _fields_ = [("per_rank", ctypes.c_uint64), ("nranks", ctypes.c_int32),
                ("rank", ctypes.c_int32), ("cands", ctypes.c_uint32), ("reps", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("budget_bytes", ctypes.c_uint64)]


class RxGatherC(ctypes.Structure):
    """struct pptk_rx_gather."""
    _fields_ = [("d_out", ctypes.c_void_p * 2), ("per_rank", ctypes.c_uint64),
                ("nranks", ctypes.c_int32), ("rank", ctypes.c_int32), ("device", ctypes.c_int32),
                ("cands", ctypes.c_uint32), ("chosen", ctypes.c_int32),
                ("chosen_ms", ctypes.c_float), ("first_ms", ctypes.c_float),
                ("settle_ms", ctypes.c_uint32), ("freed_bytes", ctypes.c_uint64),
                ("cand_ms", ctypes.c_float * 16)]


assert ctypes.sizeof(RxGatherSpec) == 40 and ctypes.sizeof(RxGatherC) == 128


class RxRingC(ctypes.Structure):
    """struct pptk_rx_ring."""
    _fields_ = [("d_frames", ctypes.c_void_p), ("d_recs", ctypes.c_void_p),
                ("frame_bytes", ctypes.c_uint64), ("nrec", ctypes.c_uint64),
                ("rec_bytes", ctypes.c_uint32), ("device", ctypes.c_int32),
                ("frame_cands", ctypes.c_uint32), ("rec_cands", ctypes.c_uint32),
                ("chosen_frames", ctypes.c_int32), ("chosen_recs", ctypes.c_int32),
                ("chosen_ms", ctypes.c_float), ("first_ms", ctypes.c_float),
                ("probe_frames", ctypes.c_uint64), ("freed_bytes", ctypes.c_uint64),
                ("settle_ms", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


RING_SETTLE = 0x1
RING_PROBE_HASH = 0x2


class _RingOwner:
    """Frees a pptk_rx_ring when the last tensor over it is gone."""

    def __init__(self, L, ring):
        self.L, self.ring = L, ring

    def __del__(self):
        try:
            if self.ring is not None:
                self.L.pptk_rx_ring_free(ctypes.byref(self.ring))
        except Exception:
            pass
        self.ring = None


class _DevMem:
    """A device range as a __cuda_array_interface__ object: torch.as_tensor
    wraps it without copying and keeps it (and so the ring) alive."""

    def __init__(self, owner, ptr, nbytes):
        self.owner = owner
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (ptr, False), "version": 3, "strides": None}


class _GatherOwner:
    """Frees a pptk_rx_gather when the last tensor over it is gone."""

    def __init__(self, L, g):
        self.L, self.g = L, g

    def __del__(self):
        try:
            if self.g is not None:
                self.L.pptk_rx_gather_free(ctypes.byref(self.g))
        except Exception:
            pass
        self.g = None


class DeviceGather:
    """Library-placed gather buffers (pptk_rx_gather_alloc): .out[0], .out[1]
    (torch int64, nranks * per_rank each) and the probe .report; freed once
    no tensor over them is referenced."""

    def __init__(self, ctx, g):
        import torch
        dev = torch.device("cuda", ctx.device)
        own = _GatherOwner(ctx._L, g)
        nb = g.nranks * g.per_rank * 8
        self.out = [torch.as_tensor(_DevMem(own, g.d_out[k], nb), device=dev).view(torch.int64)
                    for k in range(2)]
        self.report = {"candidates": g.cands, "chosen": g.chosen,
                       "chosen_ms": round(g.chosen_ms, 4), "first_ms": round(g.first_ms, 4),
                       "freed_bytes": g.freed_bytes, "settle_ms": g.settle_ms,
                       "candidate_ms": [round(x, 4) for x in g.cand_ms[:g.cands]],
                       "alloc": "pptk_rx_gather_alloc"}


class DeviceRing:
    """Library-owned placed device rings (pptk_rx_ring_alloc): .frames (torch
    uint8, frame_bytes + 64), .recs (torch uint8 (nrec, rec_bytes)) and the
    probe .report.  The rings are freed (pptk_rx_ring_free) once neither
    tensor (nor a view of one) is referenced any more."""

    def __init__(self, ctx, ring):
        import torch
        dev = torch.device("cuda", ctx.device)
        own = _RingOwner(ctx._L, ring)
        self.frames = torch.as_tensor(_DevMem(own, ring.d_frames, ring.frame_bytes + 64),
                                      device=dev)
        self.recs = torch.as_tensor(_DevMem(own, ring.d_recs, ring.nrec * ring.rec_bytes),
                                    device=dev).view(ring.nrec, ring.rec_bytes)
        self.report = {k: getattr(ring, k) for k in (
            "frame_cands", "rec_cands", "chosen_frames", "chosen_recs", "settle_ms",
            "probe_frames", "freed_bytes")}
        self.report["chosen_ms"] = round(ring.chosen_ms, 4)
        self.report["first_ms"] = round(ring.first_ms, 4)


class LdpPacket(ctypes.Structure):
    """struct ldp_packet (include/ldp_packet.h; reference ldp/ldp.h:98-108)."""
    _fields_ = [("data", ctypes.c_void_p), ("sz", ctypes.c_uint32),
                ("ancillary64", ctypes.c_uint64)]


assert ctypes.sizeof(LdpPacket) == 24
assert ctypes.sizeof(RxOpts) == 40

EXPORTS = ("pptk_rx_opts_default", "pptk_rx_ctx_create", "pptk_rx_ctx_destroy",
           "pptk_rx_batch", "pptk_rx_batch32", "pptk_rx_batch_submit", "pptk_rx_batch_submit32",
           "pptk_rx_batch_complete",
           "pptk_rx_batch_pending", "pptk_rx_batch_device", "pptk_rx_bin_scratch_bytes",
           "pptk_rx_bin_device", "pptk_rx_batch_device_mixed", "pptk_rx_version", "pptk_rx_set_tuning",
           "pptk_rx_variant_count", "pptk_rx_last_variant", "pptk_rx_register_ring", "pptk_rx_unregister_ring",
           "pptk_rx_permit_scratch_bytes", "pptk_rx_permit_device", "pptk_rx_permit_keys_device",
           "pptk_rx_permit_status", "pptk_rx_tokens_refill_device", "pptk_tx_cksum_device", "pptk_tx_set_side_buffer",
           "pptk_tx_rewrite_device",
           "pptk_tcp_mss_clamp_device", "pptk_rx_autotune", "pptk_rx_place_records",
           "pptk_rx_place_buffers", "pptk_rx_ring_alloc", "pptk_rx_ring_free",
           "pptk_rx_gather_alloc", "pptk_rx_gather_free",
           # multi-GPU (RCCL)
           "pptk_rx_device_count", "pptk_rx_comm_uid", "pptk_rx_comm_create",
           "pptk_rx_comm_create_all", "pptk_rx_comm_destroy", "pptk_rx_comm_info",
           "pptk_rx_comm_abort", "pptk_rx_comm_sync",
           "pptk_rx_shard_range", "pptk_rx_allgather_hash", "pptk_rx_stream_split",
           "pptk_rx_stream_destroy", "pptk_rx_abi",
           # kept per-packet APIs (ipcksum.h, hashseed.h)
           "ip_cksum_feed", "ip_hdr_cksum_calc", "tcp_cksum_calc", "udp_cksum_calc",
           "tcp6_cksum_calc", "udp6_cksum_calc", "hash_seed_init",
           "tcp_parse_options", "tcp_find_sack_ts_headers", "tcp_find_sack_header")

# Kernel variants, in the order of enum RxVariant (pptk_amd/csrc/rx_internal.h).
VARIANTS = ("T4S1", "T4S2", "T16S2", "T16S6", "T32S3", "T64S2", "T16S7L", "T32S4L",
            "T32S3D7", "T16S6D1", "T8S2", "T16S4", "L4", "M6")
RX_L4 = VARIANTS.index("L4")

_libs = {}
ABI = 6   # include/pptk_rx.h PPTK_RX_ABI


def lib(path=None):
    """Load libpptkrx.so (or the A/B build at `path`) once; raise if it is
    missing (no fallback)."""
    path = path or LIB_PATH
    if path not in _libs:
        if not os.path.exists(path):
            raise ImportError(f"{path} not built: run `make` or __graft_entry__.build()")
        L = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        # the struct layouts below are PPTK_RX_ABI's (older A/B builds lack
        # the symbol and are taken as they are)
        if hasattr(L, "pptk_rx_abi") and L.pptk_rx_abi() != ABI:
            raise ImportError(f"{path}: struct layout revision {L.pptk_rx_abi()}, "
                              f"this binding expects {ABI}")
        L.pptk_rx_opts_default.argtypes = [ctypes.POINTER(RxOpts)]
        L.pptk_rx_opts_default.restype = None
        L.pptk_rx_ctx_create.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(RxOpts)]
        L.pptk_rx_ctx_create.restype = ctypes.c_int
        L.pptk_rx_ctx_destroy.argtypes = [vp]
        L.pptk_rx_ctx_destroy.restype = None
        L.pptk_rx_batch.argtypes = [vp, vp, ctypes.c_int, vp]
        L.pptk_rx_batch.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_batch32"):   # (absent from older A/B builds)
            for f in ("pptk_rx_batch32", "pptk_rx_batch_submit32"):
                getattr(L, f).argtypes = [vp, vp, ctypes.c_int, vp]
                getattr(L, f).restype = ctypes.c_int
        L.pptk_rx_batch_device.argtypes = [vp, ctypes.POINTER(RxDevBatch), vp]
        L.pptk_rx_batch_device.restype = ctypes.c_int
        L.pptk_rx_bin_scratch_bytes.argtypes = [ctypes.c_uint64]
        L.pptk_rx_bin_scratch_bytes.restype = ctypes.c_size_t
        L.pptk_rx_bin_device.argtypes = [vp, vp, ctypes.c_uint64, vp, vp, vp]
        L.pptk_rx_bin_device.restype = ctypes.c_int
        if hasattr(L, "pptk_tx_cksum_device"):         # absent from older A/B builds
            L.pptk_tx_cksum_device.argtypes = [vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32,
                                               ctypes.c_uint64, ctypes.c_uint32, vp]
            L.pptk_tx_cksum_device.restype = ctypes.c_int
        if hasattr(L, "pptk_tx_set_side_buffer"):      # absent from older A/B builds
            L.pptk_tx_set_side_buffer.argtypes = [vp, vp, ctypes.c_uint64]
            L.pptk_tx_set_side_buffer.restype = ctypes.c_int
        if hasattr(L, "pptk_tx_rewrite_device"):       # absent from older A/B builds
            L.pptk_tx_rewrite_device.argtypes = [vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32,
                                                 ctypes.c_uint64, vp, ctypes.c_uint64, vp, vp]
            L.pptk_tx_rewrite_device.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_autotune"):             # absent from older A/B builds
            L.pptk_rx_autotune.argtypes = [vp, ctypes.POINTER(RxDevBatch), ctypes.c_int, vp]
            L.pptk_rx_autotune.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_place_records"):        # absent from older A/B builds
            L.pptk_rx_place_records.argtypes = [vp, ctypes.POINTER(RxDevBatch), ctypes.POINTER(vp),
                                                ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_int),
                                                ctypes.POINTER(ctypes.c_float), vp]
            L.pptk_rx_place_records.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_place_buffers"):        # absent from older A/B builds
            L.pptk_rx_place_buffers.argtypes = [vp, ctypes.POINTER(RxDevBatch), ctypes.POINTER(vp),
                                                ctypes.c_int, ctypes.POINTER(vp), ctypes.c_int,
                                                ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                ctypes.POINTER(ctypes.c_int),
                                                ctypes.POINTER(ctypes.c_float), vp]
            L.pptk_rx_place_buffers.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_ring_alloc"):           # absent from older A/B builds
            L.pptk_rx_ring_alloc.argtypes = [vp, ctypes.POINTER(RxRingSpec),
                                             ctypes.POINTER(RxRingC), vp]
            L.pptk_rx_ring_alloc.restype = ctypes.c_int
            L.pptk_rx_ring_free.argtypes = [ctypes.POINTER(RxRingC)]
            L.pptk_rx_ring_free.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_gather_alloc"):         # absent from older A/B builds
            L.pptk_rx_gather_alloc.argtypes = [vp, ctypes.POINTER(RxDevBatch),
                                               ctypes.POINTER(RxGatherSpec),
                                               ctypes.POINTER(RxGatherC), vp]
            L.pptk_rx_gather_alloc.restype = ctypes.c_int
            L.pptk_rx_gather_free.argtypes = [ctypes.POINTER(RxGatherC)]
            L.pptk_rx_gather_free.restype = ctypes.c_int
        if hasattr(L, "pptk_tcp_mss_clamp_device"):    # absent from older A/B builds
            L.pptk_tcp_mss_clamp_device.argtypes = [vp, vp, vp, vp, ctypes.c_uint64,
                                                    ctypes.c_uint32, ctypes.c_uint64,
                                                    ctypes.c_uint16, ctypes.c_uint32, vp, vp]
            L.pptk_tcp_mss_clamp_device.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_permit_device"):        # absent from older A/B builds
            L.pptk_rx_permit_scratch_bytes.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
            L.pptk_rx_permit_scratch_bytes.restype = ctypes.c_size_t
            L.pptk_rx_permit_device.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_int, vp,
                                                vp, vp, vp, vp]
            L.pptk_rx_permit_device.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_permit_keys_device"):   # absent from older A/B builds
            L.pptk_rx_permit_keys_device.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_int, vp,
                                                     vp, vp, vp, vp]
            L.pptk_rx_permit_keys_device.restype = ctypes.c_int
            L.pptk_rx_tokens_refill_device.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32,
                                                       ctypes.c_uint32, ctypes.c_uint32, vp]
            L.pptk_rx_tokens_refill_device.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_permit_status"):        # absent from older A/B builds
            L.pptk_rx_permit_status.argtypes = [vp, vp, vp]
            L.pptk_rx_permit_status.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_batch_device_mixed"):   # absent from older A/B builds
            L.pptk_rx_batch_device_mixed.argtypes = [vp, ctypes.POINTER(RxDevBatch), vp, vp, vp]
            L.pptk_rx_batch_device_mixed.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_allgather_hash"):       # absent from older A/B builds
            L.pptk_rx_device_count.argtypes = []
            L.pptk_rx_device_count.restype = ctypes.c_int
            L.pptk_rx_comm_uid.argtypes = [vp]
            L.pptk_rx_comm_uid.restype = ctypes.c_int
            L.pptk_rx_comm_create.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
            L.pptk_rx_comm_create.restype = ctypes.c_int
            L.pptk_rx_comm_create_all.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
            L.pptk_rx_comm_create_all.restype = ctypes.c_int
            L.pptk_rx_comm_destroy.argtypes = [vp]
            L.pptk_rx_comm_destroy.restype = ctypes.c_int
            L.pptk_rx_comm_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_int)]
            L.pptk_rx_comm_info.restype = ctypes.c_int
            u64p = ctypes.POINTER(ctypes.c_uint64)
            L.pptk_rx_shard_range.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                              u64p, u64p, u64p]
            L.pptk_rx_shard_range.restype = None
            L.pptk_rx_allgather_hash.argtypes = [vp, vp, ctypes.c_uint64, vp, vp]
            L.pptk_rx_allgather_hash.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_comm_sync"):            # absent from older A/B builds
            L.pptk_rx_comm_abort.argtypes = [vp]
            L.pptk_rx_comm_abort.restype = ctypes.c_int
            L.pptk_rx_comm_sync.argtypes = [vp, vp, ctypes.c_uint32]
            L.pptk_rx_comm_sync.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_stream_split"):         # absent from older A/B builds
            L.pptk_rx_stream_split.argtypes = [vp, ctypes.c_int, ctypes.POINTER(vp),
                                               ctypes.POINTER(vp)]
            L.pptk_rx_stream_split.restype = ctypes.c_int
            L.pptk_rx_stream_destroy.argtypes = [vp]
            L.pptk_rx_stream_destroy.restype = ctypes.c_int
        L.pptk_rx_version.restype = ctypes.c_char_p
        L.pptk_rx_set_tuning.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.pptk_rx_set_tuning.restype = ctypes.c_int
        L.pptk_rx_variant_count.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_last_variant"):   # (absent from older A/B builds)
            L.pptk_rx_last_variant.argtypes = [vp]
            L.pptk_rx_last_variant.restype = ctypes.c_int
        if hasattr(L, "pptk_rx_batch_submit"):   # (absent from older A/B builds)
            L.pptk_rx_batch_submit.argtypes = [vp, vp, ctypes.c_int, vp]
            L.pptk_rx_batch_submit.restype = ctypes.c_int
            L.pptk_rx_batch_complete.argtypes = [vp]
            L.pptk_rx_batch_complete.restype = ctypes.c_int
            L.pptk_rx_batch_pending.argtypes = [vp]
            L.pptk_rx_batch_pending.restype = ctypes.c_int
        L.pptk_rx_register_ring.argtypes = [vp, vp, ctypes.c_size_t]
        L.pptk_rx_register_ring.restype = ctypes.c_int
        L.pptk_rx_unregister_ring.argtypes = [vp, vp]
        L.pptk_rx_unregister_ring.restype = ctypes.c_int
        L.ip_hdr_cksum_calc.argtypes = [vp, ctypes.c_uint16]
        L.ip_hdr_cksum_calc.restype = ctypes.c_uint16
        for f in ("tcp_cksum_calc", "udp_cksum_calc", "tcp6_cksum_calc", "udp6_cksum_calc"):
            getattr(L, f).argtypes = [vp, ctypes.c_uint16, vp, ctypes.c_uint16]
            getattr(L, f).restype = ctypes.c_uint16
        L.ip_cksum_feed.argtypes = [ctypes.POINTER(ctypes.c_uint32), vp, ctypes.c_size_t]
        L.ip_cksum_feed.restype = None
        _libs[path] = L
    return _libs[path]


def _dp(t):
    """Device pointer of a torch tensor (or None)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class RxContext:
    """One pptk_rx_ctx (one per rx thread in a C application)."""

    def __init__(self, device=0, key=bytes(16), iphash_bits4=0, iphash_bits6=0,
                 iphash_size=1, max_batch=8192, max_frame=9216, gather_threads=1,
                 lib_path=None, comm_timeout_ms=0):
        self._L = L = lib(lib_path)
        o = RxOpts()
        L.pptk_rx_opts_default(ctypes.byref(o))
        o.device = device
        for i, b in enumerate(bytes(key)):
            o.key[i] = b
        o.iphash_bits4, o.iphash_bits6, o.iphash_size = iphash_bits4, iphash_bits6, iphash_size
        o.max_batch, o.max_frame, o.gather_threads = max_batch, max_frame, gather_threads
        if comm_timeout_ms:
            o.comm_timeout_ms = comm_timeout_ms
        self._ctx = ctypes.c_void_p()
        self._inflight = collections.deque()   # (pkts, out) of submitted host batches
        rc = L.pptk_rx_ctx_create(ctypes.byref(self._ctx), ctypes.byref(o))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_ctx_create failed ({rc})")
        self.device = device

    def set_tuning(self, variant=-1, flags=-1):
        """Force kernel variant / memory-policy flags (speed only; -1 = auto)."""
        rc = self._L.pptk_rx_set_tuning(self._ctx, variant, flags)
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_set_tuning({variant}, {flags}) failed")

    def last_variant(self):
        """Kernel variant of the last device batch (-1: none yet)."""
        return self._L.pptk_rx_last_variant(self._ctx)

    def close(self):
        if self._ctx:
            self.stream_join()
            self._L.pptk_rx_ctx_destroy(self._ctx)   # (waits for outstanding submissions)
            self._ctx = ctypes.c_void_p()
            self._inflight.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def batch_device(self, frames, n, off=None, lens=None, stride=0, fixed_len=0,
                     perm=None, recs=None, hash_out=None, max_len=0, stream=None,
                     compact=False, frag_out=None, key_out=None):
        """Asynchronous device batch on `stream` (torch stream or None = current).
        frames/off/lens/perm/recs/hash_out are torch CUDA tensors; compact:
        32-byte struct pptk_rx_rec32 records (recs is (n, 32) bytes);
        frag_out: (n, 16) uint8 tensor of struct pptk_rx_frag side records;
        key_out: (n,) int32 tensor of dense rate-limiter keys (d_key)."""
        import torch
        rb = 32 if compact else 64
        if recs is None:
            recs = torch.empty((n, rb), dtype=torch.uint8, device=frames.device)
        b = RxDevBatch(frames.data_ptr(), None if off is None else off.data_ptr(),
                       None if lens is None else lens.data_ptr(),
                       None if perm is None else perm.data_ptr(), stride, fixed_len,
                       max_len, n, None if compact else recs.data_ptr(),
                       None if hash_out is None else hash_out.data_ptr(),
                       recs.data_ptr() if compact else None,
                       None if frag_out is None else frag_out.data_ptr(),
                       None if key_out is None else key_out.data_ptr())
        s = stream if stream is not None else torch.cuda.current_stream(frames.device)
        rc = self._L.pptk_rx_batch_device(self._ctx, ctypes.byref(b), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_batch_device failed ({rc})")
        return recs

    def autotune(self, frames, n, off=None, lens=None, stride=0, fixed_len=0, max_len=0,
                 recs=None, compact=False, reps=5, stream=None):
        """pptk_rx_autotune on this batch layout (synchronous): later device
        batches of the same shape use the fastest interchangeable kernel
        variant; returns its name (VARIANTS)."""
        import torch
        rb = 32 if compact else 64
        if recs is None:
            recs = torch.empty((n, rb), dtype=torch.uint8, device=frames.device)
        b = RxDevBatch(frames.data_ptr(), None if off is None else off.data_ptr(),
                       None if lens is None else lens.data_ptr(), None, stride, fixed_len,
                       max_len, n, None if compact else recs.data_ptr(), None,
                       recs.data_ptr() if compact else None)
        s = stream if stream is not None else torch.cuda.current_stream(frames.device)
        rc = self._L.pptk_rx_autotune(self._ctx, ctypes.byref(b), reps,
                                      ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_autotune failed ({rc})")
        return self.tuned_variant(frames, n, off, lens, stride, fixed_len, max_len, compact)

    def place_records(self, frames, n, cands, off=None, lens=None, stride=0, fixed_len=0,
                      max_len=0, compact=False, reps=3, stream=None):
        """pptk_rx_place_records: run the batch into each candidate record
        buffer (torch uint8 CUDA tensors of n x 64 or n x 32 bytes) and
        return (index of the fastest, per-candidate median ms)."""
        import torch
        arr = (ctypes.c_void_p * max(1, len(cands)))(*[t.data_ptr() for t in cands])
        c0 = cands[0].data_ptr() if cands else None
        b = RxDevBatch(frames.data_ptr(), None if off is None else off.data_ptr(),
                       None if lens is None else lens.data_ptr(), None, stride, fixed_len,
                       max_len, n, None if compact else c0, None, c0 if compact else None)
        best = ctypes.c_int(-1)
        ms = (ctypes.c_float * max(1, len(cands)))()
        s = stream if stream is not None else torch.cuda.current_stream(frames.device)
        rc = self._L.pptk_rx_place_records(self._ctx, ctypes.byref(b), arr, len(cands), reps,
                                           ctypes.byref(best), ms, ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_place_records failed ({rc})")
        return best.value, [round(x, 4) for x in ms[:len(cands)]]

    def place_buffers(self, frame_cands, n, rec_cands, off=None, lens=None, stride=0,
                      fixed_len=0, max_len=0, compact=False, reps=3, stream=None):
        """pptk_rx_place_buffers: the batch (the same bytes in every frame
        candidate) on every (frames, records) pair; returns (frame index,
        record index, median ms per pair, frames-major)."""
        import torch
        nf, nr = len(frame_cands), len(rec_cands)
        fa = (ctypes.c_void_p * max(1, nf))(*[t.data_ptr() for t in frame_cands])
        ra = (ctypes.c_void_p * max(1, nr))(*[t.data_ptr() for t in rec_cands])
        f0 = frame_cands[0].data_ptr() if nf else None
        r0 = rec_cands[0].data_ptr() if nr else None
        b = RxDevBatch(f0, None if off is None else off.data_ptr(),
                       None if lens is None else lens.data_ptr(), None, stride, fixed_len,
                       max_len, n, None if compact else r0, None, r0 if compact else None)
        bf, br = ctypes.c_int(-1), ctypes.c_int(-1)
        ms = (ctypes.c_float * max(1, nf * nr))()
        dev = frame_cands[0].device if nf else torch.device("cuda", self.device)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        rc = self._L.pptk_rx_place_buffers(self._ctx, ctypes.byref(b), fa, nf, ra, nr, reps,
                                           ctypes.byref(bf), ctypes.byref(br), ms,
                                           ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_place_buffers failed ({rc})")
        return bf.value, br.value, [round(x, 4) for x in ms[:nf * nr]]

    def ring_alloc(self, frame_bytes, nrec, rec_bytes=64, probe_len=0, frame_cands=0,
                   rec_cands=0, reps=0, settle=False, stream=None, budget_bytes=0,
                   probe_hash=False):
        """pptk_rx_ring_alloc: placed device frame and record rings (a
        DeviceRing; its .report carries the probe).  probe_hash: the probe
        batches also write dense flow hashes (PPTK_RX_RING_PROBE_HASH)."""
        import torch
        spec = RxRingSpec(frame_bytes, nrec, rec_bytes, probe_len, frame_cands, rec_cands, reps,
                          (RING_SETTLE if settle else 0) | (RING_PROBE_HASH if probe_hash else 0),
                          budget_bytes, 0)
        ring = RxRingC()
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        rc = self._L.pptk_rx_ring_alloc(self._ctx, ctypes.byref(spec), ctypes.byref(ring),
                                        ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_ring_alloc failed ({rc})")
        return DeviceRing(self, ring)

    def gather_alloc(self, frames, n, per_rank, nranks, rank, off=None, lens=None, stride=0,
                     fixed_len=0, max_len=0, recs=None, compact=False, cands=0, reps=0,
                     settle=False, budget_bytes=0, stream=None):
        """pptk_rx_gather_alloc: this rank's two gather buffers, placed by a
        probe that runs the batch (frames/recs as for batch_device) with its
        hashes into each candidate; a DeviceGather."""
        import torch
        rb = 32 if compact else 64
        if recs is None:
            recs = torch.empty((n, rb), dtype=torch.uint8, device=frames.device)
        b = RxDevBatch(frames.data_ptr(), None if off is None else off.data_ptr(),
                       None if lens is None else lens.data_ptr(), None, stride, fixed_len,
                       max_len, n, None if compact else recs.data_ptr(), None,
                       recs.data_ptr() if compact else None)
        spec = RxGatherSpec(per_rank, nranks, rank, cands, reps, RING_SETTLE if settle else 0, 0,
                            budget_bytes)
        g = RxGatherC()
        s = stream if stream is not None else torch.cuda.current_stream(frames.device)
        rc = self._L.pptk_rx_gather_alloc(self._ctx, ctypes.byref(b), ctypes.byref(spec),
                                          ctypes.byref(g), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_gather_alloc failed ({rc})")
        return DeviceGather(self, g)

    def tuned_variant(self, frames, n, off=None, lens=None, stride=0, fixed_len=0, max_len=0,
                      compact=False):
        """Name of the variant a device batch of this shape launches now
        (runs one batch of it: the variant is reported by the library)."""
        import torch
        self.batch_device(frames, n, off=off, lens=lens, stride=stride, fixed_len=fixed_len,
                          max_len=max_len, compact=compact)
        torch.cuda.synchronize(frames.device)
        return VARIANTS[self._L.pptk_rx_last_variant(self._ctx)]

    def batch_device_mixed(self, frames, n, off, lens, recs=None, hash_out=None, max_len=0,
                           perm=None, scratch=None, stream=None, frag_out=None):
        """Mixed-size batch (pptk_rx_batch_device_mixed, asynchronous): batch
        order, or device binning + one launch per length group when the batch
        mixes jumbo frames with shorter ones.  perm: optional device buffer
        that receives the processing order; scratch: optional preallocated."""
        import torch
        if recs is None:
            recs = torch.empty((n, 64), dtype=torch.uint8, device=frames.device)
        if scratch is None:
            scratch = torch.empty(self._L.pptk_rx_bin_scratch_bytes(n), dtype=torch.uint8,
                                  device=frames.device)
        b = RxDevBatch(frames.data_ptr(), off.data_ptr(), lens.data_ptr(), None, 0, 0,
                       max_len, n, recs.data_ptr(),
                       None if hash_out is None else hash_out.data_ptr(), None,
                       None if frag_out is None else frag_out.data_ptr())
        s = stream if stream is not None else torch.cuda.current_stream(frames.device)
        rc = self._L.pptk_rx_batch_device_mixed(self._ctx, ctypes.byref(b), _dp(perm),
                                                _dp(scratch), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_batch_device_mixed failed ({rc})")
        return recs

    def permit_device(self, recs, family, tokens, subject=None, compact=False, verdict=None,
                      scratch=None, stream=None):
        """Batched ip(v6)_permitted over device records (torch uint8 (n, 64)
        or (n, 32) with compact); tokens: torch int32 (iphash_size) updated
        in place; returns the uint8 verdicts (1 permit, 0 deny, 2 n/a)."""
        import torch
        n = recs.shape[0]
        if verdict is None:
            verdict = torch.empty(n, dtype=torch.uint8, device=recs.device)
        if scratch is None:
            scratch = torch.empty(self._L.pptk_rx_permit_scratch_bytes(n, tokens.numel()),
                                  dtype=torch.uint8, device=recs.device)
        s = stream if stream is not None else torch.cuda.current_stream(recs.device)
        rc = self._L.pptk_rx_permit_device(self._ctx, None if compact else _dp(recs),
                                           _dp(recs) if compact else None, n, family,
                                           _dp(subject), _dp(tokens), _dp(verdict),
                                           _dp(scratch), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_permit_device failed ({rc})")
        return verdict

    def permit_keys_device(self, keys, family, tokens, subject=None, verdict=None, scratch=None,
                           stream=None):
        """pptk_rx_permit_keys_device: the rate limiter from the dense keys
        (torch int32 (n,)) a batch wrote through key_out."""
        import torch
        n = keys.numel()
        if verdict is None:
            verdict = torch.empty(n, dtype=torch.uint8, device=keys.device)
        if scratch is None:
            scratch = torch.empty(self._L.pptk_rx_permit_scratch_bytes(n, tokens.numel()),
                                  dtype=torch.uint8, device=keys.device)
        s = stream if stream is not None else torch.cuda.current_stream(keys.device)
        rc = self._L.pptk_rx_permit_keys_device(self._ctx, _dp(keys), n, family, _dp(subject),
                                                _dp(tokens), _dp(verdict), _dp(scratch),
                                                ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_permit_keys_device failed ({rc})")
        return verdict

    def permit_status(self, scratch, stream=None):
        """pptk_rx_permit_status: 0, or -ETIMEDOUT if a permit_keys_device
        call on `scratch` since the last query aborted (synchronises the
        stream)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(scratch.device)
        return self._L.pptk_rx_permit_status(self._ctx, _dp(scratch), ctypes.c_void_p(s.cuda_stream))

    def tokens_refill_device(self, tokens, start, end, add, initial, stream=None):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(tokens.device)
        rc = self._L.pptk_rx_tokens_refill_device(self._ctx, _dp(tokens), start, end, add,
                                                  initial, ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_tokens_refill_device failed ({rc})")

    def tx_cksum_device(self, frames, n, off=None, lens=None, stride=0, fixed_len=0, max_len=0,
                        stream=None):
        """Tx side: set the checksums of the frames in `frames` (torch uint8
        CUDA tensor) in place, asynchronously."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(frames.device)
        rc = self._L.pptk_tx_cksum_device(self._ctx, _dp(frames), _dp(off), _dp(lens), stride,
                                          fixed_len, n, max_len, ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_tx_cksum_device failed ({rc})")

    def tx_set_side_buffer(self, buf):
        """pptk_tx_set_side_buffer: `buf` (a CUDA tensor of >= 8 bytes per
        frame, kept alive by the caller) as the two-pass tx side array, or
        None for the context's own."""
        nbytes = 0 if buf is None else buf.numel() * buf.element_size()
        rc = self._L.pptk_tx_set_side_buffer(self._ctx, _dp(buf), nbytes // 8)
        if rc != 0:
            raise OSError(-rc, f"pptk_tx_set_side_buffer failed ({rc})")
        self._tx_side = buf

    def tx_rewrite_device(self, frames, n, rw, off=None, lens=None, stride=0, fixed_len=0,
                          status=None, stream=None):
        """Header rewrite with incremental checksum updates, in place and
        asynchronously.  rw: torch uint8 CUDA tensor of 1 or n struct
        pptk_rewrite entries (16 bytes each, records.REWRITE_DTYPE);
        status: optional torch uint8 CUDA tensor of n PPTK_RW_ST_* bytes."""
        import torch
        count = rw.numel() // 16
        s = stream if stream is not None else torch.cuda.current_stream(frames.device)
        rc = self._L.pptk_tx_rewrite_device(self._ctx, _dp(frames), _dp(off), _dp(lens), stride,
                                            fixed_len, n, _dp(rw), count, _dp(status),
                                            ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_tx_rewrite_device failed ({rc})")

    def mss_clamp_device(self, frames, n, mss, syn_only=False, off=None, lens=None, stride=0,
                         fixed_len=0, status=None, stream=None):
        """TCP MSS clamping with incremental checksum update, in place and
        asynchronously; status: optional torch uint8 CUDA tensor of n
        PPTK_MSS_ST_* bytes."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(frames.device)
        rc = self._L.pptk_tcp_mss_clamp_device(self._ctx, _dp(frames), _dp(off), _dp(lens),
                                               stride, fixed_len, n, mss, 1 if syn_only else 0,
                                               _dp(status), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_tcp_mss_clamp_device failed ({rc})")

    # ---- multi-GPU (RCCL) -------------------------------------------------
    def comm_create(self, nranks, rank, uid):
        """Join communicator `uid` (bytes from comm_uid()) as rank/nranks."""
        rc = self._L.pptk_rx_comm_create(self._ctx, nranks, rank, bytes(uid))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_comm_create({nranks}, {rank}) failed ({rc})")

    def comm_destroy(self):
        rc = self._L.pptk_rx_comm_destroy(self._ctx)
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_comm_destroy failed ({rc})")

    def comm_abort(self):
        """pptk_rx_comm_abort: cancel the communicator (any thread)."""
        rc = self._L.pptk_rx_comm_abort(self._ctx)
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_comm_abort failed ({rc})")

    def comm_sync(self, stream=None, timeout_ms=0):
        """pptk_rx_comm_sync: bounded wait for `stream` (torch stream, None =
        current) with RCCL error checks; returns 0 or the negative errno
        (-ETIMEDOUT / -EIO / -ECANCELED: the communicator is then dead)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return self._L.pptk_rx_comm_sync(self._ctx, ctypes.c_void_p(s.cuda_stream), timeout_ms)

    def comm_info(self):
        """(nranks, rank) of the context's communicator, or None."""
        nr, r = ctypes.c_int(), ctypes.c_int()
        rc = self._L.pptk_rx_comm_info(self._ctx, ctypes.byref(nr), ctypes.byref(r))
        return None if rc != 0 else (nr.value, r.value)

    def allgather_hash(self, d_hash, n, d_out, stream=None):
        """pptk_rx_allgather_hash: n u64 per rank from d_hash into d_out
        (torch int64 CUDA tensors), asynchronous on `stream`."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(d_out.device)
        rc = self._L.pptk_rx_allgather_hash(self._ctx, _dp(d_hash), n, _dp(d_out),
                                            ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_allgather_hash failed ({rc})")

    def stream_split(self, coll_cus):
        """pptk_rx_stream_split: (rx stream, collective stream) as torch
        streams on this context's device, the collective's holding coll_cus
        CUs (a multiple of 32 on an MI355X) and the batches' the rest; the
        context sizes its grids for the rest until stream_join().  Call it
        before creating the communicator (its channel cap follows coll_cus).
        The HIP streams belong to the context and are destroyed with it."""
        import torch
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        rc = self._L.pptk_rx_stream_split(self._ctx, coll_cus, ctypes.byref(a), ctypes.byref(b))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_stream_split({coll_cus}) failed ({rc})")
        dev = torch.device("cuda", self.device)
        return (torch.cuda.ExternalStream(a.value, device=dev),
                torch.cuda.ExternalStream(b.value, device=dev))

    def stream_join(self):
        """Undo stream_split: the whole chip for this context's grids again
        (the split's streams stay the context's until close())."""
        if not hasattr(self._L, "pptk_rx_stream_split"):
            return
        self._L.pptk_rx_stream_split(self._ctx, 0, None, None)

    def bin_device(self, lens, n, stream=None):
        """Stable permutation of 0..n-1 by length class (torch uint32 tensor)."""
        import torch
        perm = torch.empty(n, dtype=torch.int32, device=lens.device)
        scratch = torch.empty(self._L.pptk_rx_bin_scratch_bytes(n), dtype=torch.uint8,
                              device=lens.device)
        s = stream if stream is not None else torch.cuda.current_stream(lens.device)
        rc = self._L.pptk_rx_bin_device(self._ctx, _dp(lens), n, _dp(perm), _dp(scratch),
                                      ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_bin_device failed ({rc})")
        return perm

    def register_ring(self, buf):
        """Register numpy buffer `buf` as a zero-copy rx ring."""
        rc = self._L.pptk_rx_register_ring(self._ctx, ctypes.c_void_p(buf.ctypes.data), buf.nbytes)
        if rc != 0:
            raise OSError(-rc, "pptk_rx_register_ring failed")

    def unregister_ring(self, buf):
        rc = self._L.pptk_rx_unregister_ring(self._ctx, ctypes.c_void_p(buf.ctypes.data))
        if rc != 0:
            raise OSError(-rc, "pptk_rx_unregister_ring failed")

    def batch_host(self, pkts, out=None, compact=False):
        """pptk_rx_batch (compact: pptk_rx_batch32, 32-byte records) over a
        ctypes array of LdpPacket; returns records (into `out`, a REC_DTYPE /
        REC32_DTYPE array of len(pkts), when given: an rx loop reuses its
        record array, so its pages are not faulted in per call)."""
        n = len(pkts)
        dt = REC32_DTYPE if compact else REC_DTYPE
        if out is not None:
            assert out.dtype == dt and out.shape == (n,) and out.flags["C_CONTIGUOUS"]
            recs = out
        else:
            recs = np.zeros(n, dtype=dt)
        fn = self._L.pptk_rx_batch32 if compact else self._L.pptk_rx_batch
        rc = fn(self._ctx, ctypes.cast(pkts, ctypes.c_void_p), n, ctypes.c_void_p(recs.ctypes.data))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_batch{'32' if compact else ''} failed ({rc})")
        return recs

    def submit_host(self, pkts, out):
        """pptk_rx_batch_submit (pptk_rx_batch_submit32 when `out` is a
        REC32_DTYPE array): enqueue one batch (len(pkts) <= max_batch);
        `pkts`, the frames they point at and `out` (len(pkts) records) must
        stay alive and untouched until complete_host() has returned this
        batch.  Raises OSError(EBUSY) with PPTK_RX_MAX_INFLIGHT batches
        outstanding."""
        n = len(pkts)
        compact = out.dtype == REC32_DTYPE
        assert (compact or out.dtype == REC_DTYPE) and out.shape == (n,) and out.flags["C_CONTIGUOUS"]
        fn = self._L.pptk_rx_batch_submit32 if compact else self._L.pptk_rx_batch_submit
        rc = fn(self._ctx, ctypes.cast(pkts, ctypes.c_void_p), n, ctypes.c_void_p(out.ctypes.data))
        if rc != 0:
            raise OSError(-rc, f"pptk_rx_batch_submit failed ({rc})")
        # the library holds pointers into both until the batch completes:
        # keep the Python objects alive until then (FIFO, as completions)
        self._inflight.append((pkts, out))

    def complete_host(self):
        """pptk_rx_batch_complete: wait for the oldest outstanding batch;
        returns its frame count."""
        rc = self._L.pptk_rx_batch_complete(self._ctx)
        if rc < 0:
            raise OSError(-rc, f"pptk_rx_batch_complete failed ({rc})")
        self._inflight.popleft()
        return rc

    def pending_host(self):
        return self._L.pptk_rx_batch_pending(self._ctx)


def comm_uid(lib_path=None):
    """A new RCCL communicator id (128 bytes), made on one rank."""
    buf = ctypes.create_string_buffer(128)
    rc = lib(lib_path).pptk_rx_comm_uid(buf)
    if rc != 0:
        raise OSError(-rc, f"pptk_rx_comm_uid failed ({rc})")
    return buf.raw


def comm_create_all(ctxs):
    """One communicator over the contexts (one per GPU) of this process."""
    arr = (ctypes.c_void_p * len(ctxs))(*[c._ctx.value for c in ctxs])
    rc = ctxs[0]._L.pptk_rx_comm_create_all(arr, len(ctxs))
    if rc != 0:
        raise OSError(-rc, f"pptk_rx_comm_create_all failed ({rc})")


def shard_range(n, nranks, rank, lib_path=None):
    """(first, count, per_rank) of the equal-shard policy (pptk_rx_shard_range)."""
    f, c, p = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    lib(lib_path).pptk_rx_shard_range(n, nranks, rank, ctypes.byref(f), ctypes.byref(c),
                                      ctypes.byref(p))
    return f.value, c.value, p.value


LDP_PACKET_DTYPE = np.dtype([("data", "<u8"), ("sz", "<u4"), ("pad", "<u4"),
                             ("ancillary64", "<u8")])


def ldp_packets(buf, off, lens):
    """Build an LdpPacket array pointing into numpy buffer `buf` (kept alive
    by the caller), as ldp_in_nextpkts() would hand out."""
    n = len(off)
    a = np.zeros(n, dtype=LDP_PACKET_DTYPE)
    a["data"] = buf.ctypes.data + np.asarray(off, dtype=np.uint64)
    a["sz"] = np.asarray(lens, dtype=np.uint32)
    a["ancillary64"] = np.arange(n, dtype=np.uint64)
    arr = (LdpPacket * n).from_buffer(a)
    arr._keep = a
    return arr
