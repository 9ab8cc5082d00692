"""BENCH/TEST TOOLING: synthetic frame batches generated in HBM
(tools/synth.hip -> tools/libpptksynth.so).  See synth.hip for the recipes."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libpptksynth.so")
CFG = {"c64": 0, "c1500": 1, "cmix": 2, "imix": 3, "jmix": 4, "c1500a": 1, "c1500g": 1}
# c1500a: 1536-byte slots; c1500g: C1500 frames described by off/len arrays
SEED = 0x5EED

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise ImportError(f"{LIB} not built (make)")
        L = ctypes.CDLL(LIB)
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        L.synth_sizes.argtypes = [ctypes.c_int, u64, u64, u64, vp, vp]
        L.synth_frames.argtypes = [ctypes.c_int, u64, u64, u64, vp, vp, u64, vp, vp]
        _lib = L
    return _lib


def make_batch(cfg, n, device, first=0, seed=SEED, stream=None):
    """Frames [first, first+n) of config `cfg` ('c64' | 'c1500' | 'cmix' | 'imix' | 'jmix') in
    HBM.  Returns dict(frames, n, stride | off+lens, expect, max_len)."""
    import torch
    c = CFG[cfg]
    s = stream if stream is not None else torch.cuda.current_stream(device)
    sp = ctypes.c_void_p(s.cuda_stream)
    out = {"n": n, "cfg": cfg}
    expect = torch.empty(n, dtype=torch.uint8, device=device)
    if cfg in ("c64", "c1500", "c1500a", "c1500g"):
        stride = {"c64": 64, "c1500": 1500, "c1500a": 1536, "c1500g": 1500}[cfg]
        flen = 64 if cfg == "c64" else 1500
        frames = torch.empty(n * stride + 64, dtype=torch.uint8, device=device)
        rc = lib().synth_frames(c, seed, first, n, frames.data_ptr(), None, stride,
                                expect.data_ptr(), sp)
        out.update(frames=frames, stride=stride, fixed_len=flen, max_len=flen,
                   bytes=n * flen)
        if cfg == "c1500g":
            out["off"] = torch.arange(n, dtype=torch.int64, device=device) * stride
            out["lens"] = torch.full((n,), flen, dtype=torch.int16, device=device)
    else:
        lens = torch.empty(n, dtype=torch.int16, device=device)
        rc = lib().synth_sizes(c, seed, first, n, lens.data_ptr(), sp)
        assert rc == 0
        # frames packed back to back at 4-byte aligned offsets
        ln = lens.to(torch.int64) & 0xFFFF
        room = ln
        off = torch.zeros(n, dtype=torch.int64, device=device)
        off[1:] = torch.cumsum((room[:-1] + 3) & ~3, 0)
        total = int(off[-1].item() + room[-1].item()) + 64
        frames = torch.empty(total, dtype=torch.uint8, device=device)
        rc = lib().synth_frames(c, seed, first, n, frames.data_ptr(), off.data_ptr(), 0,
                                expect.data_ptr(), sp)
        out.update(frames=frames, off=off, lens=lens, max_len=9000 if cfg == "jmix" else 1500,
                   bytes=int(ln.sum().item()))
    assert rc == 0, rc
    out["expect"] = expect
    return out
