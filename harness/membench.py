"""BENCH TOOLING: achievable HBM read / copy bandwidth of this box, measured
in-process (tools/membench.hip)."""
import ctypes
import os

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmembench.so")


def measure(buf, reps=10, grid=None):
    """Read and copy GB/s over torch uint8 CUDA tensor `buf` (>= 1 GiB),
    which is only read."""
    import torch
    L = ctypes.CDLL(LIB)
    vp = ctypes.c_void_p
    L.membench_read.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_int, ctypes.c_int, vp]
    L.membench_copy.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_int, vp]
    dev = buf.device
    props = torch.cuda.get_device_properties(dev)
    grid = grid or props.multi_processor_count * 8
    out = torch.zeros(1024, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    nbytes = buf.numel() // 4096 * 4096
    res = {}
    for name, nt in (("read_gbs", 0), ("read_nt_gbs", 1)):
        ts = []
        for k in range(reps + 2):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            L.membench_read(buf.data_ptr(), nbytes, out.data_ptr(), nt, grid, vp(s.cuda_stream))
            b.record()
            torch.cuda.synchronize(dev)
            if k >= 2:
                ts.append(a.elapsed_time(b))
        ts.sort()
        res[name] = round(nbytes / (ts[len(ts) // 2] * 1e-3) / 1e9, 1)
    # copy into a separate buffer: `buf` is read-only here (it holds the
    # batch under test; an in-place copy once clobbered its second half)
    half = min(nbytes // 2, 4 << 30) // 4096 * 4096
    dst = torch.empty(half, dtype=torch.uint8, device=dev)
    ts = []
    for k in range(reps + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        L.membench_copy(buf.data_ptr(), dst.data_ptr(), half, grid, vp(s.cuda_stream))
        b.record()
        torch.cuda.synchronize(dev)
        if k >= 2:
            ts.append(a.elapsed_time(b))
    ts.sort()
    res["copy_gbs"] = round(2 * half / (ts[len(ts) // 2] * 1e-3) / 1e9, 1)
    del dst
    return res
