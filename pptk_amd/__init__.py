"""pptk_amd -- MI355X-native PPTK receive transform.

The product is the C-ABI library ``pptk_amd/libpptkrx.so`` (headers in
``include/``): hand-written gfx950 HIP kernels behind PPTK's per-packet C
APIs and a batch entry point for LDP rx loops.  ``pptk_amd.rx`` is a thin
ctypes front-end used by the tests and bench.py.
"""
from .records import REC_DTYPE  # noqa: F401

__all__ = ["REC_DTYPE"]
