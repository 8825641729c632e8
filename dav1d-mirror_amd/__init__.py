"""dav1d-mirror_amd: MI355X-native (gfx950) reconstruction hot path of dav1d.

Host-side mirror of the reference's DSP-table interface for this path.  The
product is the C-ABI library libdav1d_gpu.so (include/dav1d_gpu.h): the
per-call DSP tables (drop-in for src/mc.h, src/ipred.h, src/itx.h) and the
batch tier (one fused launch per frame of transform units).  This package
only builds batches and calls the library; it never computes pixels itself.
"""
from . import abi  # noqa: F401

__all__ = ["abi", "workload", "batch"]
