"""ctypes front-end of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product.  See dsp_ref.c's header
for what this restates and why parity is unpinned against the reference
binary.
"""
import ctypes
import os
import sys
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _abi():
    pkg = sys.modules.get("dav1d_mirror_amd")
    if pkg is None:
        raise RuntimeError("load the dav1d_mirror_amd package first (tests/conftest.py does)")
    return pkg.abi


def load():
    global _LIB
    if _LIB is None:
        p = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(p):
            raise RuntimeError(f"{p} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(p)
        abi = _abi()
        for bpc in (8, 16):
            f = getattr(L, f"oracle_recon_units_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(abi.FrameBatch), ctypes.c_int, ctypes.c_int]
            f.restype = ctypes.c_int
        _LIB = L
    return _LIB


class HostFrame:
    """The same FrameData reconstructed on the CPU by the oracle."""

    def __init__(self, fd):
        abi = _abi()
        self.fd = fd
        pdt = fd.cfg.pixel_dtype
        self.dst = [np.zeros((h, w), pdt) for (w, h) in fd.plane_wh]
        self.units = np.ascontiguousarray(fd.units)
        self.coefs = fd.coefs.copy()
        self.edges = np.ascontiguousarray(fd.edges)
        self.refs = fd.refs
        bpp = 1 if fd.cfg.bpc == 8 else 2
        b = abi.FrameBatch()
        for p in range(3):
            w, h = fd.plane_wh[p]
            b.dst[p].data = self.dst[p].ctypes.data
            b.dst[p].stride = w * bpp
            b.dst[p].w, b.dst[p].h = w, h
            for r in range(len(self.refs)):
                a = self.refs[r][p]
                b.ref[r][p].data = a.ctypes.data + fd.ref_origin_offset(p) * bpp
                b.ref[r][p].stride = a.shape[1] * bpp
                b.ref[r][p].w, b.ref[r][p].h = w, h
        b.units = self.units.ctypes.data
        b.n_units = fd.n_units
        for i in range(abi.N_TX + 1):
            b.class_start[i] = int(fd.class_start[i])
        b.coef = self.coefs.ctypes.data
        b.edges = self.edges.ctypes.data
        b.bitdepth_max = fd.cfg.bitdepth_max if fd.cfg.bpc == 16 else 255
        b.zero_coefs = 0
        self.batch = b

    def run(self, u0=0, u1=None, threads=1):
        """Reconstruct units [u0, u1); `threads` > 1 splits the range over
        OS threads (ctypes releases the GIL during the call)."""
        L = load()
        fn = L.oracle_recon_units_8bpc if self.fd.cfg.bpc == 8 else L.oracle_recon_units_16bpc
        if u1 is None:
            u1 = self.fd.n_units
        if threads <= 1:
            fn(ctypes.byref(self.batch), u0, u1)
            return
        bounds = np.linspace(u0, u1, threads + 1).astype(int)
        ts = [threading.Thread(target=fn, args=(ctypes.byref(self.batch), int(bounds[i]),
                                                int(bounds[i + 1]))) for i in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
