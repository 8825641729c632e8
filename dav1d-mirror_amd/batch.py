"""Device-resident frame batches and the launch of the fused reconstruction.

torch provides device memory and the stream (plumbing only); the pixels are
produced by libdav1d_gpu.so's HIP kernels through the C ABI
(dav1d_gpu_recon_{8,16}bpc, include/dav1d_gpu.h).
"""
import ctypes
import os

import numpy as np

from . import abi


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class DeviceFrame:
    """A FrameData uploaded to one GPU, plus its output planes."""

    def __init__(self, fd, device="cuda:0", zero_coefs=False, dst_planes=None, exact_refs=None):
        """dst_planes: optional device tensors to reconstruct into, (rows >=
        h, stride in pixels >= w) each -- e.g. a frame chain's 128-aligned
        pictures -- instead of exact-size planes of its own."""
        import torch
        self.torch = torch
        self.fd = fd
        self.device = torch.device(device)
        dev = self.device
        pdt = torch.uint8 if fd.cfg.bpc == 8 else torch.int16   # int16 storage for uint16 bits
        self.units = torch.from_numpy(fd.units.view(np.uint8).copy()).to(dev)
        cf = fd.coefs.view(np.int16 if fd.cfg.bpc == 8 else np.int32)
        self.coefs = torch.from_numpy(cf.copy()).to(dev)
        ed = fd.edges if fd.cfg.bpc == 8 else fd.edges.view(np.int16)
        self.edges = torch.from_numpy(ed.copy()).to(dev)
        self.refs = []
        # exact_refs (workload.clamp_units): unpadded [ref][plane] arrays read
        # at their own origin and stride, DGPU_MX_CLAMP units clamping to them
        self.exact = exact_refs is not None
        for rp in (exact_refs if self.exact else fd.refs):
            planes = []
            for a in rp:
                src = a if fd.cfg.bpc == 8 else a.view(np.int16)
                planes.append(torch.from_numpy(src.copy()).to(dev))
            self.refs.append(planes)
        cl = fd.cfl_luma if fd.cfg.bpc == 8 else fd.cfl_luma.view(np.int16)
        self.cfl_luma = torch.from_numpy(cl.copy()).to(dev)
        if dst_planes is not None:
            self.dst = list(dst_planes)
        elif fd.dst_init is not None:
            self.dst = [torch.from_numpy((a if fd.cfg.bpc == 8 else a.view(np.int16)).copy()).to(dev)
                        for a in fd.dst_init]
        else:
            self.dst = [torch.zeros((h, w), dtype=pdt, device=dev) for (w, h) in fd.plane_wh]
        self.aux = self.aux_pool = None
        if fd.aux is not None:   # INTER_MASK masks / PAL palette records
            self.aux = torch.from_numpy(np.ascontiguousarray(fd.aux, dtype=np.int32)).to(dev)
            self.aux_pool = torch.from_numpy(np.ascontiguousarray(fd.aux_pool, dtype=np.uint8)).to(dev)
        self.zero_coefs = zero_coefs
        self.batch = self._make_batch()
        self.lib = abi.load_lib()

    def _make_batch(self):
        fd = self.fd
        bpp = 1 if fd.cfg.bpc == 8 else 2
        b = abi.FrameBatch()
        for p in range(3):
            w, h = fd.plane_wh[p]
            b.dst[p].data = self.dst[p].data_ptr()
            b.dst[p].stride = self.dst[p].shape[1] * bpp
            b.dst[p].w, b.dst[p].h = w, h
            for r in range(len(self.refs)):
                t = self.refs[r][p]
                stride = t.shape[1]
                b.ref[r][p].data = t.data_ptr() + (0 if self.exact else fd.ref_origin_offset(p)) * bpp
                b.ref[r][p].stride = stride * bpp
                b.ref[r][p].w, b.ref[r][p].h = w, h
        b.units = self.units.data_ptr()
        b.n_units = fd.n_units
        for i in range(abi.N_TX + 1):
            b.class_start[i] = int(fd.class_start[i])
        b.coef = self.coefs.data_ptr()
        b.edges = self.edges.data_ptr()
        b.bitdepth_max = fd.cfg.bitdepth_max if fd.cfg.bpc == 16 else 255
        b.zero_coefs = 1 if self.zero_coefs else 0
        b.cfl_luma.data = self.cfl_luma.data_ptr()
        b.cfl_luma.stride = self.cfl_luma.shape[1] * bpp
        b.cfl_luma.w, b.cfl_luma.h = fd.plane_wh[0]
        b.cfl_ss = 3   # 4:2:0
        if self.aux is not None:
            b.aux = self.aux.data_ptr()
            b.aux_pool = self.aux_pool.data_ptr()
        if fd.class_warp is not None:
            for i in range(abi.N_TX):
                b.class_warp[i] = int(fd.class_warp[i])
        return b

    def launch(self, stream=None):
        """Enqueue one reconstruction of the whole frame on `stream`
        (a torch.cuda.Stream; default: the current stream)."""
        torch = self.torch
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        fn = self.lib.dav1d_gpu_recon_8bpc if self.fd.cfg.bpc == 8 else self.lib.dav1d_gpu_recon_16bpc
        # (the unit batch reads references with their edge-replicated
        # borders: the whole padded allocation is the reference's range)
        _bounds_buffers(self.lib, [(self.units, 10), (self.coefs, 12), (self.edges, 13)] +
                        [(t, 14 if i == 0 else 15) for i, t in enumerate((self.aux, self.aux_pool))] +
                        [(t, 1) for planes in self.refs for t in planes])
        rc = fn(ctypes.byref(self.batch), ctypes.c_void_p(s.cuda_stream))
        _bounds_buffers(self.lib, None)
        if rc != 0:
            raise RuntimeError(f"dav1d_gpu_recon failed: {rc}")

    def planes_host(self):
        """Reconstructed planes as numpy arrays (uint8 / uint16)."""
        out = []
        for p, t in enumerate(self.dst):
            w, h = self.fd.plane_wh[p]
            a = t[:h, :w].cpu().numpy()
            out.append(a if self.fd.cfg.bpc == 8 else a.view(np.uint16))
        return out

    def device_tensors(self):
        """Every device buffer the batch reads or writes (footprint accounting)."""
        ts = [self.units, self.coefs, self.edges, self.cfl_luma] + list(self.dst)
        ts += [t for planes in self.refs for t in planes]
        return ts + [t for t in (self.aux, self.aux_pool) if t is not None]


def _bounds_buffers(lib, bufs):
    """The diagnostics build (DAV1D_GPU_LIB_VARIANT=bounds): register the
    batch's own device buffers for its next launch (ids: csrc/bounds.hpp),
    each up to the end of the 16-byte block holding its last byte (the
    kernels read coefficients, edges and records as aligned 16-byte blocks;
    include/dav1d_gpu.h states the contract).  bufs=None clears the list."""
    if os.environ.get("DAV1D_GPU_LIB_VARIANT") != "bounds":
        return
    lib.dav1d_gpu_debug_register_buffer(None, 0, 0)   # clear
    for t, bid in bufs or ():
        if t is not None and t.numel():
            n = t.numel() * t.element_size()
            n += (-(t.data_ptr() + n)) & 15
            lib.dav1d_gpu_debug_register_buffer(t.data_ptr(), n, bid)


class DeviceTiles:
    """A TileData (tiles.build_tiles) uploaded to one GPU, plus its output
    planes: the superblock-tile batch (dav1d_gpu_recon_tiles_{8,16}bpc)."""

    def __init__(self, fd, td, device="cuda:0", zero_coefs=False):
        import torch
        self.torch = torch
        self.fd, self.td = fd, td
        self.device = torch.device(device)
        dev = self.device
        hbd = fd.cfg.bpc != 8
        pdt = torch.uint8 if not hbd else torch.int16   # int16 storage for uint16 bits
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).to(dev)   # noqa: E731
        self.tiles = up(td.tiles.view(np.uint8))
        self.preds = up(td.preds.view(np.uint8))
        self.txs = up(td.txs.view(np.uint8))
        self.coefs = up(td.coefs.view(np.int16 if not hbd else np.int32))
        self.edges = up(td.edges if not hbd else td.edges.view(np.int16))
        self.aux_pool = up(td.aux_pool) if td.aux_pool is not None else None
        self.refs = [[up(a if not hbd else a.view(np.int16)) for a in rp] for rp in fd.refs]
        self.cfl_luma = up(fd.cfl_luma if not hbd else fd.cfl_luma.view(np.int16))
        if fd.dst_init is not None:
            self.dst = [up(a if not hbd else a.view(np.int16)) for a in fd.dst_init]
        else:
            self.dst = [torch.zeros((h, w), dtype=pdt, device=dev) for (w, h) in fd.plane_wh]
        self.zero_coefs = zero_coefs
        self.batch = self._make_batch()
        self.lib = abi.load_lib()

    def _make_batch(self):
        fd, td = self.fd, self.td
        bpp = 1 if fd.cfg.bpc == 8 else 2
        b = abi.TileBatch()
        for p in range(3):
            w, h = fd.plane_wh[p]
            b.dst[p].data = self.dst[p].data_ptr()
            b.dst[p].stride = self.dst[p].shape[1] * bpp
            b.dst[p].w, b.dst[p].h = w, h
            for r in range(len(self.refs)):
                t = self.refs[r][p]
                b.ref[r][p].data = t.data_ptr() + fd.ref_origin_offset(p) * bpp
                b.ref[r][p].stride = t.shape[1] * bpp
                b.ref[r][p].w, b.ref[r][p].h = w, h   # the clamp bounds (emu_edge)
        b.tiles = self.tiles.data_ptr()
        b.n_tiles = len(td.tiles)
        b.n_tiles_huge = td.n_tiles_huge
        b.bitdepth_max = fd.cfg.bitdepth_max if fd.cfg.bpc == 16 else 255
        b.preds = self.preds.data_ptr()
        b.txs = self.txs.data_ptr()
        b.coef = self.coefs.data_ptr()
        b.edges = self.edges.data_ptr()
        b.aux_pool = self.aux_pool.data_ptr() if self.aux_pool is not None else None
        b.cfl_luma.data = self.cfl_luma.data_ptr()
        b.cfl_luma.stride = self.cfl_luma.shape[1] * bpp
        b.cfl_luma.w, b.cfl_luma.h = fd.plane_wh[0]
        b.cfl_ss = 3   # 4:2:0
        b.zero_coefs = 1 if self.zero_coefs else 0
        return b

    def launch(self, stream=None):
        """Enqueue one reconstruction of every tile on `stream` (a
        torch.cuda.Stream; default: the current stream)."""
        torch = self.torch
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        fn = self.lib.dav1d_gpu_recon_tiles_8bpc if self.fd.cfg.bpc == 8 else self.lib.dav1d_gpu_recon_tiles_16bpc
        _bounds_buffers(self.lib, ((self.tiles, 21), (self.preds, 22), (self.txs, 23), (self.coefs, 12),
                                   (self.edges, 13), (self.aux_pool, 15)))
        rc = fn(ctypes.byref(self.batch), ctypes.c_void_p(s.cuda_stream))
        _bounds_buffers(self.lib, None)
        if rc != 0:
            raise RuntimeError(f"dav1d_gpu_recon_tiles failed: {rc}")

    def planes_host(self):
        out = []
        for t in self.dst:
            a = t.cpu().numpy()
            out.append(a if self.fd.cfg.bpc == 8 else a.view(np.uint16))
        return out
