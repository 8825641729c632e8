"""Device intra edge preparation (include/dav1d_gpu.h, Dav1dGpuIntraEdgeBatch):
the batch form of bytefn(dav1d_prepare_intra_edges)
(src/ipred_prepare_tmpl.c:76-204), SURVEY 8(f) row 1.

`EdgeCase` is a seeded random batch of edge records over random pictures
(every coded mode and angle delta, every flag, blocks at the picture and
tile edges, superblock-top rows read from a top_edge buffer); `DeviceEdges`
uploads one and runs dav1d_gpu_prepare_intra_edges_{8,16}bpc on it.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import abi


@dataclass
class EdgeCase:
    bpc: int
    bitdepth_max: int
    pics: list          # 3 planes, (h, w) pixel arrays
    top_edge: list      # 3 arrays (sb rows, w): the pre-filter row above each
    sb_log2: tuple      # superblock height per plane, log2 px
    units: np.ndarray   # abi.UNIT_DTYPE
    recs: np.ndarray    # abi.INTRA_EDGE_DTYPE
    edges: np.ndarray   # edge pool, prefilled with noise (untouched entries must stay)

    @property
    def pixel_dtype(self):
        return np.uint8 if self.bpc == 8 else np.uint16


def make_edge_case(seed=1, bpc=8, bitdepth_max=255, n=2000, width=256, height=128, sb_log2=6):
    """Random records over one 4:2:0 picture.  Positions sit on the transform
    grid; the tile end (w4, h4) is often close to the block so the
    px_have < sz extension paths run; have_left / have_top only where a
    neighbour exists; TOP_SB_EDGE only on superblock-top rows."""
    rng = np.random.default_rng(seed)
    bdmax = 255 if bpc == 8 else bitdepth_max
    pdt = np.uint8 if bpc == 8 else np.uint16
    whs = [(width, height), (width // 2, height // 2), (width // 2, height // 2)]
    sbl = (sb_log2, sb_log2 - 1, sb_log2 - 1)
    pics = [rng.integers(0, bdmax + 1, (h, w)).astype(pdt) for (w, h) in whs]
    top = [rng.integers(0, bdmax + 1, (max(1, h >> s), w)).astype(pdt) for (w, h), s in zip(whs, sbl)]
    units = np.zeros(n, abi.UNIT_DTYPE)
    recs = np.zeros(n, abi.INTRA_EDGE_DTYPE)
    order = rng.permutation(n)          # records reach their units indirectly
    off = 0
    for i in range(n):
        pl = 0 if rng.random() < 0.5 else int(rng.integers(1, 3))
        pw4, ph4 = whs[pl][0] // 4, whs[pl][1] // 4
        while True:
            tx = int(rng.integers(0, abi.N_TX))
            tw, th = (d // 4 for d in abi.TX_WH[tx])
            if tw <= pw4 and th <= ph4:
                break
        x4 = int(rng.integers(0, pw4 // tw)) * tw
        y4 = int(rng.integers(0, ph4 // th)) * th
        w4 = pw4 if rng.random() < 0.5 else min(pw4, x4 + int(rng.integers(1, 2 * tw + 3)))
        h4 = ph4 if rng.random() < 0.5 else min(ph4, y4 + int(rng.integers(1, 2 * th + 3)))
        mode = int(rng.integers(0, 14))
        angle = int(rng.integers(-3, 4)) if 1 <= mode <= 8 else int(rng.integers(0, 5)) if mode == 13 else 0
        fl = 0
        if x4 > 0 and rng.random() < 0.8:
            fl |= abi.IE_HAVE_LEFT
        if y4 > 0 and rng.random() < 0.8:
            fl |= abi.IE_HAVE_TOP
            if (y4 * 4) % (1 << sbl[pl]) == 0 and rng.random() < 0.5:
                fl |= abi.IE_TOP_SB_EDGE
        for bit in (abi.IE_TOP_HAS_RIGHT, abi.IE_LEFT_HAS_BOTTOM, abi.IE_FILTER_EDGE, abi.IE_SMOOTH):
            if rng.random() < 0.6:
                fl |= bit
        u = int(order[i])
        units[u]["plane"], units[u]["tx"], units[u]["pred"] = pl, tx, abi.PRED_INTRA
        units[u]["txtp"] = abi.NO_RESIDUAL
        units[u]["edge_off"] = off + 8 * th
        units[u]["max_w"], units[u]["max_h"] = tw * 4, th * 4
        off += 8 * th + 8 * tw + 1
        recs[i] = (u, x4, y4, w4, h4, mode, angle, fl, 0)
    edges = rng.integers(0, bdmax + 1, off).astype(pdt)
    return EdgeCase(bpc, bdmax, pics, top, sbl, units, recs, edges)


def fill_batch(b, case, pics, tops, units, edges, recs):
    """Populate an abi.IntraEdgeBatch from addresses (ints) of the buffers."""
    bpp = 1 if case.bpc == 8 else 2
    for p in range(3):
        h, w = case.pics[p].shape
        b.pic[p].data, b.pic[p].stride, b.pic[p].w, b.pic[p].h = pics[p], w * bpp, w, h
        b.top_edge[p].data, b.top_edge[p].stride = tops[p], case.top_edge[p].shape[1] * bpp
        b.top_edge[p].w, b.top_edge[p].h = case.top_edge[p].shape[1], case.top_edge[p].shape[0]
        b.sb_log2[p] = case.sb_log2[p]
    b.units, b.edges, b.recs = units, edges, recs
    b.n_recs = len(case.recs)
    b.bitdepth_max = case.bitdepth_max
    return b


class DeviceEdges:
    """An EdgeCase uploaded to one GPU."""

    def __init__(self, case, device="cuda:0"):
        import torch
        self.torch, self.case = torch, case
        dev = torch.device(device)
        hbd = case.bpc != 8
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).to(dev)   # noqa: E731
        px = lambda a: up(a.view(np.int16) if hbd else a)                        # noqa: E731
        self.pics = [px(a) for a in case.pics]
        self.tops = [px(a) for a in case.top_edge]
        self.units = up(case.units.view(np.uint8))
        self.edges = px(case.edges)
        self.recs = up(case.recs.view(np.uint8))
        self.batch = fill_batch(abi.IntraEdgeBatch(), case, [t.data_ptr() for t in self.pics],
                                [t.data_ptr() for t in self.tops], self.units.data_ptr(),
                                self.edges.data_ptr(), self.recs.data_ptr())
        self.lib = abi.load_lib()

    def launch(self, stream=None):
        s = stream if stream is not None else self.torch.cuda.current_stream()
        fn = getattr(self.lib, f"dav1d_gpu_prepare_intra_edges_{8 if self.case.bpc == 8 else 16}bpc")
        rc = fn(ctypes.byref(self.batch), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"dav1d_gpu_prepare_intra_edges failed: {rc}")

    def results_host(self):
        units = self.units.cpu().numpy().view(abi.UNIT_DTYPE)
        e = self.edges.cpu().numpy()
        return units, (e if self.case.bpc == 8 else e.view(np.uint16))
