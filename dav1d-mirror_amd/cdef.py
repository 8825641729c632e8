"""CDEF on the device (include/dav1d_gpu.h,
Dav1dGpuCdefFrame): bytefn(dav1d_cdef_brow) (src/cdef_apply_tmpl.c:97-309)
over a whole deblocked frame, as dav1d_filter_sbrow_cdef
(src/recon_tmpl.c:2076-2102) runs it superblock row by superblock row.

`make_cdef_case` builds a synthetic deblocked picture (smooth content with
noise and edges, so the filter has work to do, plus checkasm's under- and
overflow fills, tests/checkasm/cdef.c:42-53), per-64x64 cdef indices, per-8x8
skip flags and the frame header's strengths; `DeviceCdef` runs
dav1d_gpu_cdef_frame_{8,16}bpc on it.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import abi


@dataclass
class CdefCase:
    bpc: int
    bitdepth_max: int
    layout: int            # 0 I400, 1 I420, 2 I422, 3 I444
    width: int             # picture size (luma pixels)
    height: int
    damping: int           # frame_hdr->cdef.damping, 3..6
    y_strength: list       # 8 entries, (pri << 2) | sec
    uv_strength: list
    cdef_idx: np.ndarray   # int8 [(bh + 15) >> 4][(bw + 15) >> 4]
    noskip: np.ndarray     # uint8 [bh >> 1][bw >> 1]
    planes: list           # 1 or 3 pixel arrays over the 8x8 grid (deblocked picture)

    @property
    def n_planes(self):
        return 3 if self.layout else 1

    @property
    def grid(self):
        """Luma size of the 8x8 block grid the reference walks (f->bw, f->bh rounded to 8 px)."""
        return ((self.width + 7) >> 3) * 8, ((self.height + 7) >> 3) * 8

    def plane_wh(self, p):
        """Visible size of plane p."""
        if p == 0:
            return self.width, self.height
        sx, sy = int(self.layout != 3), int(self.layout == 1)
        return (self.width + sx) >> sx, (self.height + sy) >> sy


def _content(rng, h, w, bdmax):
    """Smooth gradients + texture + a few edges, with per-region noise levels."""
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    f = rng.uniform(0.005, 0.05, 4)
    base = (0.5 + 0.25 * np.sin(xx * f[0] + yy * f[1]) + 0.2 * np.cos(xx * f[2] - yy * f[3])) * bdmax
    for _ in range(max(1, (h * w) // 8192)):       # step edges in random directions
        a, c = rng.uniform(-1, 1, 2)
        base += np.where(a * (xx - rng.uniform(0, w)) + c * (yy - rng.uniform(0, h)) > 0, 1, -1) * \
            rng.uniform(0, 0.15) * bdmax
    noise = np.repeat(np.repeat(rng.uniform(0, 0.06, ((h + 15) // 16, (w + 15) // 16)), 16, 0), 16, 1)[:h, :w]
    img = base + rng.standard_normal((h, w)) * noise * bdmax
    img = np.clip(np.rint(img), 0, bdmax)
    # checkasm's extreme fills on some 16x16 regions (cdef.c:42-53)
    for _ in range(max(1, (h * w) // 16384)):
        y0, x0 = int(rng.integers(0, max(1, h - 16))), int(rng.integers(0, max(1, w - 16)))
        r = rng.integers(0, 2, (16, 16))
        img[y0:y0 + 16, x0:x0 + 16] = (r if rng.random() < 0.5 else bdmax - r)[:h - y0, :w - x0]
    return img


def make_cdef_case(seed=1, width=256, height=128, bpc=8, bitdepth_max=255, layout=1, p_skip_sb=0.1,
                   p_noskip=0.85, damping=None, strengths=None):
    rng = np.random.default_rng(seed)
    bdmax = 255 if bpc == 8 else bitdepth_max
    pdt = np.uint8 if bpc == 8 else np.uint16
    bw, bh = ((width + 7) >> 3) << 1, ((height + 7) >> 3) << 1   # f->bw, f->bh (src/decode.c:3598)
    gw, gh = bw * 4, bh * 4
    sx, sy = int(layout != 3), int(layout == 1)
    planes = [_content(rng, gh, gw, bdmax).astype(pdt)]
    if layout:
        planes += [_content(rng, gh >> sy, gw >> sx, bdmax).astype(pdt) for _ in range(2)]
    if strengths is None:
        ys = [int(v) for v in rng.integers(0, 64, 8)]
        uvs = [int(v) for v in rng.integers(0, 64, 8)] if layout else [0] * 8
        ys[0], uvs[0] = 0, (uvs[0] if layout else 0)   # one index with no luma filtering
    else:
        ys, uvs = list(strengths[0]), list(strengths[1])
    n_idx = int(rng.integers(1, 9))
    sbw, sbh = (bw + 15) >> 4, (bh + 15) >> 4
    cdef_idx = rng.integers(0, n_idx, (sbh, sbw)).astype(np.int8)
    cdef_idx[rng.random((sbh, sbw)) < p_skip_sb] = -1
    noskip = (rng.random((bh >> 1, bw >> 1)) < p_noskip).astype(np.uint8)
    d = int(rng.integers(3, 7)) if damping is None else damping
    return CdefCase(bpc, bdmax, layout, width, height, d, ys, uvs, cdef_idx, noskip, planes)


def fill_frame(f, case, ins, outs, cdef_idx_ptr, noskip_ptr):
    """ins / outs: (address, stride in pixels) per plane."""
    bpp = 1 if case.bpc == 8 else 2
    for p in range(case.n_planes):
        w, h = case.plane_wh(p)
        f.in_[p].data, f.in_[p].stride, f.in_[p].w, f.in_[p].h = ins[p][0], ins[p][1] * bpp, w, h
        f.out[p].data, f.out[p].stride, f.out[p].w, f.out[p].h = outs[p][0], outs[p][1] * bpp, w, h
    f.cdef_idx, f.noskip = cdef_idx_ptr, noskip_ptr
    f.layout, f.bitdepth_max, f.damping = case.layout, case.bitdepth_max, case.damping
    for i in range(8):
        f.y_strength[i], f.uv_strength[i] = case.y_strength[i], case.uv_strength[i]
    return f


def algorithmic_bytes(case):
    """Picture read once + written once over the 8x8 grid, plus the per-block parameters."""
    bpp = 1 if case.bpc == 8 else 2
    return sum(2 * a.size * bpp for a in case.planes) + case.cdef_idx.size + case.noskip.size


class DeviceCdef:
    """A CdefCase on one GPU: input planes, output planes, parameter arrays."""

    def __init__(self, case, device="cuda:0"):
        import torch
        self.torch, self.case = torch, case
        hbd = case.bpc != 8
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a.view(np.int16) if hbd else a).copy()).to(device)  # noqa: E731
        self.ins = [up(a) for a in case.planes]
        self.outs = [torch.zeros_like(t) for t in self.ins]
        self.idx = torch.from_numpy(case.cdef_idx.copy()).to(device)
        self.noskip = torch.from_numpy(case.noskip.copy()).to(device)
        self.frame = fill_frame(abi.CdefFrame(), case, [(t.data_ptr(), t.shape[1]) for t in self.ins],
                                [(t.data_ptr(), t.shape[1]) for t in self.outs], self.idx.data_ptr(),
                                self.noskip.data_ptr())
        self.lib = abi.load_lib()

    def launch(self, stream=None, rows=None):
        """rows=(start, end): luma rows, multiples of 64 (a superblock-row
        range: the frame struct's row_start / row_end); None: the frame."""
        s = stream if stream is not None else self.torch.cuda.current_stream()
        fn = getattr(self.lib, f"dav1d_gpu_cdef_frame_{8 if self.case.bpc == 8 else 16}bpc")
        self.frame.row_start, self.frame.row_end = rows if rows is not None else (0, 0)
        rc = fn(ctypes.byref(self.frame), ctypes.c_void_p(s.cuda_stream))
        self.frame.row_start = self.frame.row_end = 0
        if rc:
            raise RuntimeError(f"dav1d_gpu_cdef_frame failed: {rc}")

    def outputs_host(self):
        return [t.cpu().numpy().view(np.uint16) if self.case.bpc != 8 else t.cpu().numpy() for t in self.outs]
