"""Loop restoration on the device (include/dav1d_gpu.h,
Dav1dGpuLrFrame): bytefn(dav1d_lr_sbrow) (src/lr_apply_tmpl.c:169-202) over a
whole frame.

`make_lr_case` builds the three inputs dav1d holds at that point: the CDEF
output (smooth content with noise), the deblocked pre-CDEF picture it came
from (the same content with different noise; dav1d_copy_lpf saves its rows at
stripe boundaries), and a grid of restoration units per plane (none / Wiener
with taps in checkasm's ranges / self-guided with a random sgr_idx and
weights, tests/checkasm/looprestoration.c:75-160).  `DeviceLr` runs
dav1d_gpu_lr_frame_{8,16}bpc on it.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import abi


def unit_count(size, unit_size):
    """Units along one dimension (lr_sbrow's loop: the last unit takes up to 1.5x)."""
    return max(1, (size + (unit_size >> 1)) // unit_size)


@dataclass
class LrCase:
    bpc: int
    bitdepth_max: int
    layout: int
    width: int
    height: int
    sb128: int
    unit_log2: tuple        # (luma, chroma)
    restore_planes: int
    ins: list               # CDEF output per plane
    lpfs: list              # deblocked, pre-CDEF picture per plane
    units: list             # per plane: structured array [rows][cols] of abi.LrUnit

    @property
    def n_planes(self):
        return 3 if self.layout else 1

    def plane_wh(self, p):
        if p == 0:
            return self.width, self.height
        sx, sy = int(self.layout != 3), int(self.layout == 1)
        return (self.width + sx) >> sx, (self.height + sy) >> sy


def _content(rng, h, w, bdmax):
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    f = rng.uniform(0.01, 0.08, 2)
    return (0.5 + 0.35 * np.sin(xx * f[0]) * np.cos(yy * f[1])) * bdmax


def make_lr_case(seed=1, width=256, height=160, bpc=8, bitdepth_max=255, layout=1, sb128=0, unit_log2=None,
                 restore_planes=7, p_none=0.15):
    rng = np.random.default_rng(seed)
    bdmax = 255 if bpc == 8 else bitdepth_max
    pdt = np.uint8 if bpc == 8 else np.uint16
    if unit_log2 is None:
        ul = int(rng.integers(6 + sb128, 9))
        unit_log2 = (ul, max(5, ul - int(rng.integers(0, 2)) if layout == 1 else ul))
    case = LrCase(bpc, bdmax, layout, width, height, sb128, unit_log2, restore_planes, [], [], [])
    for p in range(case.n_planes):
        w, h = case.plane_wh(p)
        base = _content(rng, h, w, bdmax)
        noise = rng.uniform(0.01, 0.05) * bdmax
        case.ins.append(np.clip(np.rint(base + rng.standard_normal((h, w)) * noise), 0, bdmax).astype(pdt))
        case.lpfs.append(np.clip(np.rint(base + rng.standard_normal((h, w)) * noise), 0, bdmax).astype(pdt))
        us = 1 << unit_log2[min(p, 1)]
        rows, cols = unit_count(h, us), unit_count(w, us)
        u = (abi.LrUnit * (rows * cols))()
        for i in range(rows * cols):
            r = rng.random()
            if r < p_none:
                u[i].type = 0
            elif r < 0.55:
                u[i].type = 2
                u[i].filter_h[0] = int(rng.integers(0, 16)) - 5
                u[i].filter_h[1] = int(rng.integers(0, 32)) - 23
                u[i].filter_h[2] = int(rng.integers(0, 64)) - 17
                u[i].filter_v[0] = int(rng.integers(0, 16)) - 5
                u[i].filter_v[1] = int(rng.integers(0, 32)) - 23
                u[i].filter_v[2] = int(rng.integers(0, 64)) - 17
                if rng.random() < 0.3:   # a 5-tap unit (outer taps 0)
                    u[i].filter_h[0] = u[i].filter_v[0] = 0
            else:
                idx = int(rng.integers(0, 16))
                u[i].type = 3 + idx
                u[i].sgr_weights[0] = int(rng.integers(-96, 32)) if idx < 10 or idx >= 14 else 0
                u[i].sgr_weights[1] = int(rng.integers(-32, 96)) if idx < 14 else 0
        case.units.append((u, rows, cols))
    return case


def fill_frame(f, case, ins, lpfs, outs, unit_ptrs):
    """ins / lpfs / outs: (address, stride in pixels) per plane."""
    bpp = 1 if case.bpc == 8 else 2
    for p in range(case.n_planes):
        w, h = case.plane_wh(p)
        for dst, src in ((f.in_, ins), (f.lpf, lpfs), (f.out, outs)):
            dst[p].data, dst[p].stride, dst[p].w, dst[p].h = src[p][0], src[p][1] * bpp, w, h
        f.units[p] = unit_ptrs[p]
        f.unit_rows[p], f.unit_cols[p] = case.units[p][1], case.units[p][2]
    f.unit_size_log2[0], f.unit_size_log2[1] = case.unit_log2
    f.layout, f.bitdepth_max, f.sb128, f.restore_planes = case.layout, case.bitdepth_max, case.sb128, case.restore_planes
    return f


def algorithmic_bytes(case):
    bpp = 1 if case.bpc == 8 else 2
    return sum(2 * a.size * bpp for a in case.ins)


class DeviceLr:
    def __init__(self, case, device="cuda:0"):
        import torch
        self.torch, self.case = torch, case
        hbd = case.bpc != 8
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a.view(np.int16) if hbd else a).copy()).to(device)  # noqa: E731
        self.ins = [up(a) for a in case.ins]
        self.lpfs = [up(a) for a in case.lpfs]
        self.outs = [torch.zeros_like(t) for t in self.ins]
        self.units = [torch.from_numpy(np.frombuffer(bytes(u), np.uint8).copy()).to(device) for (u, _, _) in case.units]
        self.frame = fill_frame(abi.LrFrame(), case, [(t.data_ptr(), t.shape[1]) for t in self.ins],
                                [(t.data_ptr(), t.shape[1]) for t in self.lpfs],
                                [(t.data_ptr(), t.shape[1]) for t in self.outs], [t.data_ptr() for t in self.units])
        self.lib = abi.load_lib()

    def launch(self, stream=None, rows=None):
        """rows=(start, end): luma rows, multiples of 64 (a superblock-row
        range: the frame struct's row_start / row_end); None: the frame."""
        s = stream if stream is not None else self.torch.cuda.current_stream()
        fn = getattr(self.lib, f"dav1d_gpu_lr_frame_{8 if self.case.bpc == 8 else 16}bpc")
        self.frame.row_start, self.frame.row_end = rows if rows is not None else (0, 0)
        rc = fn(ctypes.byref(self.frame), ctypes.c_void_p(s.cuda_stream))
        self.frame.row_start = self.frame.row_end = 0
        if rc:
            raise RuntimeError(f"dav1d_gpu_lr_frame failed: {rc}")

    def outputs_host(self):
        return [t.cpu().numpy().view(np.uint16) if self.case.bpc != 8 else t.cpu().numpy() for t in self.outs]
