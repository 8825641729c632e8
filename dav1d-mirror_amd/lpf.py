"""Deblocking loop filter on the device (include/
dav1d_gpu.h, Dav1dGpuLoopFilterFrame): dav1d_loopfilter_sbrow_cols / _rows
(src/lf_apply_tmpl.c:314-466) over a whole frame, in place.

`make_lpf_case` builds what the decoder holds when it deblocks: a picture with
block artifacts (smooth content, a random offset per transform block, a
little noise), a transform partition (a random quadtree per 64x64 superblock,
chroma at half size, at least 4x4), the Av1Filter edge masks the partition
implies (a filter no longer than the smaller transform on either side of the
edge, as dav1d_create_lf_mask_* derive them, src/lf_mask.c), the per-4x4
level array and the limit LUT of dav1d_calc_eih (src/lf_mask.c:412-429).
`DeviceLpf` runs dav1d_gpu_loopfilter_frame_{8,16}bpc on it.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import abi

AV1F_DTYPE = np.dtype([("filter_y", np.uint16, (2, 32, 3, 2)), ("filter_uv", np.uint16, (2, 32, 2, 2)),
                       ("cdef_idx", np.int8, (4,)), ("noskip_mask", np.uint16, (16, 2))])
assert AV1F_DTYPE.itemsize == 1348


def calc_eih(sharp):
    """dav1d_calc_eih, src/lf_mask.c:412-429."""
    e, i = np.zeros(64, np.uint8), np.zeros(64, np.uint8)
    for level in range(64):
        limit = level
        if sharp > 0:
            limit >>= (sharp + 3) >> 2
            limit = min(limit, 9 - sharp)
        limit = max(limit, 1)
        i[level], e[level] = limit, 2 * (level + 2) + limit
    return e, i, ((sharp + 3) >> 2, 9 - sharp if sharp else 0xff)


@dataclass
class LpfCase:
    bpc: int
    bitdepth_max: int
    layout: int
    width: int
    height: int
    sb128: int
    planes: list          # pixel arrays (picture before deblocking, 128-aligned allocation)
    masks: np.ndarray     # AV1F_DTYPE [sb128h][sb128w]
    level: np.ndarray     # uint8 [rows][b4_stride][4]
    lut: tuple            # (e[64], i[64], sharp[2])
    filter_uv: int

    @property
    def n_planes(self):
        return 3 if self.layout else 1

    def plane_wh(self, p):
        if p == 0:
            return self.width, self.height
        sx, sy = int(self.layout != 3), int(self.layout == 1)
        return (self.width + sx) >> sx, (self.height + sy) >> sy


def _quadtree(rng, n4, p_split):
    """Square transform sizes (in 4x4 units) per 4x4 cell of an n4 x n4 superblock."""
    out = np.zeros((n4, n4), np.int32)

    def rec(y, x, s):
        if s > 1 and (s > 16 or rng.random() < p_split):
            h = s // 2
            for dy in (0, h):
                for dx in (0, h):
                    rec(y + dy, x + dx, h)
        else:
            out[y:y + s, x:x + s] = s
    rec(0, 0, n4)
    return out


def _block_ids(tx):
    """Label each 4x4 cell with its square block (top-left cell index)."""
    h, w = tx.shape
    ids = np.zeros((h, w), np.int64)
    for y in range(h):
        for x in range(w):
            s = tx[y, x]
            ids[y, x] = ((y // s) * s) * 100000 + (x // s) * s
    return ids


def make_lpf_case(seed=1, width=256, height=128, bpc=8, bitdepth_max=255, layout=1, sb128=0, p_split=0.55,
                  p_zero_level=0.1, sharp=None, filter_uv=1):
    rng = np.random.default_rng(seed)
    bdmax = 255 if bpc == 8 else bitdepth_max
    bd8 = bdmax.bit_length() - 8
    pdt = np.uint8 if bpc == 8 else np.uint16
    w4, h4 = (width + 3) >> 2, (height + 3) >> 2
    bw, bh = ((width + 7) >> 3) << 1, ((height + 7) >> 3) << 1
    b4_stride = (bw + 31) & ~31
    sb128w, sb128h = (bw + 31) >> 5, (bh + 31) >> 5
    sx, sy = int(layout != 3), int(layout == 1)
    # the picture as dav1d allocates it: 128-aligned (src/picture.c:49-50), so
    # filters next to the bottom / right edge read allocated pixels
    aw, ah = (width + 127) & ~127, (height + 127) & ~127
    # luma transform partition: quadtree per 64x64
    S4 = 16
    tx = np.zeros((ah // 4, aw // 4), np.int32)
    for y in range(0, tx.shape[0], S4):
        for x in range(0, tx.shape[1], S4):
            tx[y:y + S4, x:x + S4] = _quadtree(rng, S4, p_split)
    masks = np.zeros((sb128h, sb128w), AV1F_DTYPE)
    level = np.zeros((sb128h * 32, b4_stride, 4), np.uint8)

    def planes_for(txp, ids, pw, ph, npl):
        out = []
        for _ in range(npl):
            yy, xx = np.mgrid[0:ph, 0:pw].astype(np.float64)
            f = rng.uniform(0.003, 0.03, 2)
            base = (0.5 + 0.3 * np.sin(xx * f[0] + yy * f[1])) * bdmax
            cells = ids[:(ph + 3) // 4, :(pw + 3) // 4]
            uniq, inv = np.unique(cells, return_inverse=True)
            off = rng.integers(-24, 25, len(uniq)) * (1 << bd8)
            offc = off[inv.reshape(cells.shape)]
            offp = np.repeat(np.repeat(offc, 4, 0), 4, 1)[:ph, :pw]
            noise = rng.integers(-2, 3, (ph, pw)) * (1 << bd8) * (rng.random() < 0.7)
            out.append(np.clip(base + offp + noise, 0, bdmax).astype(pdt))
        return out

    ids = _block_ids(tx)
    planes = planes_for(tx, ids, aw, ah, 1)
    # luma levels per block, [0] column and [1] row edges
    uniq, inv = np.unique(ids, return_inverse=True)
    for comp in (0, 1):
        per = rng.integers(0, 64, len(uniq))
        per[rng.random(len(uniq)) < p_zero_level] = 0
        lv = per[inv.reshape(ids.shape)]
        r, c = min(level.shape[0], lv.shape[0]), min(b4_stride, lv.shape[1])
        level[:r, :c, comp] = lv[:r, :c]

    def set_bit(arr, plane_key, d, i_line, size_idx, pos, per_half):
        half, bit = divmod(pos, per_half)
        arr[plane_key][d, i_line, size_idx, half] |= np.uint16(1 << bit)

    # luma edges: column edges at x (between cells x-1 and x), row edges at y
    for y in range(h4):
        for x in range(1, w4):
            if ids[y, x] != ids[y, x - 1]:
                s = min(tx[y, x], tx[y, x - 1])
                idx = 0 if s == 1 else 1 if s == 2 else 2
                set_bit(masks[y >> 5, x >> 5], "filter_y", 0, x & 31, idx, y & 31, 16)
    for y in range(1, h4):
        for x in range(w4):
            if ids[y, x] != ids[y - 1, x]:
                s = min(tx[y, x], tx[y - 1, x])
                idx = 0 if s == 1 else 1 if s == 2 else 2
                set_bit(masks[y >> 5, x >> 5], "filter_y", 1, y & 31, idx, x & 31, 16)
    if layout:
        cw4, ch4 = (w4 + sx) >> sx, (h4 + sy) >> sy
        acw4, ach4 = (aw >> sx) // 4, (ah >> sy) // 4
        # chroma blocks: the luma block at half size, at least 4x4
        ctx = np.zeros((ach4, acw4), np.int32)
        cids = np.zeros((ach4, acw4), np.int64)
        for cy in range(ach4):
            for cx in range(acw4):
                ly, lx = min(cy << sy, tx.shape[0] - 1), min(cx << sx, tx.shape[1] - 1)
                s = tx[ly, lx]
                cs = max(1, s >> max(sx, sy)) if s > 1 else 1
                ctx[cy, cx] = cs
                cids[cy, cx] = ((cy // cs) * cs) * 100000 + (cx // cs) * cs
        planes += planes_for(ctx, cids, aw >> sx, ah >> sy, 2)
        uniq, inv = np.unique(cids, return_inverse=True)
        for comp in (2, 3):
            per = rng.integers(0, 64, len(uniq))
            per[rng.random(len(uniq)) < p_zero_level] = 0
            level[:ch4, :cw4, comp] = per[inv.reshape(cids.shape)][:ch4, :cw4]
        cpx, cpy = 32 >> sx, 32 >> sy   # chroma 4x4 units per 128x128 area
        for cy in range(ch4):
            for cx in range(1, cw4):
                if cids[cy, cx] != cids[cy, cx - 1]:
                    idx = 0 if min(ctx[cy, cx], ctx[cy, cx - 1]) == 1 else 1
                    set_bit(masks[cy // cpy, cx // cpx], "filter_uv", 0, cx % cpx, idx, cy % cpy, 16 >> sy)
        for cy in range(1, ch4):
            for cx in range(cw4):
                if cids[cy, cx] != cids[cy - 1, cx]:
                    idx = 0 if min(ctx[cy, cx], ctx[cy - 1, cx]) == 1 else 1
                    set_bit(masks[cy // cpy, cx // cpx], "filter_uv", 1, cy % cpy, idx, cx % cpx, 16 >> sx)
    sh = int(rng.integers(0, 8)) if sharp is None else sharp
    return LpfCase(bpc, bdmax, layout, width, height, sb128, planes, masks, level, calc_eih(sh), filter_uv)


def fill_frame(f, case, pics, masks_ptr, level_ptr):
    """pics: (address, stride in pixels) per plane."""
    bpp = 1 if case.bpc == 8 else 2
    for p in range(case.n_planes):
        w, h = case.plane_wh(p)
        f.pic[p].data, f.pic[p].stride, f.pic[p].w, f.pic[p].h = pics[p][0], pics[p][1] * bpp, w, h
    f.masks, f.level, f.b4_stride = masks_ptr, level_ptr, case.level.shape[1]
    e, i, sharp = case.lut
    for k in range(64):
        f.lut.e[k], f.lut.i[k] = int(e[k]), int(i[k])
    f.lut.sharp[0], f.lut.sharp[1] = sharp
    f.layout, f.bitdepth_max, f.filter_uv = case.layout, case.bitdepth_max, case.filter_uv
    return f


def algorithmic_bytes(case):
    """Each pass reads and writes the picture once, plus the masks and levels."""
    bpp = 1 if case.bpc == 8 else 2
    return sum(4 * a.size * bpp for a in case.planes) + case.masks.nbytes + case.level.nbytes


class DeviceLpf:
    def __init__(self, case, device="cuda:0"):
        import torch
        self.torch, self.case = torch, case
        hbd = case.bpc != 8
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a.view(np.int16) if hbd else a).copy()).to(device)  # noqa: E731
        self.pics = [up(a) for a in case.planes]
        self.masks = torch.from_numpy(case.masks.view(np.uint8).reshape(-1).copy()).to(device)
        self.level = torch.from_numpy(case.level.reshape(-1).copy()).to(device)
        self.frame = fill_frame(abi.LoopFilterFrame(), case, [(t.data_ptr(), t.shape[1]) for t in self.pics],
                                self.masks.data_ptr(), self.level.data_ptr())
        self.lib = abi.load_lib()

    def reset(self):
        hbd = self.case.bpc != 8
        for t, a in zip(self.pics, self.case.planes):
            t.copy_(self.torch.from_numpy(np.ascontiguousarray(a.view(np.int16) if hbd else a)))

    def launch(self, stream=None, rows=None):
        """rows=(start, end): luma rows, multiples of 64 (a superblock-row
        range: the frame struct's row_start / row_end); None: the frame."""
        s = stream if stream is not None else self.torch.cuda.current_stream()
        fn = getattr(self.lib, f"dav1d_gpu_loopfilter_frame_{8 if self.case.bpc == 8 else 16}bpc")
        self.frame.row_start, self.frame.row_end = rows if rows is not None else (0, 0)
        rc = fn(ctypes.byref(self.frame), ctypes.c_void_p(s.cuda_stream))
        self.frame.row_start = self.frame.row_end = 0
        if rc:
            raise RuntimeError(f"dav1d_gpu_loopfilter_frame failed: {rc}")

    def outputs_host(self):
        return [t.cpu().numpy().view(np.uint16) if self.case.bpc != 8 else t.cpu().numpy() for t in self.pics]
