"""Film grain on the device (include/dav1d_gpu.h,
Dav1dGpuFilmGrainBatch): bitfn(dav1d_apply_grain) (src/fg_apply_tmpl.c:
222-241) for a whole picture.

`make_grain_data` draws film grain parameters over the ranges the
reference's checkasm uses (tests/checkasm/filmgrain.c:59-330); `GrainCase`
is a random picture plus parameters; `DeviceGrain` runs
dav1d_gpu_apply_grain_{8,16}bpc on it.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import abi


def _points(rng, num):
    """Strictly increasing x, as checkasm builds them (filmgrain.c:176-182)."""
    pad = 0xff // num
    return [(0xff * n // num + int(rng.integers(0, pad)), int(rng.integers(0, 256))) for n in range(num)]


def make_grain_data(rng, lag=None, csfl=None, num_y=None, num_uv=(None, None), overlap=None):
    d = abi.FilmGrainData()
    d.seed = int(rng.integers(0, 0x10000))
    d.grain_scale_shift = int(rng.integers(0, 4))
    d.ar_coeff_shift = int(rng.integers(6, 10))
    d.ar_coeff_lag = int(rng.integers(0, 4)) if lag is None else lag
    npos = 2 * d.ar_coeff_lag * (d.ar_coeff_lag + 1)
    for n in range(npos):
        d.ar_coeffs_y[n] = int(rng.integers(-128, 128))
    ny = (int(rng.integers(2, 15)) if rng.random() < 0.85 else 0) if num_y is None else num_y
    d.num_y_points = ny
    for n, (x, y) in enumerate(_points(rng, ny) if ny else []):
        d.y_points[n][0], d.y_points[n][1] = x, y
    d.chroma_scaling_from_luma = (1 if rng.random() < 0.25 else 0) if csfl is None else int(csfl)
    for uv in range(2):
        for n in range(npos + 1):
            d.ar_coeffs_uv[uv][n] = int(rng.integers(-128, 128))
        if d.chroma_scaling_from_luma:
            continue
        nu = (int(rng.integers(2, 11)) if rng.random() < 0.8 else 0) if num_uv[uv] is None else num_uv[uv]
        d.num_uv_points[uv] = nu
        for n, (x, y) in enumerate(_points(rng, nu) if nu else []):
            d.uv_points[uv][n][0], d.uv_points[uv][n][1] = x, y
        d.uv_mult[uv] = int(rng.integers(-128, 128))
        d.uv_luma_mult[uv] = int(rng.integers(-128, 128))
        d.uv_offset[uv] = int(rng.integers(-256, 256))
    if d.chroma_scaling_from_luma and not d.num_y_points:   # csfl scales by the luma points
        d.num_y_points = 2
        for n, (x, y) in enumerate(_points(rng, 2)):
            d.y_points[n][0], d.y_points[n][1] = x, y
    d.scaling_shift = int(rng.integers(8, 12))
    d.overlap_flag = (1 if rng.random() < 0.6 else 0) if overlap is None else int(overlap)
    d.clip_to_restricted_range = int(rng.integers(0, 2))
    return d


@dataclass
class GrainCase:
    bpc: int
    bitdepth_max: int
    layout: int          # 1 I420, 2 I422, 3 I444
    is_id: int
    data: abi.FilmGrainData
    planes: list         # 3 (h, w) pixel arrays (the reconstructed picture)

    @property
    def plane_wh(self):
        return [(a.shape[1], a.shape[0]) for a in self.planes]


def make_grain_case(seed=1, width=256, height=128, bpc=8, bitdepth_max=255, layout=1, **kw):
    rng = np.random.default_rng(seed)
    bdmax = 255 if bpc == 8 else bitdepth_max
    sx, sy = int(layout != 3), int(layout == 1)
    pdt = np.uint8 if bpc == 8 else np.uint16
    whs = [(width, height)] + [((width + sx) >> sx, (height + sy) >> sy)] * 2
    planes = [rng.integers(0, bdmax + 1, (h, w)).astype(pdt) for (w, h) in whs]
    return GrainCase(bpc, bdmax, layout, int(rng.integers(0, 2)), make_grain_data(rng, **kw), planes)


def fill_batch(b, case, ins, outs, scratch):
    """ins / outs: (address, stride in pixels) per plane."""
    bpp = 1 if case.bpc == 8 else 2
    for p, (w, h) in enumerate(case.plane_wh):
        b.in_[p].data, b.in_[p].stride, b.in_[p].w, b.in_[p].h = ins[p][0], ins[p][1] * bpp, w, h
        b.out[p].data, b.out[p].stride, b.out[p].w, b.out[p].h = outs[p][0], outs[p][1] * bpp, w, h
    b.data = case.data
    b.layout, b.bitdepth_max, b.is_id = case.layout, case.bitdepth_max, case.is_id
    b.scratch = scratch
    return b


class DeviceGrain:
    """A GrainCase on one GPU: input planes, output planes, the scratch."""

    def __init__(self, case, device="cuda:0"):
        import torch
        self.torch, self.case = torch, case
        hbd = case.bpc != 8
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a.view(np.int16) if hbd else a).copy()).to(device)  # noqa: E731
        self.ins = [up(a) for a in case.planes]
        self.outs = [torch.zeros_like(t) for t in self.ins]
        self.scratch = torch.zeros(abi.GRAIN_SCRATCH_BYTES, dtype=torch.uint8, device=device)
        self.batch = fill_batch(abi.FilmGrainBatch(), case, [(t.data_ptr(), t.shape[1]) for t in self.ins],
                                [(t.data_ptr(), t.shape[1]) for t in self.outs], self.scratch.data_ptr())
        self.lib = abi.load_lib()

    def launch(self, stream=None):
        s = stream if stream is not None else self.torch.cuda.current_stream()
        fn = getattr(self.lib, f"dav1d_gpu_apply_grain_{8 if self.case.bpc == 8 else 16}bpc")
        rc = fn(ctypes.byref(self.batch), ctypes.c_void_p(s.cuda_stream))
        if rc:
            raise RuntimeError(f"dav1d_gpu_apply_grain failed: {rc}")

    def outputs_host(self):
        return [t.cpu().numpy().view(np.uint16) if self.case.bpc != 8 else t.cpu().numpy() for t in self.outs]

    def luts_host(self):
        s = self.scratch.cpu().numpy()
        g = s[:3 * abi.GRAIN_H * abi.GRAIN_W * 2].view(np.int16).reshape(3, abi.GRAIN_H, abi.GRAIN_W)
        return g, s[3 * abi.GRAIN_H * abi.GRAIN_W * 2:].reshape(3, 4096)
