"""Super-res frame tier: dav1d_gpu_resize_frame_* runs
bytefn(dav1d_filter_sbrow_resize) (src/recon_tmpl.c:2104-2137) for a whole
frame.  Host side: the frame parameters as dav1d derives them (the coded
width from the super-res denominator, resize_step / resize_start of
src/decode.c:3365-3369, 3575-3583), seeded test pictures, the device launch.
Nothing here is timed."""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import abi


def _cdiv(a, b):   # C integer division (truncation toward zero)
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def scale_fac(ref_sz, this_sz):   # src/decode.c:3517-3518
    return _cdiv((ref_sz << 14) + (this_sz >> 1), this_sz)


def upscale_x0(in_w, out_w, step):   # get_upscale_x0, src/decode.c:3365-3369
    err = out_w * step - (in_w << 14)
    x0 = _cdiv(-((out_w - in_w) << 13) + (out_w >> 1), out_w) + 128 - _cdiv(err, 2)
    return x0 & 0x3fff


def coded_width(W, denom):
    """The frame's coded (downscaled) width for upscaled width W and
    super-res denominator 9..16 (AV1 spec 7.21: (W * 8 + d / 2) / d, at
    least min(W, 16))."""
    return max((W * 8 + denom // 2) // denom, min(W, 16))


@dataclass
class ResizeCase:
    W: int                    # upscaled luma width (f->sr_cur.p.p.w)
    H: int                    # picture height (f->cur.p.h)
    denom: int                # super-res denominator, 9..16
    layout: int = 1           # 0 I400, 1 I420, 2 I422, 3 I444
    bpc: int = 8
    bitdepth_max: int = 255
    sb128: int = 0
    seed: int = 1
    w: int = 0                # coded width, derived
    step: tuple = (0, 0)
    start: tuple = (0, 0)
    ins: list = field(default_factory=list)      # per plane: rows x stride, valid up to src_w
    src_w: list = field(default_factory=list)
    dst_w: list = field(default_factory=list)

    @property
    def n_planes(self):
        return 3 if self.layout else 1

    @property
    def dtype(self):
        return np.uint8 if self.bpc == 8 else np.uint16


def make_case(W, H, denom, layout=1, bpc=8, bitdepth_max=255, sb128=0, seed=1):
    c = ResizeCase(W=W, H=H, denom=denom, layout=layout, bpc=bpc, bitdepth_max=bitdepth_max, sb128=sb128, seed=seed)
    c.w = coded_width(W, denom)
    ss_hor, ss_ver = layout in (1, 2), layout == 1
    in_cw, out_cw = (c.w + ss_hor) >> ss_hor, (W + ss_hor) >> ss_hor
    s0 = scale_fac(c.w, W)
    s1 = scale_fac(in_cw, out_cw)
    c.step = (s0, s1)
    c.start = (upscale_x0(c.w, W, s0), upscale_x0(in_cw, out_cw, s1))
    rng = np.random.default_rng(seed)
    grid_w = ((c.w + 7) >> 3) << 3   # 4 * f->bw
    for p in range(c.n_planes):
        sh, sv = (ss_hor, ss_ver) if p else (0, 0)
        sw, rows = (grid_w + sh) >> sh, (H + sv) >> sv
        stride = (sw + 16 + 15) // 16 * 16   # some columns past src_w (never read)
        a = rng.integers(0, bitdepth_max + 1, size=(rows, stride), dtype=c.dtype)
        c.ins.append(a)
        c.src_w.append(sw)
        c.dst_w.append((W + sh) >> sh)
    return c


def fill(case, ins, outs):
    """A Dav1dGpuResizeFrame over (pointer, stride in pixels) pairs."""
    f = abi.ResizeFrame()
    B = case.bpc // 8
    for p in range(case.n_planes):
        f.in_[p].data, f.in_[p].stride = ins[p][0], ins[p][1] * B
        f.in_[p].w, f.in_[p].h = case.src_w[p], case.ins[p].shape[0]
        f.out[p].data, f.out[p].stride = outs[p][0], outs[p][1] * B
        f.out[p].w, f.out[p].h = case.dst_w[p], case.ins[p].shape[0]
    f.step[0], f.step[1] = case.step
    f.start[0], f.start[1] = case.start
    f.layout, f.bitdepth_max, f.sb128 = case.layout, case.bitdepth_max, case.sb128
    return f


def out_shapes(case):
    return [(case.ins[p].shape[0], (case.dst_w[p] + 15) // 16 * 16) for p in range(case.n_planes)]


class DeviceResize:
    """A case's planes on one GPU and its launch (buffers kept for repeats)."""

    def __init__(self, case, dev):
        import torch
        self.torch, self.case, self.dev = torch, case, torch.device(dev)
        tdt = torch.uint8 if case.bpc == 8 else torch.int16
        self.ins = [torch.from_numpy(a.view(np.int16) if case.bpc != 8 else a).to(self.dev) for a in case.ins]
        self.outs = [torch.zeros(sh, dtype=tdt, device=self.dev) for sh in out_shapes(case)]
        self.f = fill(case, [(t.data_ptr(), t.shape[1]) for t in self.ins], [(t.data_ptr(), t.shape[1]) for t in self.outs])
        self.fn = getattr(abi.load_lib(), f"dav1d_gpu_resize_frame_{8 if case.bpc == 8 else 16}bpc")
        self.fn.argtypes = [ctypes.POINTER(abi.ResizeFrame), ctypes.c_void_p]
        self.fn.restype = ctypes.c_int

    def launch(self, stream=None):
        s = stream if stream is not None else self.torch.cuda.current_stream(self.dev)
        rc = self.fn(ctypes.byref(self.f), ctypes.c_void_p(s.cuda_stream))
        if rc:
            raise RuntimeError(f"dav1d_gpu_resize_frame: {rc}")

    def outputs_host(self):
        res = []
        for p, t in enumerate(self.outs):
            a = t.cpu().numpy()
            res.append((a.view(np.uint16) if self.case.bpc != 8 else a)[:, :self.case.dst_w[p]])
        return res


def algorithmic_bytes(case):
    """Each source row read once (coded width) and each output row written once."""
    B = case.bpc // 8
    return sum(a.shape[0] * (case.src_w[p] + case.dst_w[p]) * B for p, a in enumerate(case.ins))


def run_gpu(case, dev, stream=None, reps=1):
    """The frame tier on `dev`; returns the upscaled planes (host arrays,
    cropped to dst_w)."""
    import torch
    L = abi.load_lib()
    tdt = torch.uint8 if case.bpc == 8 else torch.int16
    ins = [torch.from_numpy(a.view(np.int16) if case.bpc != 8 else a).to(dev) for a in case.ins]
    outs = [torch.zeros(sh, dtype=tdt, device=dev) for sh in out_shapes(case)]
    f = fill(case, [(t.data_ptr(), t.shape[1]) for t in ins], [(t.data_ptr(), t.shape[1]) for t in outs])
    fn = getattr(L, f"dav1d_gpu_resize_frame_{8 if case.bpc == 8 else 16}bpc")
    fn.argtypes = [ctypes.POINTER(abi.ResizeFrame), ctypes.c_void_p]
    fn.restype = ctypes.c_int
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    for _ in range(reps):
        rc = fn(ctypes.byref(f), ctypes.c_void_p(s.cuda_stream))
        if rc:
            raise RuntimeError(f"dav1d_gpu_resize_frame: {rc}")
    torch.cuda.synchronize(dev)
    res = []
    for p, t in enumerate(outs):
        a = t.cpu().numpy()
        res.append((a.view(np.uint16) if case.bpc != 8 else a)[:, :case.dst_w[p]])
    return res


def resize_filters():
    """dav1d_resize_filter (src/tables.c) as csrc/dsp_tables.h holds it
    (tools/gen_tables.py): [64][8] int8."""
    import os
    import re
    txt = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "dsp_tables.h")).read()
    body = txt[txt.index("dspt_resize[64 * 8] = {"):]
    body = body[body.index("{") + 1:body.index("};")]
    v = [int(x) for x in re.findall(r"-?\d+", body)]
    assert len(v) == 512
    return np.array(v, np.int64).reshape(64, 8)


def restate_rows(case):
    """Second restatement (numpy): resize_c (src/mc_tmpl.c:877-903) applied to
    every row of every plane at once, with no superblock-row walk."""
    out = []
    k = resize_filters()   # [64][8] int8
    for p in range(case.n_planes):
        src = case.ins[p][:, :case.src_w[p]].astype(np.int64)
        x = np.arange(case.dst_w[p], dtype=np.int64)
        pos = case.start[1 if p else 0] + x * case.step[1 if p else 0]
        sx = (pos >> 14) - 1
        taps = k[(pos & 0x3fff) >> 8]                       # [dst_w][8]
        idx = np.clip(sx[:, None] + np.arange(8)[None, :] - 3, 0, case.src_w[p] - 1)
        s = (src[:, idx] * taps[None, :, :]).sum(axis=2)    # [rows][dst_w]
        out.append(np.clip((-s + 64) >> 7, 0, case.bitdepth_max).astype(case.dtype))
    return out
