"""One frame through the whole pixel pipeline on one stream, every picture
resident in HBM: reconstruction (the unit batch, dav1d_gpu_recon_*), then
what dav1d_filter_sbrow runs per superblock row (src/recon_tmpl.c:2104-2160,
driven from src/decode.c / thread_task.c) -- deblocking
(dav1d_gpu_loopfilter_frame_*), CDEF (dav1d_gpu_cdef_frame_*), loop
restoration (dav1d_gpu_lr_frame_*) -- and film grain on the output picture
(dav1d_gpu_apply_grain_*, src/fg_apply_tmpl.c:222-241).

Pictures are allocated the way dav1d's picture allocator does (128-aligned
width and height, src/picture.c:49-66), so every stage reads and writes the
same buffers in place of host copies:

    recon -> A (deblocked in place) -> CDEF: A -> B -> LR: B (+ A's rows
    around each stripe, what dav1d_copy_lpf keeps) -> C -> grain: C -> D

Post-filter parameters (edge masks and levels, CDEF indices and strengths,
restoration units, grain parameters) are each stage's synthetic generator
at the frame's size.  `host_chain` runs the oracle walkers in the same
order (test infrastructure).  4:2:0 only."""
import ctypes
import dataclasses

import numpy as np

from . import abi


def aligned_dims(w, h):
    aw, ah = (w + 127) & ~127, (h + 127) & ~127
    return [(aw, ah), (aw >> 1, ah >> 1), (aw >> 1, ah >> 1)]


@dataclasses.dataclass
class ChainCases:
    lpf: object
    cdef: object
    lr: object
    grain: object


def make_cases(fd, seed=1):
    from . import cdef, grain, lpf, lr
    c = fd.cfg
    kw = dict(width=c.width, height=c.height, bpc=c.bpc, bitdepth_max=c.bitdepth_max, layout=1)
    return ChainCases(lpf=lpf.make_lpf_case(seed=seed, **kw),
                      cdef=cdef.make_cdef_case(seed=seed + 1, **kw),
                      lr=lr.make_lr_case(seed=seed + 2, unit_log2=(6, 5), **kw),
                      grain=grain.make_grain_case(seed=seed + 3, lag=3, overlap=True, **kw))


class DeviceChain:
    """The frame and its post-filter stages on one GPU (buffers A..D)."""

    def __init__(self, fd, cases, device="cuda:0"):
        import torch
        from . import batch, cdef, grain, lpf, lr
        self.torch, self.fd, self.cases = torch, fd, cases
        dev = torch.device(device)
        pdt = torch.uint8 if fd.cfg.bpc == 8 else torch.int16
        dims = aligned_dims(fd.cfg.width, fd.cfg.height)
        pics = lambda: [torch.zeros((h, w), dtype=pdt, device=dev) for (w, h) in dims]  # noqa: E731
        self.A, self.B, self.C, self.D = pics(), pics(), pics(), pics()
        ptrs = lambda P: [(t.data_ptr(), t.shape[1]) for t in P]  # noqa: E731
        self.recon = batch.DeviceFrame(fd, dev, dst_planes=self.A)
        self.lpf = lpf.DeviceLpf(cases.lpf, dev)
        self.lpf.frame = lpf.fill_frame(abi.LoopFilterFrame(), cases.lpf, ptrs(self.A), self.lpf.masks.data_ptr(),
                                        self.lpf.level.data_ptr())
        self.cdef = cdef.DeviceCdef(cases.cdef, dev)
        self.cdef.frame = cdef.fill_frame(abi.CdefFrame(), cases.cdef, ptrs(self.A), ptrs(self.B),
                                          self.cdef.idx.data_ptr(), self.cdef.noskip.data_ptr())
        self.lr = lr.DeviceLr(cases.lr, dev)
        self.lr.frame = lr.fill_frame(abi.LrFrame(), cases.lr, ptrs(self.B), ptrs(self.A), ptrs(self.C),
                                      [t.data_ptr() for t in self.lr.units])
        self.grain = grain.DeviceGrain(cases.grain, dev)
        self.grain.batch = grain.fill_batch(abi.FilmGrainBatch(), cases.grain, ptrs(self.C), ptrs(self.D),
                                            self.grain.scratch.data_ptr())

    def launch(self, stream=None):
        """Enqueue the whole chain on `stream`, in dav1d's order."""
        s = stream if stream is not None else self.torch.cuda.current_stream()
        self.recon.launch(s)
        self.lpf.launch(s)
        self.cdef.launch(s)
        self.lr.launch(s)
        self.grain.launch(s)

    def launch_per_row(self, stream=None, step=64):
        """The same chain with the post-filters interleaved per superblock
        row as a decoder runs them behind its flushes (round 5 row ranges,
        INTEGRATION.md 2d): deblock row k, then CDEF and LR of row k - 1 --
        CDEF reads two deblocked rows below its own, which row k's
        deblocking finishes, and LR's stripes of row k - 1 end 8 rows above
        its bottom -- then the last row's CDEF and LR, then grain."""
        s = stream if stream is not None else self.torch.cuda.current_stream()
        self.recon.launch(s)
        rows = list(range(0, self.fd.cfg.height, step))
        for k, y in enumerate(rows):
            self.lpf.launch(s, rows=(y, y + step))
            if k:
                self.cdef.launch(s, rows=(y - step, y))
                self.lr.launch(s, rows=(y - step, y))
        self.cdef.launch(s, rows=(rows[-1], rows[-1] + step))
        self.lr.launch(s, rows=(rows[-1], rows[-1] + step))
        self.grain.launch(s)

    def stage_host(self, P):
        out = []
        for p, t in enumerate(P):
            w, h = self.fd.plane_wh[p]
            a = t[:h, :w].cpu().numpy()
            out.append(a if self.fd.cfg.bpc == 8 else a.view(np.uint16))
        return out


def host_chain(fd, cases, oracle, threads=4):
    """The oracle walkers chained in the same order on host copies: returns
    the visible planes after each stage (recon, deblock, cdef, lr, grain)."""
    pdt = fd.cfg.pixel_dtype
    dims = aligned_dims(fd.cfg.width, fd.cfg.height)
    hf = oracle.HostFrame(fd)
    hf.run(threads=threads)
    A = []
    for p, (w, h) in enumerate(dims):
        a = np.zeros((h, w), pdt)
        vw, vh = fd.plane_wh[p]
        a[:vh, :vw] = hf.dst[p]
        A.append(a)
    vis = lambda P: [P[p][:fd.plane_wh[p][1], :fd.plane_wh[p][0]].copy() for p in range(3)]  # noqa: E731
    stages = [vis(A)]
    A = oracle.loopfilter_frame(dataclasses.replace(cases.lpf, planes=A))
    stages.append(vis(A))
    B = oracle.cdef_frame(dataclasses.replace(cases.cdef, planes=A))
    stages.append(vis(B))
    C = oracle.lr_frame(dataclasses.replace(cases.lr, ins=B, lpfs=A))
    stages.append(vis(C))
    D, _, _ = oracle.apply_grain(dataclasses.replace(cases.grain, planes=vis(C)))
    stages.append([np.asarray(d) for d in D])
    return stages
