"""Synthetic frame batches for the reconstruction hot path.

A frame is tiled into square prediction blocks by a seeded quadtree over
64x64 superblocks (luma area mix 8x8 25% / 16x16 35% / 32x32 25% / 64x64
15%); 4:2:0 chroma blocks follow at half size.  Blocks are inter (single-ref
put or compound 2x prep + avg, one of the 9 8-tap filter pairs, integer MV
uniform in +-64 px, 1/16-pel fraction uniform) or intra (one of the 14
intra_pred modes, per-transform-block edge arrays).  Every block is split
into transform units of one size <= 32x32 (rect included); each unit gets a
transform type valid for its size (the reference's 156-entry table) and
coefficients from a floating-point forward transform of uniform residuals
(the idea of tests/checkasm/itx.c:183-240), truncated to a DC-only (25%),
partial (50%) or full (25%) coefficient region.

Blocks are independent: intra edges come from an edge pool, not from
reconstructed neighbours.  The "mc" config is
config 2: inter only, prediction-only units (one per block, no residual).

Everything here is host-side numpy; nothing is timed.
"""
import dataclasses
import os
from dataclasses import dataclass, field

import numpy as np

from . import abi

Z_ANGLES = np.array([3, 6, 9, 14, 17, 20, 23, 26, 29, 32, 36, 39, 42, 45, 48, 51, 54,
                     58, 61, 64, 67, 70, 73, 76, 81, 84, 87], np.int32)

# leaf probability at each quadtree level, giving the 15/25/35/25 area mix
_LEVELS = [(64, 0.15), (32, 0.25 / 0.85), (16, 0.35 / 0.60), (8, 1.0)]

REF_PAD = 96   # reference planes carry this many padding pixels on every side

# picture bands of the unit sort (see make_frame); DAV1D_GPU_SORT_BANDS overrides (tuning)
SORT_BANDS = int(os.environ.get("DAV1D_GPU_SORT_BANDS", "16"))
# order inside (class, band, pred kind): "txtp" (transform type, then filter /
# mode), "block" (prediction block, so a block's units share a wave),
# "raster" (picture position), "txblk" (txtp, then block); tuning knob
SORT_MODE = os.environ.get("DAV1D_GPU_SORT_MODE", "txtp")

_SCALE = [4.0, 4.0 * 2 ** -0.5, 2.0, 2.0 * 2 ** -0.5, 1.0, 0.5 * 2 ** -0.5, 0.25,
          0.125 * 2 ** -0.5, 0.0625]


@dataclass
class FrameConfig:
    width: int = 3840
    height: int = 2160
    bpc: int = 8                  # 8 or 16 (ABI); 16 uses bitdepth_max
    bitdepth_max: int = 255
    # "full" (mc + ipred + itx, config 3), "mc" (put/avg only, one unit per
    # block, config 2), or a per-family frame for the bench breakdown:
    # "ipred" (every block intra / CfL, no residual) or "itx" (no prediction:
    # inv_txfm_add onto the picture, the reference's dst read + write)
    kind: str = "full"
    intra_frac: float = 0.30
    compound_frac: float = 0.50   # of inter blocks
    seed: int = 0x5EED0001
    tx64: bool = False            # allow 64-point transforms (64x64 luma blocks)
    cfl_frac: float = 0.50        # of intra blocks: chroma predicted with CfL (config 3)
    # "mc" frames: prediction-only blocks wider than this are cut into units of
    # this size (the prediction of a piece is the block's prediction there:
    # mc is pointwise and the filter bank follows the block size, bw4/bh4), so
    # a 64x64 block does not need the 64-point class group's long waves
    mc_split: int = int(os.environ.get("DAV1D_GPU_MC_SPLIT", "32"))   # env: tuning knob
    # integer MV range in luma pixels (+-); beyond REF_PAD - 8 the footprints
    # leave the padded reference planes: only the tile batch (which clamps,
    # emu_edge semantics) may then run the frame
    mv_range: int = 64
    # reference planes padded by replicating their edge pixels (what
    # emu_edge would read) instead of random pixels: then every footprint,
    # clamped or read from the padding, sees the same values
    edge_pad: bool = True
    # prediction only (no inv_txfm_add) for every kind, and units of at most
    # unit_split px per side cut from the prediction blocks instead of their
    # transform blocks (0: transform blocks): the same blocks cut two ways
    # must give the same picture (tests/test_cpu.py)
    no_residual: bool = False
    unit_split: int = 0
    # fraction of the 4x4 units with a residual whose transform is WHT_WHT
    # (lossless, src/itx_tmpl.c:166-185), with coefficients drawn over the
    # whole range the decoder's dequantisation allows (cf_max,
    # src/recon_tmpl.c:594); 0 leaves every other draw of the frame unchanged
    lossless: float = 0.0

    @property
    def ref_pad(self):
        return max(REF_PAD, self.mv_range + 32)

    @property
    def pixel_dtype(self):
        return np.uint8 if self.bpc == 8 else np.uint16

    @property
    def coef_dtype(self):
        return np.int16 if self.bpc == 8 else np.int32


@dataclass
class FrameData:
    cfg: FrameConfig
    units: np.ndarray
    class_start: np.ndarray
    coefs: np.ndarray
    edges: np.ndarray
    refs: list                    # [ref][plane] padded 2-D arrays
    plane_wh: list                # [(w, h)] per plane
    blk: np.ndarray = None        # prediction-block id of each unit (stats only)
    cfl_luma: np.ndarray = None   # luma plane CFL units read (synthetic "reconstructed" luma)
    dst_init: list = None         # starting picture planes ("itx" frames add onto them)
    aux: np.ndarray = None        # per-unit int32: aux_pool offset (INTER_MASK / PAL units)
    aux_pool: np.ndarray = None   # u8 pool: block masks, palette records
    class_warp: np.ndarray = None # WARP units at the end of each class range
    src_xy: np.ndarray = None     # [unit][ref][x|y]: integer source position of the unit's
                                  # top-left in the reference plane (visible coordinates)
    deferred: object = None       # clamp_units: a second batch to launch after this one
    stats: dict = field(default_factory=dict)

    @property
    def n_units(self):
        return len(self.units)

    def ref_origin_offset(self, plane):
        stride = self.refs[0][plane].shape[1]
        return self.cfg.ref_pad * stride + self.cfg.ref_pad


def _partition(rng, W, H):
    """Quadtree leaves (x, y, size) covering W x H (multiples of 8)."""
    ys, xs = np.meshgrid(np.arange(0, H, 64), np.arange(0, W, 64), indexing="ij")
    xs, ys = xs.ravel(), ys.ravel()
    out = []
    for s, p in _LEVELS:
        inside = (xs + s <= W) & (ys + s <= H)
        outside = (xs >= W) | (ys >= H)
        leaf = inside & (rng.random(len(xs)) < p)
        out.append((xs[leaf], ys[leaf], np.full(leaf.sum(), s)))
        split = ~outside & ~leaf
        if s == 8:
            break
        h = s // 2
        sx, sy = xs[split], ys[split]
        xs = np.concatenate([sx, sx + h, sx, sx + h])
        ys = np.concatenate([sy, sy, sy + h, sy + h])
    return (np.concatenate([o[0] for o in out]), np.concatenate([o[1] for o in out]),
            np.concatenate([o[2] for o in out]))


def _dct_mat(n):
    k = np.arange(n)[:, None]
    j = np.arange(n)[None, :]
    m = np.cos(np.pi * (2 * j + 1) * k / (2.0 * n))
    m[0] *= 2 ** -0.5
    return m


def _adst_mat(n):
    i = np.arange(n)[:, None]
    j = np.arange(n)[None, :]
    if n == 4:
        return np.sin(np.pi * (j + 1) * (2 * i + 1) / 9.0)
    return np.sin(np.pi * (2 * j + 1) * (2 * i + 1) / (4.0 * n))


def _fwd_mat(kind, n):
    if kind == 0:
        return _dct_mat(n)
    if kind == 3:
        return np.eye(n)
    return _adst_mat(n)


# {vertical, horizontal} 1-D kinds per TxfmType (0 dct, 1 adst, 2 flipadst, 3 identity)
_KV = [0, 1, 0, 1, 2, 0, 2, 1, 2, 3, 0, 3, 1, 3, 2, 3]
_KH = [0, 0, 1, 1, 0, 2, 2, 2, 1, 3, 3, 0, 3, 1, 3, 2]


def _tx_candidates(s, tx64=False):
    """(tw, th) transform sizes tiling an s x s block: sides in {s, s/2, s/4}
    within [4, 32] (or [4, 64] with tx64), aspect ratio at most 4 (all such
    pairs are reference transform sizes)."""
    top = 64 if tx64 else 32
    sides = [v for v in (s, s // 2, s // 4) if 4 <= v <= top]
    return [(a, b) for a in sides for b in sides if max(a, b) <= 4 * min(a, b)]


def make_residuals(rng, tx, tw, th, bdmax, coef_dtype):
    """Transform types (uniform over the reference's valid ones per size),
    stored coefficient regions (25% DC-only, 50% partial, 25% full) and
    coefficients from a seeded forward transform of uniform residuals
    (SURVEY 8(d) config 3).  Returns (txtp, nzw, nzh, coef_off, coefs)."""
    n = len(tx)
    txtp = np.zeros(n, np.int32)
    for t in range(abi.N_TX):
        sel = np.nonzero(tx == t)[0]
        if not len(sel):
            continue
        ok = [tp for tp in range(16) if abi.itx_supported(t, tp)]
        txtp[sel] = np.array(ok)[rng.integers(0, len(ok), len(sel))]
    eclass = rng.random(n)          # <.25 DC-only, <.75 partial, else full
    sw = np.minimum(tw, 32)
    sh = np.minimum(th, 32)
    nzw = np.where(eclass < 0.25, np.where(txtp == abi.DCT_DCT, 0, 1),
                   np.where(eclass < 0.75, 1 + (rng.random(n) * sw).astype(np.int32), sw))
    nzh = np.where(eclass < 0.25, np.where(txtp == abi.DCT_DCT, 0, 1),
                   np.where(eclass < 0.75, 1 + (rng.random(n) * sh).astype(np.int32), sh))
    ncoef = np.where(nzw == 0, 1, nzw * nzh)
    coef_off = np.concatenate([[0], np.cumsum(ncoef)[:-1]])
    coefs = np.zeros(int(ncoef.sum()), coef_dtype)
    lim = np.iinfo(np.int16)
    for t in range(abi.N_TX):
        w_, h_ = abi.TX_WH[t]
        for tp in range(16):
            sel = np.nonzero((tx == t) & (txtp == tp))[0]
            if not len(sel):
                continue
            res = rng.integers(-bdmax, bdmax + 1, size=(len(sel), h_, w_)).astype(np.float64)
            mh = _fwd_mat(_KH[tp], w_)
            mvv = _fwd_mat(_KV[tp], h_)
            sc = _SCALE[int(np.log2(w_ * h_)) - 4]
            c = np.einsum("yk,nkx->nyx", mvv, np.einsum("nyk,xk->nyx", res, mh)) * sc
            c = np.floor(c + 0.5)
            c = np.clip(c, lim.min, lim.max).astype(np.int64)
            for j, i in enumerate(sel):
                a, b, o = int(nzw[i]), int(nzh[i]), int(coef_off[i])
                if a == 0:
                    coefs[o] = c[j, 0, 0]
                else:
                    coefs[o:o + a * b] = c[j, :b, :a].T.ravel()
    return txtp, nzw, nzh, coef_off, coefs


def lossless_residuals(cfg, tx, txtp, nzw, nzh, coef_off, coefs):
    """WHT_WHT on a seeded cfg.lossless fraction of the 4x4 units, in place:
    the unit keeps its stored region (a DC-only unit becomes a 1x1 region, the
    same one coefficient), so the coefficient layout does not move; the
    values are uniform over [-(cf_max + 1), cf_max] (src/recon_tmpl.c:594,
    :659), extremes the row pass of the other types would clip."""
    lr = np.random.default_rng(cfg.seed ^ 0x1055)
    sel = np.nonzero((tx == 0) & (lr.random(len(tx)) < cfg.lossless))[0]
    bits = 8 if cfg.bpc == 8 else int(cfg.bitdepth_max).bit_length()
    cf_max = (127 << bits) | ((1 << bits) - 1)
    txtp[sel] = abi.WHT_WHT
    nzw[sel] = np.maximum(nzw[sel], 1)
    nzh[sel] = np.maximum(nzh[sel], 1)
    for i in sel:
        n, o = int(nzw[i]) * int(nzh[i]), int(coef_off[i])
        coefs[o:o + n] = lr.integers(-(cf_max + 1), cf_max + 1, n)


def _ext2_records(cfg, rng, units, pk, plane_u, ux, uy, tw, th, blk, bsz, lx, ly, ls, mv, ref_stride, planes):
    """aux records of the "ext2" kinds (include/dav1d_gpu.h, Dav1dGpuPredKind):

    * INTER_WMASK luma units / their chroma INTER_MASK units: the block's seg
      mask at 4:2:0 resolution, (s/2)^2 bytes, written by the luma units
      (w_mask_420) and read by the chroma ones (recon_tmpl.c:1854, :1900);
      p.inter.weight = mask_sign.
    * INTER_OBMC: the neighbour predictions of obmc() (recon_tmpl.c:1071-1133)
      with the reference's geometry: above (when the block is not on the top
      row; chroma only if bw + bh >= 16 plane pixels), up to min(log2 w4, 4)
      inter neighbours of random widths, lap size ow4 x (oh4 * 3 + 3) >> 2,
      blend_h over (v_mul * oh4 * 3) >> 2 rows with obmc_masks[v_mul * oh4];
      left (not on the left column), blend_v over (h_mul * ow4 * 3) >> 2
      columns with obmc_masks[h_mul * ow4]; each clipped to the unit.
    * INTER_SCALED: per reference a step dx, dy in [256, 2048] and a 1/1024
      phase; the unit's integer position and phase are the block's call's at
      its top-left (running sums, src/mc_tmpl.c:182-199).  Positions are kept
      inside the padded reference planes."""
    n = len(units)
    xr = np.random.default_rng(cfg.seed ^ 0xA2A2)
    aux = np.zeros(n, np.int32)
    chunks, off = [], 0

    def put(rec):
        nonlocal off
        rec = np.asarray(rec, np.uint8)
        pad = (-len(rec)) % 16
        at = off
        chunks.append(rec)
        if pad:
            chunks.append(np.zeros(pad, np.uint8))
        off += len(rec) + pad
        return at

    nb = len(lx)
    sign = xr.integers(0, 2, nb)
    # ---- w_mask: one 4:2:0 mask chunk per block
    wm_blk = np.unique(blk[pk == abi.PRED_INTER_WMASK])
    chunk_at = {}
    for b in wm_blk:
        cs = int(ls[b]) // 2
        chunk_at[b] = put(np.zeros(cs * cs, np.uint8))
    for i in np.nonzero((pk == abi.PRED_INTER_WMASK) | ((pk == abi.PRED_INTER_MASK) & np.isin(blk, wm_blk)))[0]:
        b = int(blk[i])
        s_ = int(bsz[i])
        bx0, by0 = (int(lx[b]) >> (1 if plane_u[i] else 0)), (int(ly[b]) >> (1 if plane_u[i] else 0))
        if plane_u[i] == 0:
            aux[i] = chunk_at[b] + ((int(uy[i]) - by0) >> 1) * (s_ >> 1) + ((int(ux[i]) - bx0) >> 1)
            units["weight"][i] = sign[b]
        else:
            aux[i] = chunk_at[b] + (int(uy[i]) - by0) * s_ + (int(ux[i]) - bx0)
    # ---- OBMC: block-level neighbour lists, then per unit the clipped entries
    nb_list = {}
    for b in np.unique(blk[pk == abi.PRED_INTER_OBMC]):
        bw4 = int(ls[b]) // 4
        lw = bw4.bit_length() - 1          # dav1d_block_dimensions[bs][2] (square blocks)
        ents = {"top": [], "left": []}
        if ly[b] > 0:
            x = 0
            while x < bw4 and len(ents["top"]) < min(lw, 4):
                step4 = int(np.clip(1 << int(xr.integers(1, 5)), 2, 16))
                if xr.random() < 0.8:
                    ents["top"].append((x, step4, xr.integers(-48 * 16, 48 * 16 + 1, 2), int(xr.integers(0, 10)),
                                        int(xr.integers(0, 2))))
                x += step4
        if lx[b] > 0:
            y = 0
            while y < bw4 and len(ents["left"]) < min(lw, 4):
                step4 = int(np.clip(1 << int(xr.integers(1, 5)), 2, 16))
                if xr.random() < 0.8:
                    ents["left"].append((y, step4, xr.integers(-48 * 16, 48 * 16 + 1, 2), int(xr.integers(0, 10)),
                                         int(xr.integers(0, 2))))
                y += step4
        nb_list[b] = ents
    for i in np.nonzero(pk == abi.PRED_INTER_OBMC)[0]:
        b, p = int(blk[i]), int(plane_u[i])
        sub = 1 if p else 0
        hm = vm = 4 >> sub                 # h_mul, v_mul (4:2:0)
        bw4 = int(ls[b]) // 4
        bx0, by0 = int(lx[b]) >> sub, int(ly[b]) >> sub
        ox, oy = int(ux[i]) - bx0, int(uy[i]) - by0   # the unit in the block
        w_, h_ = int(tw[i]), int(th[i])
        rs = int(ref_stride[p])
        rec = []
        regions = []
        if not p or bw4 * hm + bw4 * vm >= 16:
            for (x, step4, m_, f2d, r) in nb_list[b]["top"]:
                ow4, oh4 = min(step4, bw4), min(bw4, 16) >> 1
                regions.append((0, x * hm, x * hm + ow4 * hm, 0, (vm * oh4 * 3) >> 2, ow4, (oh4 * 3 + 3) >> 2,
                                vm * oh4, m_, f2d, r))
        for (y, step4, m_, f2d, r) in nb_list[b]["left"]:
            ow4, oh4 = min(bw4, 16) >> 1, min(step4, bw4)
            regions.append((1, 0, (hm * ow4 * 3) >> 2, y * vm, y * vm + oh4 * vm, ow4, oh4, hm * ow4, m_, f2d, r))
        for (dr, xa, xb, ya, yb, lw4, lh4, mbase, m_, f2d, r) in regions:
            x0, x1 = max(xa - ox, 0), min(xb - ox, w_)
            y0, y1 = max(ya - oy, 0), min(yb - oy, h_)
            if x0 >= x1 or y0 >= y1:
                continue
            mvx, mvy = (int(m_[0]) >> 1, int(m_[1]) >> 1) if p else (int(m_[0]), int(m_[1]))
            soff = (int(uy[i]) + (mvy >> 4)) * rs + int(ux[i]) + (mvx >> 4)
            e = np.zeros(16, np.uint8)
            e[0:4] = np.array([soff], "<i4").view(np.uint8)
            # lap call size in plane pixels / 4 (its filter banks)
            # lap size in 4-px units (2 px -> 0: both mean "<= 4", the 4-tap bank)
            e[4:16] = [mvx & 15, mvy & 15, f2d, r, x0, y0, x1, y1, (lw4 * hm) // 4, (lh4 * vm) // 4, dr,
                       mbase + (ox if dr else oy)]
            rec.append(e)
        hdr = np.zeros(16, np.uint8)
        hdr[0:4] = np.array([len(rec)], "<i4").view(np.uint8)
        aux[i] = put(np.concatenate([hdr] + rec))
    # ---- scaled references
    pad = cfg.ref_pad
    nref_b = xr.integers(1, 3, nb)
    wt_b = np.where(xr.random(nb) < 0.5, 0, xr.integers(1, 16, nb))
    steps = xr.integers(256, 2049, size=(nb, 2, 2))
    phase = xr.integers(0, 1024, size=(nb, 2, 2))
    for i in np.nonzero(pk == abi.PRED_INTER_SCALED)[0]:
        b, p = int(blk[i]), int(plane_u[i])
        sub = 1 if p else 0
        pw, ph = planes[p]
        s_ = int(bsz[i])
        bx0, by0 = int(lx[b]) >> sub, int(ly[b]) >> sub
        ox, oy = int(ux[i]) - bx0, int(uy[i]) - by0
        rs = int(ref_stride[p])
        recs = []
        for k in range(int(nref_b[b])):
            dx, dy = int(steps[b, k, 0]), int(steps[b, k, 1])
            mx0, my0 = int(phase[b, k, 0]), int(phase[b, k, 1])
            mvx, mvy = int(mv[b, k, 0]) >> 4 >> sub, int(mv[b, k, 1]) >> 4 >> sub
            # the block's integer origin, kept so its footprint stays inside
            # the padded plane: columns origin - 3 .. origin + ((s-1)dx+mx)>>10 + 4
            span_x, span_y = ((s_ - 1) * dx + mx0) >> 10, ((s_ - 1) * dy + my0) >> 10
            gx = int(np.clip(bx0 + mvx, -pad + 4, pw + pad - 6 - span_x))
            gy = int(np.clip(by0 + mvy, -pad + 4, ph + pad - 6 - span_y))
            px_, py_ = mx0 + ox * dx, my0 + oy * dy
            ex = gx + (px_ >> 10)
            ey = gy + (py_ >> 10)
            r = np.zeros(16, np.uint8)
            r[0:4] = np.array([ey * rs + ex], "<i4").view(np.uint8)
            r[4:12] = np.array([px_ & 1023, py_ & 1023, dx, dy], "<u2").view(np.uint8)
            recs.append(r)
        hdr = np.zeros(16, np.uint8)
        hdr[0:4] = np.array([len(recs)], "<i4").view(np.uint8)
        aux[i] = put(np.concatenate([hdr] + recs))
        units["weight"][i] = wt_b[b] if len(recs) == 2 else 0
    return aux, (np.concatenate(chunks) if chunks else np.zeros(16, np.uint8))


def make_frame(cfg: FrameConfig) -> FrameData:
    rng = np.random.default_rng(cfg.seed)
    W, H = cfg.width, cfg.height
    bdmax = cfg.bitdepth_max if cfg.bpc == 16 else 255
    planes = [(W, H), (W // 2, H // 2), (W // 2, H // 2)]

    # reference pictures: 2 x 3 planes, padded, uniform random pixels
    refs = []
    pad = cfg.ref_pad
    for _ in range(2):
        rp = []
        for (pw, ph) in planes:
            stride = (pw + 2 * pad + 63) // 64 * 64
            a = rng.integers(0, bdmax + 1, size=(ph + 2 * pad, stride), dtype=cfg.pixel_dtype)
            if cfg.edge_pad:
                a[:, :] = np.pad(a[pad:pad + ph, pad:pad + pw], ((pad, pad), (pad, stride - pw - pad)), mode="edge")
            rp.append(a)
        refs.append(rp)

    lx, ly, ls = _partition(rng, W, H)
    nb = len(lx)
    r = rng.random(nb)
    if cfg.kind == "mc":
        kind = np.where(rng.random(nb) < cfg.compound_frac, abi.PRED_INTER_AVG, abi.PRED_INTER)
    elif cfg.kind == "ext":
        # the batch tier's other prediction kinds, with residual as in
        # "full": put / avg / w_avg / mask compound and palette blocks
        rng.random(nb)   # keep the later draws aligned with "full"
        e = np.random.default_rng(cfg.seed ^ 0xE7E7).random(nb)
        kind = np.select([e < 0.18, e < 0.30, e < 0.44, e < 0.58, e < 0.74, e < 0.88],
                         [abi.PRED_INTER, abi.PRED_INTER_AVG, abi.PRED_INTER_WAVG, abi.PRED_INTER_MASK,
                          abi.PRED_PAL, abi.PRED_WARP], abi.PRED_INTER_INTRA)
    elif cfg.kind == "ext2":
        # the second launch's reference-semantics kinds: w_mask compound
        # (COMP_INTER_SEG), OBMC and scaled references, beside plain put
        rng.random(nb)
        e = np.random.default_rng(cfg.seed ^ 0xE2E2).random(nb)
        kind = np.select([e < 0.3, e < 0.6, e < 0.9], [abi.PRED_INTER_WMASK, abi.PRED_INTER_OBMC,
                                                       abi.PRED_INTER_SCALED], abi.PRED_INTER)
    elif cfg.kind in ("ipred", "itx"):
        rng.random(nb)   # keep the later draws aligned with "full"
        kind = np.full(nb, abi.PRED_INTRA if cfg.kind == "ipred" else abi.PRED_NONE)
    else:
        kind = np.where(r < cfg.intra_frac, abi.PRED_INTRA,
                        np.where(rng.random(nb) < cfg.compound_frac, abi.PRED_INTER_AVG,
                                 abi.PRED_INTER))
    filt = rng.integers(0, 9, nb)
    mv = rng.integers(-cfg.mv_range * 16, cfg.mv_range * 16 + 1, size=(nb, 2, 2))   # [block][ref][x|y], 1/16 px
    mode = rng.integers(0, 14, nb)
    zang = Z_ANGLES[rng.integers(0, 27, nb)]
    zflags = rng.integers(0, 4, nb) << 9
    fidx = rng.integers(0, 5, nb)
    z2mw = rng.integers(1, 65, nb)
    z2mh = rng.integers(1, 65, nb)
    # CfL (own stream): chroma of these intra blocks is one CFL unit per block
    crng = np.random.default_rng(cfg.seed ^ 0xCF1C)
    cfl_blk = (kind == abi.PRED_INTRA) & (crng.random(nb) < (cfg.cfl_frac if cfg.kind != "mc" else 0.0))
    cfl_alpha = crng.integers(1, 17, size=(nb, 2)) * np.where(crng.random((nb, 2)) < 0.5, -1, 1)
    cfl_dc = np.array([abi.DC_PRED, abi.LEFT_DC_PRED, abi.TOP_DC_PRED, abi.DC_128_PRED])[crng.integers(0, 4, nb)]

    rows = []   # per-unit python tuples assembled below (vectorised per block)
    unit_fields = {k: [] for k in ("plane", "x", "y", "tw", "th", "blk", "bs")}
    for plane in range(3):
        sub = 0 if plane == 0 else 1
        bx, by, bs = lx >> sub, ly >> sub, ls >> sub
        for b in range(nb):
            s = int(bs[b])
            if cfg.kind == "mc":
                tw = th = min(s, cfg.mc_split)
            elif cfg.unit_split:
                tw = th = min(s, cfg.unit_split)
            else:
                cands = _tx_candidates(s, cfg.tx64)
                if kind[b] == abi.PRED_WARP and plane == 0:   # warp units are whole 8x8s
                    cands = [c for c in cands if min(c) >= 8]
                if kind[b] in abi.SECOND_LAUNCH_KINDS:   # second launch: no 64-point class
                    cands = [c for c in cands if max(c) <= 32]
                tw, th = cands[(b * 7 + plane * 3 + int(rng.integers(0, 1 << 20))) % len(cands)]
                if plane > 0 and cfl_blk[b]:
                    tw = th = s   # CfL predicts the whole chroma block (<= 32x32)
            for oy in range(0, s, th):
                for ox in range(0, s, tw):
                    unit_fields["plane"].append(plane)
                    unit_fields["x"].append(int(bx[b]) + ox)
                    unit_fields["y"].append(int(by[b]) + oy)
                    unit_fields["tw"].append(tw)
                    unit_fields["th"].append(th)
                    unit_fields["blk"].append(b)
                    unit_fields["bs"].append(s)
    del rows
    plane_u = np.array(unit_fields["plane"], np.int32)
    ux = np.array(unit_fields["x"], np.int32)
    uy = np.array(unit_fields["y"], np.int32)
    tw = np.array(unit_fields["tw"], np.int32)
    th = np.array(unit_fields["th"], np.int32)
    blk = np.array(unit_fields["blk"], np.int32)
    bsz = np.array(unit_fields["bs"], np.int32)
    n = len(ux)
    tx = np.array([abi.TX_INDEX[(a, b)] for a, b in zip(tw, th)], np.int32)

    units = np.zeros(n, abi.UNIT_DTYPE)
    pw = np.array([planes[p][0] for p in range(3)])
    units["dst_off"] = uy * pw[plane_u] + ux
    units["tx"] = tx
    units["plane"] = plane_u
    pk = kind[blk].copy()
    pk[(pk == abi.PRED_WARP) & (plane_u > 0)] = abi.PRED_INTER   # chroma of warped blocks: translation
    # chroma of COMP_INTER_SEG blocks: mask_c on the luma's seg mask (recon_tmpl.c:1900)
    pk[(pk == abi.PRED_INTER_WMASK) & (plane_u > 0)] = abi.PRED_INTER_MASK
    cfl = (plane_u > 0) & cfl_blk[blk]
    pk[cfl] = abi.PRED_CFL
    units["pred"] = pk
    units["bw4"] = bsz // 4
    units["bh4"] = bsz // 4

    # inter parameters
    inter = np.isin(pk, abi.INTER_KINDS + (abi.PRED_INTER_INTRA, abi.PRED_INTER_WMASK, abi.PRED_INTER_OBMC,
                         abi.PRED_INTER_SCALED))
    ref_stride = np.array([refs[0][p].shape[1] for p in range(3)])
    src_xy = np.zeros((n, 2, 2), np.int32)
    for k in range(2):
        mvx = mv[blk, k, 0]
        mvy = mv[blk, k, 1]
        chroma = plane_u > 0
        mvx = np.where(chroma, mvx >> 1, mvx)
        mvy = np.where(chroma, mvy >> 1, mvy)
        sx = ux + (mvx >> 4)
        sy = uy + (mvy >> 4)
        units[f"src_off{k}"] = np.where(inter, sy * ref_stride[plane_u] + sx, 0)
        src_xy[:, k, 0] = np.where(inter, sx, 0)
        src_xy[:, k, 1] = np.where(inter, sy, 0)
        units[f"mx{k}"] = np.where(inter, mvx & 15, 0)
        units[f"my{k}"] = np.where(inter, mvy & 15, 0)
        units[f"ref{k}"] = k
    units["filter2d"] = np.where(inter, filt[blk], 0)
    aux = aux_pool = None
    if cfg.kind == "ext":
        xr = np.random.default_rng(cfg.seed ^ 0xA0A0)
        # jnt_comp weight per prediction block (f->jnt_weights, src/recon_tmpl.c:1873)
        units["weight"] = np.where(pk == abi.PRED_INTER_WAVG, xr.integers(1, 16, nb)[blk], 0)
        aux = np.zeros(n, np.int32)
        chunks, off = [], 0
        # INTER_MASK: one mask 0..64 per prediction block (per plane), row
        # stride = the block width; a unit points at its top-left inside it
        mb = np.nonzero((pk == abi.PRED_INTER_MASK) | (pk == abi.PRED_INTER_INTRA))[0]
        mask_at = np.zeros(n, np.int64)   # INTER_INTRA: the mask offset goes into its record
        bkey = blk * 3 + plane_u
        first_of = {}
        for i in mb:
            k = int(bkey[i])
            if k not in first_of:
                s_ = int(bsz[i])
                first_of[k] = off
                chunks.append(xr.integers(0, 65, s_ * s_, dtype=np.uint8))
                off += (s_ * s_ + 15) // 16 * 16
                chunks.append(np.zeros((s_ * s_ + 15) // 16 * 16 - s_ * s_, np.uint8))
            bx0 = (int(ux[i]) // int(bsz[i])) * int(bsz[i])   # blocks are aligned to their size
            by0 = (int(uy[i]) // int(bsz[i])) * int(bsz[i])
            mask_at[i] = first_of[k] + (int(uy[i]) - by0) * int(bsz[i]) + (int(ux[i]) - bx0)
            if pk[i] == abi.PRED_INTER_MASK:
                aux[i] = mask_at[i]
        # PAL: per unit a 16-B record of 8 entries, then the packed index map
        pb = np.nonzero(pk == abi.PRED_PAL)[0]
        bpp_ = 1 if cfg.bpc == 8 else 2
        for i in pb:
            w_, h_ = int(tw[i]), int(th[i])
            pal = xr.integers(0, bdmax + 1, 8).astype(cfg.pixel_dtype).view(np.uint8)
            rec = np.zeros(16 + (w_ * h_ // 2 + 15) // 16 * 16, np.uint8)
            rec[:8 * bpp_] = pal
            idx = xr.integers(0, 8, size=(h_, w_))
            rec[16:16 + w_ * h_ // 2] = (idx[:, 0::2] | (idx[:, 1::2] << 4)).astype(np.uint8).ravel()
            aux[i] = off
            chunks.append(rec)
            off += len(rec)
        # WARP: per unit abcd[4] (int16), 8 pad bytes, then per 8x8 of the
        # unit int16 x, y (its source position), int16 mx >> 6, int16 my >> 6
        # (warp_affine, src/recon_tmpl.c:1134-1193, with shear parameters
        # within +-1024)
        wb = np.nonzero(pk == abi.PRED_WARP)[0]
        babcd = xr.integers(-1024, 1025, size=(nb, 4)).astype(np.int16)
        for i in wb:
            w_, h_ = int(tw[i]), int(th[i])
            a_ = babcd[blk[i]]
            rec = np.zeros(16 + 8 * (w_ // 8) * (h_ // 8), np.uint8)
            rec[:8] = a_.view(np.uint8)
            mvx, mvy = int(mv[blk[i], 0, 0]) >> 4, int(mv[blk[i], 0, 1]) >> 4
            sub = np.zeros((h_ // 8) * (w_ // 8), dtype=[("x", "<i2"), ("y", "<i2"), ("mx", "<i2"), ("my", "<i2")])
            k_ = 0
            for sy in range(h_ // 8):
                for sx in range(w_ // 8):
                    x_ = int(ux[i]) + 8 * sx + mvx + int(xr.integers(-2, 3))
                    y_ = int(uy[i]) + 8 * sy + mvy + int(xr.integers(-2, 3))
                    sub["x"][k_], sub["y"][k_] = x_, y_
                    mx_ = (int(xr.integers(0, 65536)) - 4 * int(a_[0]) - 7 * int(a_[1])) & ~63
                    my_ = (int(xr.integers(0, 65536)) - 4 * int(a_[2]) - 4 * int(a_[3])) & ~63
                    sub["mx"][k_], sub["my"][k_] = mx_ >> 6, my_ >> 6
                    k_ += 1
            rec[16:] = sub.view(np.uint8)
            aux[i] = off
            chunks.append(rec)
            off += len(rec) + (-len(rec)) % 16
            chunks.append(np.zeros((-len(rec)) % 16, np.uint8))

    if cfg.kind == "ext2":
        aux, aux_pool = _ext2_records(cfg, rng, units, pk, plane_u, ux, uy, tw, th, blk, bsz, lx, ly, ls, mv,
                                      ref_stride, planes)

    # intra parameters
    intra = pk == abi.PRED_INTRA
    m = mode[blk]
    ang = np.where((m >= abi.Z1_PRED) & (m <= abi.Z3_PRED),
                   (90 * (m - abi.Z1_PRED) + zang[blk]) | zflags[blk],
                   np.where(m == abi.FILTER_PRED, fidx[blk], 0))
    # the intra fields share bytes with the inter ones (a C union): write
    # them only where the unit is intra
    iiu = pk == abi.PRED_INTER_INTRA
    edge_len = np.where(intra | cfl | iiu, 2 * th + 2 * tw + 1, 0)
    edge_start = np.concatenate([[0], np.cumsum(edge_len)[:-1]])
    if cfg.kind == "ext":
        # INTER_INTRA records: edge_off, mode (the inter-intra modes DC / V /
        # H / SMOOTH, src/recon_tmpl.c:1550), angle 0, mask offset
        ii_modes = np.array([abi.DC_PRED, abi.VERT_PRED, abi.HOR_PRED, abi.SMOOTH_PRED])
        bmode = ii_modes[xr.integers(0, 4, nb)]
        for i in np.nonzero(iiu)[0]:
            rec = np.zeros(16, np.uint8)
            rec[0:4] = np.array([edge_start[i] + 2 * th[i]], "<i4").view(np.uint8)
            rec[4] = bmode[blk[i]]
            rec[8:12] = np.array([mask_at[i]], "<i4").view(np.uint8)
            aux[i] = off
            chunks.append(rec)
            off += 16
        aux_pool = np.concatenate(chunks) if chunks else np.zeros(16, np.uint8)
    iu = units[intra]
    iu["src_off1"] = 0
    iu["filter2d"] = 0
    iu["ref0"] = 0
    iu["ref1"] = 0
    iu["edge_off"] = (edge_start + 2 * th)[intra]
    iu["mode"] = m[intra]
    iu["angle"] = ang[intra]
    z2 = m[intra] == abi.Z2_PRED
    iu["max_w"] = np.where(z2, z2mw[blk][intra], 0)
    iu["max_h"] = np.where(z2, z2mh[blk][intra], 0)
    units[intra] = iu
    # CfL parameters (union view "cfl"): DC source, alpha per chroma plane,
    # co-located luma offset in the cfl_luma plane (4:2:0, no edge padding)
    cu = units[cfl]
    cu["src_off1"] = 0
    cu["filter2d"] = 0
    cu["ref0"] = 0
    cu["ref1"] = 0
    cu["max_w"] = 0
    cu["max_h"] = 0
    cu["edge_off"] = (edge_start + 2 * th)[cfl]
    cu["mode"] = cfl_dc[blk][cfl]
    cu["cfl_alpha"] = cfl_alpha[blk[cfl], plane_u[cfl] - 1]
    cu["cfl_pad_wh"] = 0
    luma_stride = (W + 63) // 64 * 64
    cu["cfl_luma_off"] = (2 * uy[cfl]) * luma_stride + 2 * ux[cfl]
    units[cfl] = cu
    cfl_luma = crng.integers(0, bdmax + 1, size=(H, luma_stride), dtype=cfg.pixel_dtype)
    m = np.where(cfl, cfl_dc[blk], m)
    sort_minor = np.where(inter, filt[blk], 16 + np.where(pk == abi.PRED_PAL, 0, m))
    edges = rng.integers(0, bdmax + 1, size=max(int(edge_len.sum()), 1), dtype=cfg.pixel_dtype)

    # transform types, coefficient regions and coefficients
    if cfg.kind in ("mc", "ipred") or cfg.no_residual:
        units["txtp"] = abi.NO_RESIDUAL
        coefs = np.zeros(1, cfg.coef_dtype)
    else:
        txtp, nzw, nzh, coef_off, coefs = make_residuals(rng, tx, tw, th, bdmax, cfg.coef_dtype)
        if cfg.lossless > 0:
            lossless_residuals(cfg, tx, txtp, nzw, nzh, coef_off, coefs)
        units["txtp"] = txtp
        units["nzw"] = nzw
        units["nzh"] = nzh
        units["coef_off"] = coef_off

    # sort by (class, picture band, pred kind, then transform type / filter
    # for inter and mode / transform type for intra).  The kernel cuts each
    # class into 16 equal segments scheduled together (spatial locality of
    # the writes); inside a band, waves then see one prediction kind and one
    # transform type, so the per-unit branches (1-D transform kind, intra
    # mode) do not diverge.  Order inside a class is free for correctness.
    ph = np.array([planes[p][1] for p in range(3)])
    band = (uy * SORT_BANDS) // ph[plane_u]
    tt = units["txtp"].astype(np.int64)
    minor = np.where(inter, tt * 16 + sort_minor, sort_minor * 256 + tt)
    pos = uy.astype(np.int64) * W + ux
    if SORT_MODE == "block":
        keys = (pos, blk, units["pred"], band, units["tx"])
    elif SORT_MODE == "raster":
        keys = (ux, uy, units["pred"], band, units["tx"])
    elif SORT_MODE == "txblk":
        keys = (pos, blk, minor, units["pred"], band, units["tx"])
    else:
        keys = (minor, units["pred"], band, units["tx"])
    # WARP units go last inside their class (the batch's class_warp ranges,
    # run by the warp launch)
    is_warp = np.isin(units["pred"], abi.SECOND_LAUNCH_KINDS)
    order = np.lexsort(keys[:-1] + (is_warp, units["tx"]))
    units = units[order]
    counts = np.bincount(units["tx"], minlength=abi.N_TX)
    class_start = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    class_warp = np.bincount(units["tx"][np.isin(units["pred"], abi.SECOND_LAUNCH_KINDS)],
                             minlength=abi.N_TX).astype(np.int32)

    dst_init = None
    if cfg.kind == "itx":   # a picture for the residual to land on (own stream)
        drng = np.random.default_rng(cfg.seed ^ 0x1D57)
        dst_init = [drng.integers(0, bdmax + 1, size=(ph_, pw_), dtype=cfg.pixel_dtype) for (pw_, ph_) in planes]
    fd = FrameData(cfg=cfg, units=units, class_start=class_start, coefs=coefs, edges=edges,
                   refs=refs, plane_wh=planes, blk=(blk * 3 + plane_u)[order], cfl_luma=cfl_luma,
                   dst_init=dst_init, aux=None if aux is None else aux[order], aux_pool=aux_pool,
                   class_warp=class_warp, src_xy=src_xy[order])
    fd.stats = algorithmic_bytes(fd)
    return fd


def algorithmic_bytes(fd: FrameData):
    """Bytes the reconstruction must move per frame: the
    reference footprint each mc call reads, edge arrays, stored
    coefficients, one write of every output pixel (plus the picture read of
    residual-only units and the aux records).  The batch's own 32-B unit
    descriptors are the builder's format, not algorithmic work: reported as
    desc_bytes, outside total_bytes."""
    u = fd.units
    bpp = 1 if fd.cfg.bpc == 8 else 2
    cb = 2 if fd.cfg.bpc == 8 else 4
    w = np.array([abi.TX_WH[t][0] for t in u["tx"]])
    h = np.array([abi.TX_WH[t][1] for t in u["tx"]])
    bw, bh = u["bw4"].astype(np.int64) * 4, u["bh4"].astype(np.int64) * 4
    # the reference reads each prediction block's footprint once per mc call
    # (src/recon_tmpl.c:957-1059): count it per block, not per transform unit
    inter = np.isin(u["pred"], abi.INTER_KINDS + (abi.PRED_INTER_INTRA,))
    _, first = np.unique(np.where(inter, fd.blk, -1), return_index=True)
    first = first[inter[first]]
    src = np.zeros(len(u), np.int64)
    for k in range(2):
        use = np.isin(u["pred"], (abi.PRED_INTER, abi.PRED_INTER_INTRA, abi.PRED_INTER_OBMC,
                                  abi.PRED_INTER_SCALED)) if k == 0 else np.zeros(len(u), bool)
        use = use | np.isin(u["pred"], abi.COMPOUND_KINDS + (abi.PRED_INTER_WMASK,))
        mx, my = u[f"mx{k}"], u[f"my{k}"]
        fh = np.where(mx > 0, np.where(bw > 4, 7, 3), 0)
        fv = np.where(my > 0, np.where(bh > 4, 7, 3), 0)
        src[first] += np.where(use, (bw + fh) * (bh + fv), 0)[first]
    intra = u["pred"] == abi.PRED_INTRA
    cfl = u["pred"] == abi.PRED_CFL
    nopred = u["pred"] == abi.PRED_NONE
    edge = np.where(intra | cfl, 2 * w + 2 * h + 1, 0)
    src = src + np.where(cfl, 4 * w * h, 0)   # co-located 4:2:0 luma the cfl_ac reads
    # mask compound reads its mask (u8 per pixel); palette units their
    # entries and packed index map
    aux_bytes = int((w * h)[u["pred"] == abi.PRED_INTER_MASK].sum())
    pal = u["pred"] == abi.PRED_PAL
    aux_bytes += int((w * h // 2)[pal].sum()) + int(pal.sum()) * 8 * bpp
    ii = u["pred"] == abi.PRED_INTER_INTRA   # + its edge array, mask and 16-B record
    edge = edge + np.where(ii, 2 * w + 2 * h + 1, 0)
    aux_bytes += int((w * h + 16)[ii].sum())
    warp = u["pred"] == abi.PRED_WARP   # warp8x8: a 15x15 footprint per 8x8 + its parameters
    src = src + np.where(warp, (w // 8) * (h // 8) * 225, 0)
    aux_bytes += int(((w // 8) * (h // 8) * 8 + 16)[warp].sum())
    ncoef = np.where(u["txtp"] == abi.NO_RESIDUAL, 0, np.where(u["nzw"] == 0, 1,
                     u["nzw"].astype(np.int64) * u["nzh"]))
    out_px = int((w * h).sum())
    # PRED_NONE: inv_txfm_add reads the picture it adds to (dst read + write)
    dst_read = int((w * h)[nopred].sum()) * bpp
    return {
        "units": int(len(u)),
        "ref_bytes": int(src.sum()) * bpp,
        "edge_bytes": int(edge.sum()) * bpp,
        "coef_bytes": int(ncoef.sum()) * cb,
        "dst_bytes": out_px * bpp,
        "dst_read_bytes": dst_read,
        "aux_bytes": aux_bytes,
        "desc_bytes": int(len(u)) * 32,
        "pixels": out_px,
        "total_bytes": int(src.sum()) * bpp + int(edge.sum()) * bpp + int(ncoef.sum()) * cb
                       + out_px * bpp + dst_read + aux_bytes,
        "n_intra": int(intra.sum()),
        "n_cfl": int(cfl.sum()),
        "n_inter": int(inter.sum()),
        "n_pal": int(pal.sum()),
        "n_warp": int(warp.sum()),
        "n_inter_intra": int(ii.sum()),
        "n_nopred": int(nopred.sum()),
    }


def _decode_off(off, rs, pad):
    """(x, y) of a padded-plane offset y * rs + x (x in [-pad, rs - pad))."""
    off = np.asarray(off, np.int64)
    y = (off + pad) // rs
    return off - y * rs, y


def _xy16(x, y):
    return ((np.asarray(x, np.int64) & 0xffff) | ((np.asarray(y, np.int64) & 0xffff) << 16)).astype(np.uint32).view(np.int32)


def clamp_units(fd: FrameData):
    """The frame for exact-size (unpadded) reference planes, as a decoder
    with dav1d's own pictures would hand it to the unit batch: every inter
    unit's footprint is tested against its reference plane the way
    recon_tmpl.c's mc() decides emu_edge (src/recon_tmpl.c:986-999), here with
    the unit batch's load margins (the rectangle -3 / +4 pixels, plus the 3
    bytes before and 5 after each row its aligned loads touch).  A unit
    whose footprint stays inside reads the plane with its src_off
    re-expressed in the exact plane's stride; a unit whose footprint leaves
    it gets DGPU_MX_CLAMP on that reference with src_off = x | y << 16 and
    moves to the end of its class range (the class_warp sub-range of the
    second launch, which clamps every footprint pixel).

    Round 6: the launch-ahead kinds clamp too, each of them
    flagged whatever its footprint (they already run in the second launch,
    and a clamped read of an inside pixel is that pixel):
      * INTER_WMASK / INTER_OBMC / INTER_SCALED / INTER_INTRA: DGPU_MX_CLAMP
        in mx[k] and src_off[k] = x | y << 16, as above;
      * OBMC lap records (aux_pool): DGPU_MX_CLAMP in the lap's mx byte and
        its source offset as x | y << 16 (src/recon_tmpl.c:1071-1133);
      * INTER_SCALED records: bit 15 of the x phase and the integer origin as
        x | y << 16 (:1036-1046);
      * WARP: DGPU_MX_CLAMP in mx[0] and src_off[0] = 0, the per-8x8 source
        positions then being the plane's own (:1168-1177).
    Returns (frame, exact reference planes [ref][plane])."""
    u = fd.units.copy()
    pad = fd.cfg.ref_pad
    exact = [[np.ascontiguousarray(a[pad:pad + h, pad:pad + w]) for a, (w, h) in zip(rp, fd.plane_wh)]
             for rp in fd.refs]
    for (w, h) in fd.plane_wh:
        assert (w * np.dtype(fd.cfg.pixel_dtype).itemsize) % 4 == 0, "reference rows are read as aligned dwords"
    tw = np.array([abi.TX_WH[t][0] for t in u["tx"]])
    th = np.array([abi.TX_WH[t][1] for t in u["tx"]])
    pw = np.array([wh[0] for wh in fd.plane_wh])[u["plane"]]
    ph = np.array([wh[1] for wh in fd.plane_wh])[u["plane"]]
    comp = np.isin(u["pred"], (abi.PRED_INTER_AVG, abi.PRED_INTER_WAVG, abi.PRED_INTER_MASK))
    inter = np.isin(u["pred"], abi.INTER_KINDS)
    clamp_any = np.zeros(len(u), bool)
    for k in range(2):
        used = inter & (comp if k else True)
        x = fd.src_xy[:, k, 0].astype(np.int64)
        y = fd.src_xy[:, k, 1].astype(np.int64)
        inside = (x - 6 >= 0) & (x + tw + 12 <= pw) & (y - 3 >= 0) & (y + th + 4 <= ph - 1)
        cl = used & ~inside
        clamp_any |= cl
        off = np.where(cl, (x & 0xffff) | ((y & 0xffff) << 16), (y * pw + x) & 0xffffffff)
        u[f"src_off{k}"] = np.where(used, off.astype(np.uint32).view(np.int32), u[f"src_off{k}"])
        u[f"mx{k}"] = np.where(cl, u[f"mx{k}"] | 0x80, u[f"mx{k}"])
    # the launch-ahead kinds, every one flagged
    aux_pool = None if fd.aux_pool is None else fd.aux_pool.copy()
    rs = np.array([fd.refs[0][p].shape[1] for p in range(3)])
    ext = np.isin(u["pred"], (abi.PRED_INTER_WMASK, abi.PRED_INTER_OBMC, abi.PRED_INTER_SCALED,
                              abi.PRED_INTER_INTRA))
    for k in range(2):
        used = ext & ((u["pred"] == abi.PRED_INTER_WMASK) if k else True)
        xy = _xy16(fd.src_xy[:, k, 0], fd.src_xy[:, k, 1])
        u[f"src_off{k}"] = np.where(used, xy, u[f"src_off{k}"])
        u[f"mx{k}"] = np.where(used, u[f"mx{k}"] | 0x80, u[f"mx{k}"])
    clamp_any |= ext
    warp = u["pred"] == abi.PRED_WARP
    u["src_off0"] = np.where(warp, 0, u["src_off0"])
    u["mx0"] = np.where(warp, u["mx0"] | 0x80, u["mx0"])
    clamp_any |= warp
    if aux_pool is not None:
        ap32 = aux_pool.view(np.int32)
        for i in np.nonzero(u["pred"] == abi.PRED_INTER_OBMC)[0]:
            o = int(fd.aux[i])
            n = int(ap32[o // 4])
            for e in range(n):
                b = o + 16 + 16 * e
                x, y = _decode_off(ap32[b // 4], rs[u["plane"][i]], pad)
                ap32[b // 4] = _xy16(x, y)
                aux_pool[b + 4] |= 0x80
        for i in np.nonzero(u["pred"] == abi.PRED_INTER_SCALED)[0]:
            o = int(fd.aux[i])
            n = int(ap32[o // 4]) & 3
            for e in range(n):
                b = o + 16 + 16 * e
                x, y = _decode_off(ap32[b // 4], rs[u["plane"][i]], pad)
                ap32[b // 4] = _xy16(x, y)
                aux_pool[b + 5] |= 0x80   # bit 15 of the u16 x phase
    # A clamped INTER_MASK unit on the seg mask an INTER_WMASK unit of this
    # batch writes (COMPOUND_SEG chroma, src/recon_tmpl.c:1900) would run in
    # the same launch as its writer: it goes into a second batch, launched
    # after this one (out.deferred), as a decoder's next flush would run it
    dep = np.zeros(len(u), bool)
    if fd.blk is not None:
        wm_blk = np.unique(fd.blk[u["pred"] == abi.PRED_INTER_WMASK] // 3)
        dep = (u["pred"] == abi.PRED_INTER_MASK) & np.isin(fd.blk // 3, wm_blk) & clamp_any

    def build(sel):
        idx = np.nonzero(sel)[0]
        order = idx[np.lexsort((idx, clamp_any[idx], u["tx"][idx]))]
        uu = u[order]
        counts = np.bincount(uu["tx"], minlength=abi.N_TX)
        cs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
        cw = np.bincount(uu["tx"][clamp_any[order]], minlength=abi.N_TX).astype(np.int32)
        f = dataclasses.replace(fd, units=uu, class_start=cs, class_warp=cw, refs=None, aux_pool=aux_pool,
                                blk=None if fd.blk is None else fd.blk[order],
                                aux=None if fd.aux is None else fd.aux[order],
                                src_xy=None if fd.src_xy is None else fd.src_xy[order])
        f.stats = dict(fd.stats, clamped_units=int(clamp_any[order].sum()))
        return f

    # clamped units last inside their class (stable), the class_warp sub-range
    out = build(~dep)
    out.deferred = build(dep) if dep.any() else None
    return out, exact


def _class_sorted(units, keys_minor, planes, blk=None):
    """units sorted as make_frame sorts a batch: (class, picture band, pred
    kind, minor); returns (units, class_start, blk)."""
    pw = np.array([p[0] for p in planes])
    ph = np.array([p[1] for p in planes])
    pl = units["plane"].astype(np.int64)
    uy = units["dst_off"].astype(np.int64) // pw[pl]
    band = (uy * SORT_BANDS) // ph[pl]
    order = np.lexsort((keys_minor, units["pred"], band, units["tx"]))
    units = units[order]
    counts = np.bincount(units["tx"], minlength=abi.N_TX)
    class_start = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    return units, class_start, (None if blk is None else blk[order])


def split_frame(fd: FrameData, piece: int = 32):
    """The two-pass form of a frame: the reference's own
    order of work, mc() once per prediction block and reference
    (src/recon_tmpl.c:957-1060, compound :1845-1866) writing the block's
    prediction into the picture, then inv_txfm_add of each transform block
    adding its residual to what is there (src/itx_tmpl.c:40-100, the
    `dst` read + clip of every entry).

    Returns (pred_fd, res_fd), both run by the unchanged unit batch on the
    same picture, pred_fd first:
      * pred_fd: one prediction-only unit (txtp NO_RESIDUAL) per inter block
        and plane, blocks wider than `piece` cut into piece x piece units
        (mc is pointwise in the block call and the filter bank follows the
        block size carried in bw4 / bh4, as for the "mc" frames); sorted by
        (class, band, kind, filter), so a wave runs one block shape and
        filter and each footprint row is read once per block, not once per
        transform unit;
      * res_fd: the intra / CfL units unchanged (prediction + residual, they
        do not share footprints) and every inter transform unit with a
        residual as PRED_NONE (residual onto the predicted picture).
    pred + residual then clip is the fused kernel's arithmetic and the
    reference's, so the picture is bit-identical (tests/test_gpu_batch.py).
    Kinds whose prediction needs per-unit block data (mask, palette, warp,
    the second launch's) are refused."""
    u = fd.units
    ok = (abi.PRED_INTER, abi.PRED_INTER_AVG, abi.PRED_INTER_WAVG, abi.PRED_INTRA, abi.PRED_CFL, abi.PRED_NONE)
    if not np.isin(u["pred"], ok).all():
        raise ValueError("split_frame: only put / avg / w_avg inter, intra, CfL and residual-only units")
    planes = fd.plane_wh
    pw = np.array([p[0] for p in planes])
    pl = u["plane"].astype(np.int64)
    ux = u["dst_off"].astype(np.int64) % pw[pl]
    uy = u["dst_off"].astype(np.int64) // pw[pl]
    inter = np.isin(u["pred"], (abi.PRED_INTER, abi.PRED_INTER_AVG, abi.PRED_INTER_WAVG))
    s = u["bw4"].astype(np.int64) * 4
    if inter.any() and not np.array_equal(u["bw4"][inter], u["bh4"][inter]):
        raise ValueError("split_frame: square prediction blocks only")
    bx0, by0 = ux // np.maximum(s, 1) * s, uy // np.maximum(s, 1) * s
    key = (pl * (1 << 40)) + by0 * (1 << 20) + bx0
    idx = np.nonzero(inter)[0]
    _, first = np.unique(key[idx], return_index=True)
    heads = idx[first]
    ref_stride = np.array([fd.refs[0][p].shape[1] for p in range(3)])
    # prediction pieces
    rows = []
    for i in heads:
        bs = int(s[i])
        t = min(bs, piece)
        dx, dy = int(ux[i] - bx0[i]), int(uy[i] - by0[i])
        for oy in range(0, bs, t):
            for ox in range(0, bs, t):
                rows.append((i, ox - dx, oy - dy, t))
    src = np.array([r[0] for r in rows], np.int64)
    ox = np.array([r[1] for r in rows], np.int64)
    oy = np.array([r[2] for r in rows], np.int64)
    tsz = np.array([r[3] for r in rows], np.int64)
    pu = u[src].copy()
    pl_p = pl[src]
    pu["dst_off"] = (uy[src] + oy) * pw[pl_p] + ux[src] + ox
    pu["tx"] = np.array([abi.TX_INDEX[(int(a), int(a))] for a in tsz], np.uint8)
    rs = ref_stride[pl_p]
    comp = pu["pred"] != abi.PRED_INTER
    for k in range(2):
        use = np.ones(len(pu), bool) if k == 0 else comp
        so = pu[f"src_off{k}"].astype(np.int64) + oy * rs + ox
        pu[f"src_off{k}"] = np.where(use, so, pu[f"src_off{k}"]).astype(np.int32)
    pu["txtp"] = abi.NO_RESIDUAL
    pu["nzw"] = 0
    pu["nzh"] = 0
    pu["coef_off"] = 0
    pblk = None if fd.blk is None else fd.blk[src]
    pu, pcs, pblk = _class_sorted(pu, pu["filter2d"].astype(np.int64), planes, pblk)
    pred_fd = dataclasses.replace(fd, units=pu, class_start=pcs, blk=pblk, aux=None,
                                  class_warp=np.zeros(abi.N_TX, np.int32), src_xy=None)
    # residual pass: intra / CfL / residual-only as they are, inter units with
    # a residual as PRED_NONE
    keep = ~inter | (u["txtp"] != abi.NO_RESIDUAL)
    ru = u[keep].copy()
    rin = inter[keep]
    ru["pred"] = np.where(rin, abi.PRED_NONE, ru["pred"])
    for f in ("src_off0", "src_off1", "mx0", "mx1", "my0", "my1", "filter2d", "weight"):
        ru[f] = np.where(rin, 0, ru[f])
    # minor key: the transform type for the residual-only units, the original
    # rank (already (filter / mode, type) ordered) for the others
    minor = np.where(ru["pred"] == abi.PRED_NONE, ru["txtp"].astype(np.int64), np.arange(len(ru)) + 256)
    rblk = None if fd.blk is None else fd.blk[keep]
    ru, rcs, rblk = _class_sorted(ru, minor, planes, rblk)
    res_fd = dataclasses.replace(fd, units=ru, class_start=rcs, blk=rblk, aux=None,
                                 class_warp=np.zeros(abi.N_TX, np.int32), src_xy=None)
    pred_fd.stats = algorithmic_bytes(pred_fd)
    res_fd.stats = algorithmic_bytes(res_fd)
    return pred_fd, res_fd
