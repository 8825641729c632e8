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
        cfl = pl > 0 and max(tw, th) <= 8 and rng.random() < 0.3   # CfL: DC source only
        if cfl:
            mode, angle, fl = abi.DC_PRED, 0, fl & (abi.IE_HAVE_LEFT | abi.IE_HAVE_TOP | abi.IE_TOP_SB_EDGE)
            units[u]["cfl_alpha"] = int(rng.integers(1, 17))
            units[u]["cfl_pad_wh"] = 0x21
        units[u]["plane"], units[u]["tx"] = pl, tx
        units[u]["pred"] = abi.PRED_CFL if cfl else abi.PRED_INTRA
        units[u]["txtp"] = abi.NO_RESIDUAL
        units[u]["edge_off"] = off + 8 * th
        if not cfl:
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


# ---------------------------------------------------------------- wavefront
# Host mirror of the function's mode remap and edge needs (the scheduler must
# know which neighbours a record reads): av1_mode_to_angle_map,
# av1_mode_conv and av1_intra_prediction_edges, src/ipred_prepare_tmpl.c:38-75.
_DIR_ANGLE = (90, 180, 45, 135, 113, 157, 203, 67)
_NEED_L, _NEED_T, _NEED_TL, _NEED_TR, _NEED_BL = 1, 2, 4, 8, 16
_NEEDS = (3, 2, 1, 1, 2, 0, 14, 7, 21, 3, 3, 3, 7, 7)


def remap_mode(mode, angle, have_left, have_top):
    """(implementation mode, angle) as dav1d_prepare_intra_edges returns them."""
    if 1 <= mode <= 8:
        angle = _DIR_ANGLE[mode - 1] + 3 * angle
        if angle <= 90:
            return (abi.Z1_PRED if angle < 90 and have_top else abi.VERT_PRED), angle
        if angle < 180:
            return abi.Z2_PRED, angle
        return (abi.Z3_PRED if angle > 180 and have_left else abi.HOR_PRED), angle
    if mode == abi.DC_PRED:
        return ((abi.DC_PRED if have_top else abi.LEFT_DC_PRED) if have_left else
                (abi.TOP_DC_PRED if have_top else abi.DC_128_PRED)), angle
    if mode == abi.PAETH_PRED:
        return ((abi.PAETH_PRED if have_top else abi.HOR_PRED) if have_left else
                (abi.VERT_PRED if have_top else abi.DC_128_PRED)), angle
    return mode, angle


@dataclass
class IntraConfig:
    width: int = 512
    height: int = 256
    bpc: int = 8
    bitdepth_max: int = 255
    seed: int = 1
    cfl_frac: float = 0.4
    filter_edge: bool = True
    tx64: bool = True
    sb_log2: int = 6          # 64x64 superblocks
    tile_cols: int = 1        # uniform tiling (in superblocks); tiles cut the
    tile_rows: int = 1        # edge dependencies (have_left / have_top, w4 / h4)
    sb_edge_backup: bool = True   # superblock-top rows read through top_edge
    # mixed frames: this fraction of blocks is inter (put or compound avg from
    # two edge-replicated random references, MVs within +-mv_range px); intra
    # blocks next to them read their reconstructed pixels
    inter_frac: float = 0.0
    mv_range: int = 32
    ref_pad: int = 64
    # blocks at the right / bottom edge may overhang the picture as AV1's
    # partition allows (a square block is a leaf when its centre is inside):
    # the decoder cuts only the part inside into transform blocks, which may
    # themselves run past the edge (recon_tmpl.c:1208); planes get dst_pad
    # pixels of padding for them
    overhang: bool = False
    # recorder kinds with block data (dav1d_gpu_rec_block_aux): this fraction
    # of inter blocks becomes INTER_MASK / WARP / INTER_OBMC / INTER_WMASK /
    # INTER_SCALED, and half as many intra blocks become palette blocks
    ext_frac: float = 0.0
    # fraction of the 4x4 transform blocks with a residual that are WHT_WHT
    # (lossless), full-range coefficients (workload.lossless_residuals)
    lossless: float = 0.0

    @property
    def pixel_dtype(self):
        return np.uint8 if self.bpc == 8 else np.uint16

    @property
    def coef_dtype(self):
        return np.int16 if self.bpc == 8 else np.int32


@dataclass
class IntraFrame:
    cfg: IntraConfig
    plane_wh: list
    units: np.ndarray        # abi.UNIT_DTYPE, level order (size classes inside a level)
    coefs: np.ndarray
    edges: np.ndarray        # edge pool (written by the edge stage)
    recs: np.ndarray         # INTRA_EDGE_DTYPE, level order
    runs: np.ndarray         # abi.EDGE_BACKUP_DTYPE, level order (per column run)
    unit_start: np.ndarray   # int32 [n_levels + 1]
    class_start: np.ndarray  # int32 [n_levels, N_TX + 1]
    rec_start: np.ndarray
    run_start: np.ndarray
    steps: np.ndarray        # int32 [n, 2]: the decoder's own order (0 unit / 1 oracle run)
    unit_rec: np.ndarray     # int32 per unit: its record or -1
    oracle_runs: np.ndarray  # whole-row backups at superblock-row ends
    top_rows: list           # top_edge shapes (rows, w) per plane
    sb_log2: tuple
    refs: list = None        # [ref][plane] padded reference planes (mixed frames)
    dep_start: np.ndarray = None   # int32 [n + 1]: per unit (level order), its producers (CSR)
    deps: np.ndarray = None        # int32, level-order unit indices

    def ref_origin_offset(self, plane):
        return self.cfg.ref_pad * self.refs[0][plane].shape[1] + self.cfg.ref_pad

    @property
    def n_levels(self):
        return len(self.unit_start) - 1


class _ExtBuilder:
    """Blocks of the recorder kinds with block data (make_intra_frame's
    ext_frac): the dav1d_gpu_rec_block_aux data handed to the recorder, and
    -- independently of the recorder's own cutting (csrc/recorder.hip) --
    the unit records of the same blocks for the oracle's decoder-order walk:
    launch-ahead kinds (WARP / INTER_WMASK / INTER_OBMC / INTER_SCALED) as
    prediction units of at most 32 x 32 (the unit batch's records,
    include/dav1d_gpu.h Dav1dGpuPredKind), INTER_MASK / PAL per transform
    unit.  OBMC and scaled geometry as in workload._ext2_records."""
    PRE = (abi.PRED_WARP, abi.PRED_INTER_WMASK, abi.PRED_INTER_OBMC, abi.PRED_INTER_SCALED)
    # kinds whose prediction is one or more units of their own, the
    # residuals then residual-only units: the launch-ahead kinds and
    # inter-intra (one unit for the whole block, recon_tmpl.c:1540-1580)
    CUT = PRE + (abi.PRED_INTER_INTRA,)

    def __init__(self, cfg, rng, bdmax, refs):
        self.cfg, self.rng, self.bdmax, self.refs = cfg, rng, bdmax, refs
        self.chunks, self.off, self.used = [], 0, False
        self.bd = {}     # (block, plane) -> block state
        self.bb = {}     # block -> plane-independent draws

    def put(self, rec):
        rec = np.ascontiguousarray(rec, np.uint8).ravel()
        at = self.off
        pad = (-len(rec)) % 16
        self.chunks.append(rec)
        if pad:
            self.chunks.append(np.zeros(pad, np.uint8))
        self.off += len(rec) + pad
        self.used = True
        return at

    def pool(self):
        return np.concatenate(self.chunks) if self.chunks else np.zeros(16, np.uint8)

    def block_mode(self, b, kind, mode):
        """Dav1dGpuRecBlock.mode: the inter-intra block's intra mode (DC / V /
        H / SMOOTH, recon_tmpl.c:1547-1549), else the coded mode given."""
        return self._block(b)["iimode"] if kind == abi.PRED_INTER_INTRA else mode

    @staticmethod
    def plane_kind(k, pl):
        if not k:
            return 0
        if k == abi.PRED_WARP and pl:
            return abi.PRED_INTER        # chroma of a warped block: translation
        if k == abi.PRED_INTER_WMASK and pl:
            return abi.PRED_INTER_MASK   # COMPOUND_SEG chroma: the luma's w_mask output
        return k

    def _block(self, b):
        if b not in self.bb:
            r = self.rng
            self.bb[b] = dict(sign=int(r.integers(0, 2)), nref=int(r.integers(1, 3)),
                              iimode=int((abi.DC_PRED, abi.VERT_PRED, abi.HOR_PRED, abi.SMOOTH_PRED)[r.integers(0, 4)]),
                              wt=int(0 if r.random() < 0.5 else r.integers(1, 16)),
                              steps=r.integers(256, 2049, size=(2, 2)), phase=r.integers(0, 1024, size=(2, 2)),
                              abcd=r.integers(-1024, 1025, 4).astype(np.int16), obmc=None)
        return self.bb[b]

    def weight(self, b, kind):
        if kind == abi.PRED_INTER_WMASK:
            return self._block(b)["sign"]
        if kind == abi.PRED_INTER_SCALED:
            bb = self._block(b)
            return bb["wt"] if bb["nref"] == 2 else 0
        return 0

    def _obmc_lists(self, b, bw4):
        bb = self._block(b)
        if bb["obmc"] is None:
            r, mr = self.rng, self.cfg.mv_range * 16
            lw = bw4.bit_length() - 1
            ents = {"top": [], "left": []}
            for side in ("top", "left"):
                pos = 0
                while pos < bw4 and len(ents[side]) < min(lw, 4):
                    step4 = int(np.clip(1 << int(r.integers(1, 5)), 2, 16))
                    if r.random() < 0.8:
                        ents[side].append((pos, step4, r.integers(-mr, mr + 1, 2), int(r.integers(0, 10)),
                                           int(r.integers(0, 2))))
                    pos += step4
            bb["obmc"] = ents
        return bb["obmc"]

    def block_data(self, b, pl, kind, px, py, s, mvs, lx, ly, ls):
        """The block's dav1d_gpu_rec_block_aux data: bytes, None (no data),
        or False for a kind recorded with dav1d_gpu_rec_block."""
        cfg, r = self.cfg, self.rng
        bpp = 1 if cfg.bpc == 8 else 2
        st = {"s": s, "px": px, "py": py, "mvs": mvs}
        self.bd[(b, pl)] = st
        if kind == abi.PRED_INTER_MASK:
            if self._block(b).get("wm") is not None and pl:   # COMPOUND_SEG chroma
                st["mask_at"], st["mask_stride"] = self._block(b)["wm"], s
                return None
            st["mask"] = r.integers(0, 65, (s, s)).astype(np.uint8)
            return st["mask"].tobytes()
        if kind == abi.PRED_INTER_INTRA:   # the block's ii / wedge mask
            st["mask"] = r.integers(0, 65, (s, s)).astype(np.uint8)
            return st["mask"].tobytes()
        if kind == abi.PRED_PAL:
            st["pal"] = r.integers(0, self.bdmax + 1, 8).astype(cfg.pixel_dtype)
            idx = r.integers(0, 8, (s, s))
            st["idx"] = (idx[:, 0::2] | (idx[:, 1::2] << 4)).astype(np.uint8)   # [s][s/2]
            return st["pal"].tobytes() + st["idx"].tobytes()
        if kind == abi.PRED_INTER_WMASK:
            self._block(b)["wm"] = self.put(np.zeros((s // 2) * (s // 2), np.uint8))
            st["wm"] = self._block(b)["wm"]
            return None
        if kind == abi.PRED_WARP:
            a_ = self._block(b)["abcd"]
            n8 = s // 8
            sub = np.zeros((n8, n8), dtype=[("x", "<i2"), ("y", "<i2"), ("mx", "<i2"), ("my", "<i2")])
            mvx, mvy = mvs[0][0] >> 4, mvs[0][1] >> 4
            for sy in range(n8):
                for sx in range(n8):
                    sub["x"][sy, sx] = px + 8 * sx + mvx + int(r.integers(-2, 3))
                    sub["y"][sy, sx] = py + 8 * sy + mvy + int(r.integers(-2, 3))
                    sub["mx"][sy, sx] = ((int(r.integers(0, 65536)) - 4 * int(a_[0]) - 7 * int(a_[1])) & ~63) >> 6
                    sub["my"][sy, sx] = ((int(r.integers(0, 65536)) - 4 * int(a_[2]) - 4 * int(a_[3])) & ~63) >> 6
            st["warp"] = sub
            return a_.tobytes() + bytes(8) + sub.tobytes()
        if kind == abi.PRED_INTER_OBMC:
            sub_ = 1 if pl else 0
            hm = vm = 4 >> sub_
            bw4 = int(ls[b]) // 4
            lists = self._obmc_lists(b, bw4)
            ents = []
            if ly[b] > 0 and (not pl or bw4 * hm + bw4 * vm >= 16):
                for (x, step4, m_, f2d, rr) in lists["top"]:
                    ow4, oh4 = min(step4, bw4), min(bw4, 16) >> 1
                    ents.append((0, x * hm, x * hm + ow4 * hm, 0, (vm * oh4 * 3) >> 2, ow4, (oh4 * 3 + 3) >> 2,
                                 vm * oh4, m_, f2d, rr))
            if lx[b] > 0:
                for (y, step4, m_, f2d, rr) in lists["left"]:
                    ow4, oh4 = min(bw4, 16) >> 1, min(step4, bw4)
                    ents.append((1, 0, (hm * ow4 * 3) >> 2, y * vm, y * vm + oh4 * vm, ow4, oh4, hm * ow4, m_, f2d, rr))
            blk = np.zeros(16 + 24 * len(ents), np.uint8)
            blk[0:4] = np.array([len(ents)], "<i4").view(np.uint8)
            laps = []
            for k, (dr, xa, xb, ya, yb, lw4, lh4, mbase, m_, f2d, rr) in enumerate(ents):
                mvx, mvy = (int(m_[0]) >> 1, int(m_[1]) >> 1) if pl else (int(m_[0]), int(m_[1]))
                e = blk[16 + 24 * k:16 + 24 * (k + 1)]
                e[0:8] = np.array([mvx, mvy], "<i4").view(np.uint8)
                e[8:18] = [f2d, rr, xa, ya, xb, yb, (lw4 * hm) // 4, (lh4 * vm) // 4, dr, mbase]
                laps.append((mvx, mvy, f2d, rr, xa, ya, xb, yb, (lw4 * hm) // 4, (lh4 * vm) // 4, dr, mbase))
            st["laps"] = laps
            return blk.tobytes()
        if kind == abi.PRED_INTER_SCALED:
            bb = self._block(b)
            sub_ = 1 if pl else 0
            pw_, ph_ = (cfg.width >> sub_, cfg.height >> sub_)
            pad = cfg.ref_pad
            recs = []
            for k in range(bb["nref"]):
                dx, dy = int(bb["steps"][k, 0]), int(bb["steps"][k, 1])
                mx0, my0 = int(bb["phase"][k, 0]), int(bb["phase"][k, 1])
                span_x, span_y = ((s - 1) * dx + mx0) >> 10, ((s - 1) * dy + my0) >> 10
                gx = int(np.clip(px + (mvs[k][0] >> 4), -pad + 4, pw_ + pad - 6 - span_x))
                gy = int(np.clip(py + (mvs[k][1] >> 4), -pad + 4, ph_ + pad - 6 - span_y))
                recs.append((gx, gy, mx0, my0, dx, dy))
            st["scaled"] = recs
            blk = np.zeros(16 + 16 * len(recs), np.uint8)
            blk[0:4] = np.array([len(recs)], "<i4").view(np.uint8)
            for k, (gx, gy, mx0, my0, dx, dy) in enumerate(recs):
                blk[16 + 16 * k:24 + 16 * k] = np.array([gx, gy], "<i4").view(np.uint8)
                blk[24 + 16 * k:32 + 16 * k] = np.array([mx0, my0, dx, dy], "<u2").view(np.uint8)
            return blk.tobytes()
        return False

    def unit_record(self, b, pl, kind, ox, oy, uw, uh, ux, uy):
        """The oracle's aux value for a unit of the block at (ox, oy)."""
        st = self.bd[(b, pl)]
        s = st["s"]
        bpp = 1 if self.cfg.bpc == 8 else 2
        if kind == abi.PRED_INTER_MASK:
            if "mask_at" not in st:
                st["mask_at"], st["mask_stride"] = self.put(st["mask"]), s
            return st["mask_at"] + oy * st["mask_stride"] + ox
        if kind == abi.PRED_INTER_INTRA:   # record (its edge slot is patched in later) + mask
            rec = np.zeros(16 + s * s, np.uint8)
            rec[4] = self._block(b)["iimode"]
            rec[8:12] = np.array([self.off + 16], "<i4").view(np.uint8)   # the mask follows the record
            rec[16:] = st["mask"].ravel()
            return self.put(rec)
        if kind == abi.PRED_PAL:
            rec = np.zeros(16 + (uw // 2) * uh, np.uint8)
            rec[:8 * bpp] = st["pal"].view(np.uint8)
            rec[16:] = st["idx"][oy:oy + uh, ox // 2:(ox + uw) // 2].ravel()
            return self.put(rec)
        if kind == abi.PRED_INTER_WMASK:
            return st["wm"] + (oy >> 1) * (s >> 1) + (ox >> 1)
        if kind == abi.PRED_WARP:
            a_ = self._block(b)["abcd"]
            sub = st["warp"][oy // 8:(oy + uh) // 8, ox // 8:(ox + uw) // 8]
            return self.put(np.concatenate([a_.view(np.uint8), np.zeros(8, np.uint8),
                                            np.ascontiguousarray(sub).view(np.uint8).ravel()]))
        rs = self.refs[0][pl].shape[1]
        if kind == abi.PRED_INTER_OBMC:
            ents = []
            for (mvx, mvy, f2d, rr, xa, ya, xb, yb, lw4, lh4, dr, mbase) in st["laps"]:
                x0, x1 = max(xa - ox, 0), min(xb - ox, uw)
                y0, y1 = max(ya - oy, 0), min(yb - oy, uh)
                if x0 >= x1 or y0 >= y1:
                    continue
                e = np.zeros(16, np.uint8)
                e[0:4] = np.array([(uy + (mvy >> 4)) * rs + ux + (mvx >> 4)], "<i4").view(np.uint8)
                e[4:16] = [mvx & 15, mvy & 15, f2d, rr, x0, y0, x1, y1, lw4, lh4, dr, mbase + (ox if dr else oy)]
                ents.append(e)
            hdr = np.zeros(16, np.uint8)
            hdr[0:4] = np.array([len(ents)], "<i4").view(np.uint8)
            return self.put(np.concatenate([hdr] + ents))
        if kind == abi.PRED_INTER_SCALED:
            recs = st["scaled"]
            out = np.zeros(16 + 16 * len(recs), np.uint8)
            out[0:4] = np.array([len(recs)], "<i4").view(np.uint8)
            for k, (gx, gy, mx0, my0, dx, dy) in enumerate(recs):
                px_, py_ = mx0 + ox * dx, my0 + oy * dy
                out[16 + 16 * k:20 + 16 * k] = np.array([(gy + (py_ >> 10)) * rs + gx + (px_ >> 10)],
                                                        "<i4").view(np.uint8)
                out[20 + 16 * k:28 + 16 * k] = np.array([px_ & 1023, py_ & 1023, dx, dy], "<u2").view(np.uint8)
            return self.put(out)
        raise ValueError(kind)


def _partition_overhang(rng, W, H):
    """Quadtree leaves (x, y, size) over W x H where a block may run past the
    right / bottom edge: AV1 allows PARTITION_NONE while the block's centre
    row / column is inside (has_rows / has_cols), else the block splits."""
    from .workload import _LEVELS
    ys, xs = np.meshgrid(np.arange(0, H, 64), np.arange(0, W, 64), indexing="ij")
    xs, ys = xs.ravel(), ys.ravel()
    out = []
    for s, p in _LEVELS:
        ok = (xs + s // 2 < W) & (ys + s // 2 < H)
        outside = (xs >= W) | (ys >= H)
        leaf = ok & ((rng.random(len(xs)) < p) | (s == 8))
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


def _morton(x, y):
    r = 0
    for b in range(4):
        r |= ((x >> b) & 1) << (2 * b) | ((y >> b) & 1) << (2 * b + 1)
    return r


def make_intra_frame(cfg: IntraConfig) -> IntraFrame:
    """A seeded all-intra 4:2:0 frame coded the way recon_b_intra walks it
    (src/recon_tmpl.c:1195-1596): quadtree blocks in superblock raster and
    Z order, luma transform blocks in raster order, then U and V; luma modes
    over all 13 coded modes + filter intra (blocks <= 32x32), angle deltas
    -3..3, chroma modes or CfL (whole chroma block); block edge flags from
    decode order (what intra_edge.c's tree encodes), transform-level flags
    as recon_b_intra derives them (:1252-1266), smooth flags from the above
    / left neighbours, superblock-top rows read through top_edge.  Then the
    dependency levels: a unit's level is one more than the highest level of
    any pixel its edges (after the mode remap) or its CfL luma read."""
    from .workload import _partition, _tx_candidates, lossless_residuals, make_residuals
    assert cfg.width % 32 == 0 and cfg.height % 8 == 0
    rng = np.random.default_rng(cfg.seed)
    W, H = cfg.width, cfg.height
    bdmax = 255 if cfg.bpc == 8 else cfg.bitdepth_max
    planes = [(W, H), (W // 2, H // 2), (W // 2, H // 2)]
    sbl = (cfg.sb_log2, cfg.sb_log2 - 1, cfg.sb_log2 - 1)
    sb = 1 << cfg.sb_log2
    lx, ly, ls = _partition_overhang(rng, W, H) if cfg.overhang else _partition(rng, W, H)
    # uniform tiles of tsw x tsh superblocks, decoded in raster order
    tsw = -(-(-(-W // sb)) // cfg.tile_cols) * sb
    tsh = -(-(-(-H // sb)) // cfg.tile_rows) * sb
    order = np.lexsort((np.array([_morton((x % sb) >> 3, (y % sb) >> 3) for x, y in zip(lx, ly)]),
                        lx // sb, ly // sb, lx // tsw, ly // tsh))
    lx, ly, ls = lx[order], ly[order], ls[order]
    tile_x0, tile_y0 = (lx // tsw) * tsw, (ly // tsh) * tsh          # luma px
    tile_x1, tile_y1 = np.minimum(tile_x0 + tsw, W), np.minimum(tile_y0 + tsh, H)
    nb = len(lx)
    ymode = rng.integers(0, 14, nb)
    ymode[(ymode == abi.FILTER_PRED) & (ls > 32)] = abi.DC_PRED
    yang = np.where((ymode >= 1) & (ymode <= 8), rng.integers(-3, 4, nb),
                    np.where(ymode == abi.FILTER_PRED, rng.integers(0, 5, nb), 0))
    is_cfl = rng.random(nb) < cfg.cfl_frac
    uvmode = rng.integers(0, 13, nb)
    uvang = np.where((uvmode >= 1) & (uvmode <= 8), rng.integers(-3, 4, nb), 0)
    alpha = rng.integers(1, 17, (nb, 2)) * np.where(rng.random((nb, 2)) < 0.5, -1, 1)
    # inter blocks (own stream, so frames without them keep their draws)
    irng = np.random.default_rng(cfg.seed ^ 0x1A7E)
    bkind = np.where(irng.random(nb) < cfg.inter_frac,
                     np.where(irng.random(nb) < 0.5, abi.PRED_INTER_AVG, abi.PRED_INTER), abi.PRED_INTRA)
    bmv = irng.integers(-cfg.mv_range * 16, cfg.mv_range * 16 + 1, size=(nb, 2, 2))
    bfilt = irng.integers(0, 9, nb)
    refs = None
    if cfg.inter_frac > 0:
        refs = []
        pad = cfg.ref_pad
        for _ in range(2):
            rp = []
            for (pw_, ph_) in planes:
                stride = (pw_ + 2 * pad + 63) // 64 * 64
                a_ = irng.integers(0, bdmax + 1, size=(ph_, pw_)).astype(cfg.pixel_dtype)
                rp.append(np.ascontiguousarray(np.pad(a_, ((pad, pad), (pad, stride - pw_ - pad)), mode="edge")))
            refs.append(rp)
    is_inter = bkind != abi.PRED_INTRA
    xk = np.zeros(nb, np.int64)   # a block's recorder kind with block data, 0 none
    xr = np.random.default_rng(cfg.seed ^ 0xE7E7)
    if cfg.ext_frac > 0:
        ext_kinds = np.array([abi.PRED_INTER_MASK, abi.PRED_WARP, abi.PRED_INTER_OBMC, abi.PRED_INTER_WMASK,
                              abi.PRED_INTER_SCALED, abi.PRED_INTER_INTRA])
        xk = np.where(is_inter & (xr.random(nb) < cfg.ext_frac), ext_kinds[xr.integers(0, 6, nb)], 0)
        # inter-intra exists for blocks up to 32x32 (interintra_allowed_mask)
        xk = np.where((xk == abi.PRED_INTER_INTRA) & (ls > 32), abi.PRED_INTER_MASK, xk)
        pal_b = ~is_inter & (xr.random(nb) < cfg.ext_frac * 0.5)
        xk = np.where(pal_b, abi.PRED_PAL, xk)
        ymode[pal_b] = abi.DC_PRED     # palette blocks code DC_PRED (no smooth context)
        uvmode[pal_b] = abi.DC_PRED
        is_cfl[pal_b] = False
    XB = _ExtBuilder(cfg, xr, bdmax, refs)
    # decode index of the block covering each luma 4x4
    bmap = np.full((H // 4, W // 4), -1, np.int64)
    for b in range(nb):
        bmap[ly[b] // 4:(ly[b] + ls[b]) // 4, lx[b] // 4:(lx[b] + ls[b]) // 4] = b
    assert bmap.min() >= 0
    smooth = lambda m: 9 <= m <= 11   # noqa: E731

    U = {k: [] for k in ("plane", "x", "y", "tw", "th", "blk", "cfl", "mode", "angle", "flags", "pred", "aux",
                         "bsz", "weight", "nores", "cflpad")}
    BL = []   # per block and plane, decode order: what recon_b_* hands the recorder
    BLX = []  # per BL entry: its dav1d_gpu_rec_block_aux data (bytes), None, or False (plain block)
    for b in range(nb):
        x, y, s = int(lx[b]), int(ly[b]), int(ls[b])
        x0, y0, x1, y1 = int(tile_x0[b]), int(tile_y0[b]), int(tile_x1[b]), int(tile_y1[b])
        tr = y > y0 and x + s < x1 and bmap[(y - 1) // 4, (x + s) // 4] < b
        bl = x > x0 and y + s < y1 and bmap[(y + s) // 4, (x - 1) // 4] < b
        # mode contexts are reset at tile starts (dav1d_reset_context)
        above = bmap[(y - 1) // 4, x // 4] if y > y0 else -1
        left = bmap[y // 4, (x - 1) // 4] if x > x0 else -1
        # (inter neighbours carry no smooth mode)
        ysm = ((above >= 0 and not is_inter[above] and smooth(ymode[above])) or
               (left >= 0 and not is_inter[left] and smooth(ymode[left])))
        uvsm = ((above >= 0 and not is_inter[above] and not is_cfl[above] and smooth(uvmode[above])) or
                (left >= 0 and not is_inter[left] and not is_cfl[left] and smooth(uvmode[left])))
        cands = _tx_candidates(s, cfg.tx64)
        luma_tx = cands[int(rng.integers(0, len(cands)))]
        for pl in range(3):
            ss = 0 if pl == 0 else 1
            px_, py_, ps_ = x >> ss, y >> ss, s >> ss
            tw, th = luma_tx if pl == 0 else (ps_, ps_)
            cfl = pl > 0 and bool(is_cfl[b]) and not is_inter[b]
            bw4 = ps_ // 4
            kind_ = int(bkind[b]) if is_inter[b] else (abi.PRED_CFL if cfl else abi.PRED_INTRA)
            xkind = XB.plane_kind(int(xk[b]), pl)
            if xkind:
                kind_ = xkind
            bfl = (abi.IE_TOP_HAS_RIGHT if tr else 0) | (abi.IE_LEFT_HAS_BOTTOM if bl else 0)
            if cfg.filter_edge:
                bfl |= abi.IE_FILTER_EDGE
            if (ysm if pl == 0 else uvsm):
                bfl |= abi.IE_SMOOTH
            mvs = [(int(bmv[b, k, 0]) >> ss, int(bmv[b, k, 1]) >> ss) for k in range(2)]
            weight = XB.weight(b, kind_)
            cfl_pad = 0
            if cfl:   # cfl_ac's w_pad / h_pad (recon_tmpl.c:1372-1380), luma transform units
                w4l, h4l = min(s, W - x) // 4, min(s, H - y) // 4
                tw4l, th4l = luma_tx[0] // 4, luma_tx[1] // 4
                fr_r = ((((w4l + 1) >> 1) << 1) + tw4l - 1) & ~(tw4l - 1)
                fr_b = ((((h4l + 1) >> 1) << 1) + th4l - 1) & ~(th4l - 1)
                cfl_pad = max(0, ps_ // 4 - (fr_r >> 1)) | max(0, ps_ // 4 - (fr_b >> 1)) << 4
            BL.append((pl, px_, py_, ps_, ps_, abi.TX_INDEX[(tw, th)], kind_, x0 >> ss, y0 >> ss, x1 >> ss,
                       y1 >> ss, mvs[0][0], mvs[1][0], mvs[0][1], mvs[1][1], 0, 1, int(bfilt[b]), weight,
                       cfl_pad if cfl else XB.block_mode(b, kind_, int(ymode[b] if pl == 0 else uvmode[b])),
                       0 if cfl else int(yang[b] if pl == 0 else uvang[b]),
                       int(alpha[b, pl - 1]) if cfl else 0, 0 if cfl or is_inter[b] else bfl))
            BLX.append(XB.block_data(b, pl, kind_, px_, py_, ps_, mvs, lx, ly, ls))
            if kind_ in XB.CUT:   # prediction units of their own (<= 32 x 32), residuals apart
                us = min(ps_, 32)
                for oy in range(0, min(ps_, planes[pl][1] - py_), us):
                    for ox in range(0, min(ps_, planes[pl][0] - px_), us):
                        rec_ = XB.unit_record(b, pl, kind_, ox, oy, us, us, px_ + ox, py_ + oy)
                        for k_, v_ in (("plane", pl), ("x", px_ + ox), ("y", py_ + oy), ("tw", us), ("th", us),
                                       ("blk", b), ("cfl", False), ("mode", XB.block_mode(b, kind_, 0)),
                                       ("angle", 0), ("flags", 0),
                                       ("pred", kind_), ("aux", rec_), ("bsz", ps_), ("weight", weight),
                                       ("nores", True), ("cflpad", 0)):
                            U[k_].append(v_)
            # the part of the block inside the grid (w4 / h4, recon_tmpl.c:1208)
            bwc, bhc = min(ps_, planes[pl][0] - px_), min(ps_, planes[pl][1] - py_)
            for oy in range(0, bhc, th):
                for ox in range(0, bwc, tw):
                    x4, y4 = ox // 4, oy // 4
                    fl = 0
                    if not cfl:
                        if (y4 == 0 and tr) or x4 + tw // 4 < bwc // 4:
                            fl |= abi.IE_TOP_HAS_RIGHT
                        if x4 == 0 and (bl or y4 + th // 4 < bhc // 4):
                            fl |= abi.IE_LEFT_HAS_BOTTOM
                        if cfg.filter_edge:
                            fl |= abi.IE_FILTER_EDGE
                        if (ysm if pl == 0 else uvsm):
                            fl |= abi.IE_SMOOTH
                    U["plane"].append(pl)
                    U["x"].append(px_ + ox)
                    U["y"].append(py_ + oy)
                    U["tw"].append(tw)
                    U["th"].append(th)
                    U["blk"].append(b)
                    U["cfl"].append(cfl)
                    U["mode"].append(abi.DC_PRED if cfl else int(ymode[b] if pl == 0 else uvmode[b]))
                    U["angle"].append(0 if cfl else int(yang[b] if pl == 0 else uvang[b]))
                    U["flags"].append(fl)
                    U["pred"].append(abi.PRED_NONE if kind_ in XB.CUT else kind_)
                    U["aux"].append(XB.unit_record(b, pl, kind_, ox, oy, tw, th, px_ + ox, py_ + oy)
                                    if kind_ in (abi.PRED_INTER_MASK, abi.PRED_PAL) else -1)
                    U["bsz"].append(ps_)
                    U["weight"].append(weight)
                    U["cflpad"].append(cfl_pad)
                    # residual-only units of launch-ahead blocks: some carry none
                    U["nores"].append(kind_ in XB.CUT and XB.rng.random() < 0.3)
    plane_u = np.array(U["plane"], np.int32)
    ux, uy = np.array(U["x"], np.int32), np.array(U["y"], np.int32)
    tw, th = np.array(U["tw"], np.int32), np.array(U["th"], np.int32)
    blk = np.array(U["blk"], np.int32)
    cflu = np.array(U["cfl"], bool)
    n = len(ux)
    tx = np.array([abi.TX_INDEX[(a, b_)] for a, b_ in zip(tw, th)], np.int32)
    pw = np.array([p[0] for p in planes])
    ph = np.array([p[1] for p in planes])
    flags = np.array(U["flags"], np.int32)
    ssu = np.where(plane_u > 0, 1, 0)
    tx0, ty0 = tile_x0[blk] >> ssu, tile_y0[blk] >> ssu         # the unit's tile, plane px
    tx1, ty1 = tile_x1[blk] >> ssu, tile_y1[blk] >> ssu
    flags |= np.where(ux > tx0, abi.IE_HAVE_LEFT, 0)
    flags |= np.where(uy > ty0, abi.IE_HAVE_TOP, 0)
    sbh = np.array([1 << s_ for s_ in sbl])[plane_u]
    if cfg.sb_edge_backup:
        flags |= np.where((uy > ty0) & (uy % sbh == 0), abi.IE_TOP_SB_EDGE, 0)

    units = np.zeros(n, abi.UNIT_DTYPE)   # decode order for now
    dpad = 64 if cfg.overhang else 0   # plane padding right / below for overhanging transform blocks
    units["dst_off"] = uy * (pw[plane_u] + dpad) + ux
    units["tx"] = tx
    units["plane"] = plane_u
    predu = np.array(U["pred"], np.int32)
    units["pred"] = predu
    # units that read no picture pixels: inter kinds, palette, residual-only
    interu = ~np.isin(predu, (abi.PRED_INTRA, abi.PRED_CFL))
    # units that read edges: intra, CfL and the intra half of inter-intra
    edger = np.isin(predu, (abi.PRED_INTRA, abi.PRED_CFL, abi.PRED_INTER_INTRA))
    bsz = np.array(U["bsz"], np.int32)
    units["bw4"] = units["bh4"] = np.where(interu, bsz // 4, 0)
    txtp, nzw, nzh, coef_off, coefs = make_residuals(rng, tx, tw, th, bdmax, cfg.coef_dtype)
    if cfg.lossless > 0:
        lossless_residuals(cfg, tx, txtp, nzw, nzh, coef_off, coefs)
    txtp = np.where(np.array(U["nores"], bool), abi.NO_RESIDUAL, txtp)
    units["txtp"], units["nzw"], units["nzh"], units["coef_off"] = txtp, nzw, nzh, coef_off
    edge_len = np.where(edger, 2 * th + 2 * tw + 1, 0)
    edge_start = np.concatenate([[0], np.cumsum(edge_len)[:-1]])
    units["edge_off"] = np.where(interu, 0, edge_start + 2 * th)   # (inter-intra: in its record)
    iu = ~cflu & ~interu
    units["max_w"] = np.where(iu, pw[plane_u] - ux, 0)
    units["max_h"] = np.where(iu, ph[plane_u] - uy, 0)
    if refs is not None:   # inter parameters (the inter view of the union)
        ref_stride = np.array([refs[0][p_].shape[1] for p_ in range(3)])
        iv = units[interu]
        ib_, ip_ = blk[interu], plane_u[interu]
        for k in range(2):
            mvx, mvy = bmv[ib_, k, 0], bmv[ib_, k, 1]
            mvx = np.where(ip_ > 0, mvx >> 1, mvx)
            mvy = np.where(ip_ > 0, mvy >> 1, mvy)
            sx, sy = ux[interu] + (mvx >> 4), uy[interu] + (mvy >> 4)
            # WARP: the 8x8 positions are absolute (src_off, their base, 0)
            iv[f"src_off{k}"] = np.where(predu[interu] == abi.PRED_WARP, 0, sy * ref_stride[ip_] + sx)
            iv[f"mx{k}"] = mvx & 15
            iv[f"my{k}"] = mvy & 15
            iv[f"ref{k}"] = k
        iv["filter2d"] = bfilt[ib_]
        iv["weight"] = np.array(U["weight"], np.int32)[interu]
        units[interu] = iv
    cu = units[cflu]
    cu["cfl_alpha"] = alpha[blk[cflu], plane_u[cflu] - 1]
    cu["cfl_pad_wh"] = np.array(U["cflpad"], np.int32)[cflu]
    cu["cfl_luma_off"] = (2 * uy[cflu]) * (W + dpad) + 2 * ux[cflu]
    units[cflu] = cu

    # dependency levels, at 4x4 granularity per plane
    # (and the producers: the units owning the 4x4s a unit reads)
    lv = [np.full((h // 4, w // 4), -1, np.int64) for (w, h) in planes]
    own = [np.full((h // 4, w // 4), -1, np.int64) for (w, h) in planes]
    level = np.zeros(n, np.int64)
    producers = []
    modes, angles = U["mode"], U["angle"]
    for i in range(n):
        p, x4, y4 = int(plane_u[i]), int(ux[i]) // 4, int(uy[i]) // 4
        t4w, t4h = int(tw[i]) // 4, int(th[i]) // 4
        w4, h4 = int(tx1[i]) // 4, int(ty1[i]) // 4
        f = int(flags[i])
        hl, ht = bool(f & abi.IE_HAVE_LEFT), bool(f & abi.IE_HAVE_TOP)
        m, _ = remap_mode(modes[i], angles[i], hl, ht)
        nd = _NEEDS[m] if edger[i] else 0   # inter units read only the references
        L, O = lv[p], own[p]
        reads = []   # (plane, rows, cols) regions read
        if nd & _NEED_L:
            if hl:
                reads.append((p, slice(y4, min(y4 + t4h, h4)), slice(x4 - 1, x4)))
                if nd & _NEED_BL and y4 + t4h < h4 and (f & abi.IE_LEFT_HAS_BOTTOM):
                    reads.append((p, slice(y4 + t4h, min(y4 + 2 * t4h, h4)), slice(x4 - 1, x4)))
            elif ht:
                reads.append((p, slice(y4 - 1, y4), slice(x4, x4 + 1)))
        if nd & _NEED_T:
            if ht:
                reads.append((p, slice(y4 - 1, y4), slice(x4, min(x4 + t4w, w4))))
                if nd & _NEED_TR and x4 + t4w < w4 and (f & abi.IE_TOP_HAS_RIGHT):
                    reads.append((p, slice(y4 - 1, y4), slice(x4 + t4w, min(x4 + 2 * t4w, w4))))
            elif hl:
                reads.append((p, slice(y4, y4 + 1), slice(x4 - 1, x4)))
        if nd & _NEED_TL and (hl or ht):
            ry, rx = (y4 - 1, x4 - 1) if hl and ht else (y4, x4 - 1) if hl else (y4 - 1, x4)
            reads.append((p, slice(ry, ry + 1), slice(rx, rx + 1)))
        if cflu[i]:
            reads.append((0, slice(2 * y4, 2 * (y4 + t4h)), slice(2 * x4, 2 * (x4 + t4w))))
        if predu[i] == abi.PRED_NONE:   # the residual reads the prediction under it
            reads.append((p, slice(y4, y4 + t4h), slice(x4, x4 + t4w)))
        d, pr = -1, set()
        for (q, ry, rx) in reads:
            assert lv[q][ry, rx].min() >= 0     # (a block's luma precedes its chroma)
            d = max(d, int(lv[q][ry, rx].max()))
            pr.update(int(v) for v in np.unique(own[q][ry, rx]))
        level[i] = d + 1
        producers.append(sorted(pr))
        L[y4:y4 + t4h, x4:x4 + t4w] = d + 1
        O[y4:y4 + t4h, x4:x4 + t4w] = i
    for L in lv:
        assert L.min() >= 0

    # backup runs: each superblock row's last pixel row, per run of 4x4
    # columns written at one level, backed up right after that level
    runs, run_lv = [], []
    for p, (w, h) in enumerate(planes if cfg.sb_edge_backup else []):
        nsb = (h + (1 << sbl[p]) - 1) >> sbl[p]
        for r in range(nsb - 1):
            row = lv[p][(((r + 1) << sbl[p]) - 1) // 4]
            c0 = 0
            for c in range(1, len(row) + 1):
                if c == len(row) or row[c] != row[c0]:
                    runs.append((p, r, c0 * 4, (c - c0) * 4))
                    run_lv.append(int(row[c0]))
                    c0 = c
    runs = np.array(runs, abi.EDGE_BACKUP_DTYPE) if runs else np.zeros(0, abi.EDGE_BACKUP_DTYPE)
    run_lv = np.array(run_lv, np.int64)

    # the decoder's order with whole-row backups at superblock-row ends
    # (per tile superblock row, dav1d_backup_ipred_edge at its end)
    steps, oracle_runs = [], []
    cur = None
    for i in range(n + 1):
        key = None if i == n else (int(tile_y0[blk[i]]), int(tile_x0[blk[i]]), int(ly[blk[i]]) >> cfg.sb_log2)
        if cur is not None and key != cur and cfg.sb_edge_backup:
            _, cx0, r = cur
            cx1 = min(cx0 + tsw, W)
            for p, (w, h) in enumerate(planes):
                ss_ = 0 if p == 0 else 1
                if ((r + 1) << sbl[p]) <= h:
                    oracle_runs.append((p, r, cx0 >> ss_, (cx1 - cx0) >> ss_))
                    steps.append((1, len(oracle_runs) - 1))
        cur = key
        if i < n:
            steps.append((0, i))

    dec_units = units.copy()
    # level order, size classes inside a level, then pred / mode / type
    perm = np.lexsort((units["txtp"], np.array(modes), units["pred"], units["tx"], level))
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    units = units[perm]
    lvl_sorted = level[perm]
    n_levels = int(level.max()) + 1
    unit_start = np.searchsorted(lvl_sorted, np.arange(n_levels + 1)).astype(np.int32)
    class_start = np.zeros((n_levels, abi.N_TX + 1), np.int32)
    for l_ in range(n_levels):
        t = units["tx"][unit_start[l_]:unit_start[l_ + 1]]
        class_start[l_, 1:] = np.cumsum(np.bincount(t, minlength=abi.N_TX))
    # one record per unit (every unit is INTRA or CFL), in unit order:
    # record i serves unit i, as the fused launch requires
    recs = np.zeros(n, abi.INTRA_EDGE_DTYPE)
    recs["unit"] = inv
    recs["x4"], recs["y4"] = ux // 4, uy // 4
    recs["w4"], recs["h4"] = tx1 // 4, ty1 // 4
    recs["mode"], recs["angle"], recs["flags"] = modes, angles, flags
    recs = recs[perm]
    aux = np.array(U["aux"], np.int64)[perm].astype(np.int32)
    rec_start = unit_start.copy()
    unit_rec = np.where(np.isin(units["pred"], (abi.PRED_INTRA, abi.PRED_CFL, abi.PRED_INTER_INTRA)),
                        np.arange(n), -1).astype(np.int32)
    rp = np.argsort(run_lv, kind="stable")
    runs = runs[rp]
    run_start = np.searchsorted(run_lv[rp], np.arange(n_levels + 1)).astype(np.int32)
    steps = np.array(steps, np.int32)
    unit_steps = steps[:, 0] == 0
    steps[unit_steps, 1] = inv[steps[unit_steps, 1]]
    top_rows = [(max(1, h >> s_), w) for (w, h), s_ in zip(planes, sbl)]
    edges = np.zeros(int(edge_len.sum()), cfg.pixel_dtype)
    dep_start = np.zeros(n + 1, np.int32)
    dep_start[1:] = np.cumsum([len(producers[j]) for j in perm])
    deps = np.array([inv[q] for j in perm for q in producers[j]], np.int32)
    fr = IntraFrame(cfg, planes, units, coefs, edges, recs, runs, unit_start, class_start, rec_start,
                    run_start, steps, unit_rec, np.array(oracle_runs, abi.EDGE_BACKUP_DTYPE), top_rows, sbl,
                    refs, dep_start, deps)
    fr.blocks = BL
    fr.block_aux = BLX
    fr.dst_pad = dpad
    fr.dec_units = dec_units
    fr.aux = aux if XB.used else None
    fr.aux_pool = XB.pool() if XB.used else None
    for i in np.nonzero(predu == abi.PRED_INTER_INTRA)[0]:   # inter-intra records: their edge slots
        o = int(U["aux"][i])
        fr.aux_pool[o:o + 4] = np.array([edge_start[i] + 2 * th[i]], "<i4").view(np.uint8)
    return fr


def frame_batch(fr, dst_ptrs, units, coefs, edges, ref_ptrs=None, aux=None, aux_pool=None):
    """abi.FrameBatch of an IntraFrame (cfl_luma = the reconstructed luma;
    ref_ptrs[r][p]: addresses of the padded reference planes, mixed frames)."""
    bpp = 1 if fr.cfg.bpc == 8 else 2
    b = abi.FrameBatch()
    pad = getattr(fr, "dst_pad", 0)
    for p, (w, h) in enumerate(fr.plane_wh):
        b.dst[p].data, b.dst[p].stride, b.dst[p].w, b.dst[p].h = dst_ptrs[p], (w + pad) * bpp, w, h
        for r in range(len(ref_ptrs or [])):
            a = fr.refs[r][p]
            b.ref[r][p].data = ref_ptrs[r][p] + fr.ref_origin_offset(p) * bpp
            b.ref[r][p].stride = a.shape[1] * bpp
            b.ref[r][p].w, b.ref[r][p].h = w, h
    b.units, b.n_units = units, len(fr.units)
    b.class_start[abi.N_TX] = len(fr.units)   # unused: the driver passes per-level ranges
    b.coef, b.edges = coefs, edges
    b.bitdepth_max = fr.cfg.bitdepth_max if fr.cfg.bpc == 16 else 255
    W, H = fr.plane_wh[0]
    b.cfl_luma.data, b.cfl_luma.stride, b.cfl_luma.w, b.cfl_luma.h = dst_ptrs[0], (W + pad) * bpp, W, H
    b.cfl_ss = 3
    if aux is not None:   # per-unit aux offsets (unit order) and the aux pool
        b.aux, b.aux_pool = aux, aux_pool
    return b


def edge_batch(fr, dst_ptrs, top_ptrs, units, edges, recs):
    bpp = 1 if fr.cfg.bpc == 8 else 2
    b = abi.IntraEdgeBatch()
    pad = getattr(fr, "dst_pad", 0)
    for p, (w, h) in enumerate(fr.plane_wh):
        b.pic[p].data, b.pic[p].stride, b.pic[p].w, b.pic[p].h = dst_ptrs[p], (w + pad) * bpp, w, h
        rows, tw_ = fr.top_rows[p]
        # no top_edge when the frame does not back up superblock rows (the
        # fused launch stores superblock-bottom rows whenever it has one)
        b.top_edge[p].data = top_ptrs[p] if fr.cfg.sb_edge_backup else None
        b.top_edge[p].stride = tw_ * bpp
        b.top_edge[p].w, b.top_edge[p].h = tw_, rows
        b.sb_log2[p] = fr.sb_log2[p]
    b.units, b.edges, b.recs = units, edges, recs
    b.n_recs = len(fr.recs)
    b.bitdepth_max = fr.cfg.bitdepth_max if fr.cfg.bpc == 16 else 255
    return b


def task_group_bytes(fr):
    """Dav1dGpuIntraSchedule.task_group for an IntraFrame (schedule order):
    prediction kind << 4 | coded intra mode, the keys the level sort orders
    a size class's units by."""
    return np.ascontiguousarray(((fr.units["pred"].astype(np.uint16) & 15) << 4 |
                                 (fr.recs["mode"].astype(np.uint16) & 15)).astype(np.uint8))


def sb_schedule(fr):
    """The superblock form of an IntraFrame's schedule (DGPU_IS_SB): every
    unit goes to the superblock holding its top-left pixel (4:2:0 chroma
    superblocks are the luma ones halved, so a superblock owns its luma and
    chroma); inside a superblock a unit sits one level above the units of
    the same superblock it reads (producers elsewhere are awaited once, per
    superblock); the superblocks in raster order, which puts every
    superblock after those it reads (left, top, top-right: AV1's intra edges
    and CfL never reach further).  Returns (perm, unit_start, class_start,
    sb_level_start, sb_dep_start, sb_deps): perm[k] is the level-order index
    of the k-th unit of the superblock order."""
    n = len(fr.units)
    W, H = fr.plane_wh[0]
    sb0 = fr.sb_log2[0]
    nsbx = (W + (1 << sb0) - 1) >> sb0
    p = fr.units["plane"].astype(np.int64)
    sbl = np.array(fr.sb_log2, np.int64)[p]
    sbx = (fr.recs["x4"].astype(np.int64) * 4) >> sbl
    sby = (fr.recs["y4"].astype(np.int64) * 4) >> sbl
    sb = sby * nsbx + sbx
    ds, dp = fr.dep_start, fr.deps
    lv = np.zeros(n, np.int64)   # level inside the superblock (units are in level order: producers first)
    sdeps = [set() for _ in range(n)]
    for i in range(n):
        d = -1
        for q in dp[ds[i]:ds[i + 1]]:
            if sb[q] == sb[i]:
                d = max(d, lv[q])
            else:
                assert sb[q] < sb[i], "a unit reads a superblock after its own in raster order"
                sdeps[i].add(int(sb[q]))
        lv[i] = d + 1
    modes = fr.units["mode"].astype(np.int64)
    perm = np.lexsort((fr.units["txtp"], modes, fr.units["pred"], fr.units["tx"], lv, sb))
    sbs = np.unique(sb)
    sbidx = {int(v): k for k, v in enumerate(sbs)}
    grp = sb[perm] * 4096 + lv[perm]
    cut = np.concatenate([[0], np.nonzero(np.diff(grp))[0] + 1, [n]]).astype(np.int32)
    n_lvl = len(cut) - 1
    class_start = np.zeros((n_lvl, abi.N_TX + 1), np.int32)
    tx = fr.units["tx"][perm]
    for g in range(n_lvl):
        class_start[g, 1:] = np.cumsum(np.bincount(tx[cut[g]:cut[g + 1]], minlength=abi.N_TX))
    gsb = sb[perm][cut[:-1]]
    sb_level_start = np.searchsorted(gsb, sbs).astype(np.int32)
    sb_level_start = np.concatenate([sb_level_start, [n_lvl]]).astype(np.int32)
    per_sb = [set() for _ in sbs]
    for i in range(n):
        per_sb[sbidx[int(sb[i])]] |= sdeps[i]
    dep_lists = [sorted(sbidx[d] for d in x) for x in per_sb]
    sb_dep_start = np.concatenate([[0], np.cumsum([len(x) for x in dep_lists])]).astype(np.int32)
    sb_deps = np.array([d for x in dep_lists for d in x], np.int32)
    return perm, cut, class_start, sb_level_start, sb_dep_start, sb_deps


class DeviceIntraFrame:
    """An IntraFrame on one GPU; launch() runs the whole wavefront
    (dav1d_gpu_recon_intra_frame_*) on a stream."""

    MODES = ("persistent", "levels", "fused", "staged", "sb", "lead")

    def __init__(self, fr, device="cuda:0", top_fill=0x5A, mode="persistent", task_groups=False):
        """mode: persistent -- one launch per frame (DGPU_IS_PERSISTENT), a
        wave waits for the tasks of its units' producers (dataflow); levels --
        the same launch, a wave waits for the whole previous level; fused --
        one launch per level (DGPU_IS_FUSED); staged -- edge stage, unit
        batch and backup runs per level; sb -- one launch per frame, a
        workgroup per superblock (DGPU_IS_SB, sb_schedule): units, records
        and the schedule in superblock order (units_frame_order() maps the
        rewritten units back).  task_groups: the schedule's task_group bytes
        (prediction kind and coded intra mode per unit), so a wave task of the
        persistent kernels runs one mode's code path (measured neutral on
        the 4K frames: 17.5 against 17.8 ms with one tile, 11.4 against 11.0
        with 2x2 tiles, so off by default).  lead -- persistent with
        DGPU_IS_LEVEL0_BATCH: level 0 and each next level of >= 2048 units
        as fused launches ahead of the persistent kernel."""
        assert mode in self.MODES
        lead = mode == "lead"
        dataflow = mode in ("persistent", "lead")
        self.sb = mode == "sb"
        mode = "persistent" if mode in ("levels", "sb", "lead") else mode
        import torch
        self.torch = torch
        self.perm = None
        if self.sb:   # the same frame in superblock order
            import copy
            perm, cut, cls_start, sls, sds, sdeps = sb_schedule(fr)
            fr = copy.copy(fr)
            fr.units, fr.recs = fr.units[perm], fr.recs[perm].copy()
            fr.recs["unit"] = np.arange(len(perm))
            fr.unit_start, fr.class_start, fr.rec_start = cut, cls_start, cut.copy()
            fr.run_start = np.zeros(len(cut), np.int32)
            if getattr(fr, "aux", None) is not None:
                fr.aux = fr.aux[perm]
            self.perm = perm
            self._sb = [np.ascontiguousarray(a, np.int32) for a in (sls, sds, sdeps if len(sdeps) else np.zeros(1))]
            self.n_sb = len(sls) - 1
        self.fr = fr
        dev = torch.device(device)
        hbd = fr.cfg.bpc != 8
        pdt = torch.int16 if hbd else torch.uint8
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).to(dev)   # noqa: E731
        self.units0 = fr.units.copy()
        self.units = up(fr.units.view(np.uint8))
        self.coefs = up(fr.coefs.view(np.int16 if not hbd else np.int32))
        self.edges = up(fr.edges.view(np.int16) if hbd else fr.edges)
        self.recs = up(fr.recs.view(np.uint8))
        self.runs = up(fr.runs.view(np.uint8)) if len(fr.runs) else torch.zeros(16, dtype=torch.uint8, device=dev)
        pad = getattr(fr, "dst_pad", 0)
        self.dst = [torch.zeros((h + pad, w + pad), dtype=pdt, device=dev) for (w, h) in fr.plane_wh]
        self.top = [torch.full(s, top_fill, dtype=pdt, device=dev) for s in fr.top_rows]
        self.refs = [[up(a.view(np.int16) if hbd else a) for a in rp] for rp in (fr.refs or [])]
        d = [t.data_ptr() for t in self.dst]
        self.rb = frame_batch(fr, d, self.units.data_ptr(), self.coefs.data_ptr(), self.edges.data_ptr(),
                              [[t.data_ptr() for t in rp] for rp in self.refs])
        self.eb = edge_batch(fr, d, [t.data_ptr() for t in self.top], self.units.data_ptr(),
                             self.edges.data_ptr(), self.recs.data_ptr())
        self._host = [np.ascontiguousarray(a, dtype=np.int32) for a in
                      (fr.unit_start, fr.class_start, fr.rec_start, fr.run_start)]
        s = abi.IntraSchedule()
        s.n_levels = len(fr.unit_start) - 1
        s.flags = {"persistent": abi.IS_FUSED | abi.IS_PERSISTENT, "fused": abi.IS_FUSED, "staged": 0}[mode]
        if lead:
            s.flags |= abi.IS_LEVEL0_BATCH
        if self.sb:
            s.flags |= abi.IS_SB
            s.n_sb = self.n_sb
            s.sb_level_start, s.sb_dep_start, s.sb_deps = (a.ctypes.data for a in self._sb)
        s.unit_start, s.class_start, s.rec_start, s.run_start = (a.ctypes.data for a in self._host)
        if task_groups:
            self._tg = task_group_bytes(fr)
            s.task_group = self._tg.ctypes.data
        s.runs = self.runs.data_ptr()
        if mode == "persistent" and dataflow and fr.dep_start is not None:
            self._host += [np.ascontiguousarray(fr.dep_start, np.int32),
                           np.ascontiguousarray(fr.deps if len(fr.deps) else np.zeros(1, np.int32), np.int32)]
            s.dep_start, s.deps = self._host[-2].ctypes.data, self._host[-1].ctypes.data
        self.sched = s
        self.lib = abi.load_lib()
        self.workspace = None
        if mode == "persistent":
            nb = self.lib.dav1d_gpu_intra_workspace_bytes(ctypes.byref(s), len(fr.units))
            if nb < 0:
                raise RuntimeError(f"dav1d_gpu_intra_workspace_bytes failed: {nb}")
            self.workspace = torch.zeros(max(int(nb), 16), dtype=torch.uint8, device=dev)
            s.workspace, s.workspace_bytes = self.workspace.data_ptr(), int(nb)

    def units_frame_order(self):
        """The device's (rewritten) units in the IntraFrame's level order."""
        u = self.units.cpu().numpy().view(self.fr.units.dtype)
        if self.perm is None:
            return u
        out = np.empty_like(u)
        out[self.perm] = u
        return out

    def flow_error(self):
        """The persistent kernel's give-up flag (int32 [1] of the workspace)."""
        if self.workspace is None:
            return 0
        return int(self.workspace[4:8].cpu().numpy().view(np.int32)[0])

    def reset(self):
        """Restore the inputs the wavefront consumes (unit modes / angles are
        rewritten, coefficients kept: zero_coefs is off)."""
        self.units.copy_(self.torch.from_numpy(self.units0.view(np.uint8)))
        for t in self.dst:
            t.zero_()

    def launch(self, stream=None):
        s = stream if stream is not None else self.torch.cuda.current_stream()
        fn = getattr(self.lib, f"dav1d_gpu_recon_intra_frame_{8 if self.fr.cfg.bpc == 8 else 16}bpc")
        rc = fn(ctypes.byref(self.rb), ctypes.byref(self.eb), ctypes.byref(self.sched),
                ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"dav1d_gpu_recon_intra_frame failed: {rc}")

    def planes_host(self):
        out = []
        for p, t in enumerate(self.dst):
            w, h = self.fr.plane_wh[p]
            a = t[:h, :w].cpu().numpy()
            out.append(a if self.fr.cfg.bpc == 8 else a.view(np.uint16))
        return out


class Recorder:
    """The batch recorder (dav1d_gpu_recorder_*, csrc/recorder.hip): blocks and
    residuals as recon_b_* would hand them over, one flush per frame."""

    def __init__(self, bpc, bitdepth_max, width, height, device_index=0):
        self.lib = abi.load_lib()
        self.bpc = bpc
        self.h = self.lib.dav1d_gpu_recorder_new(bpc, bitdepth_max, width, height, device_index)
        if not self.h:
            raise RuntimeError("dav1d_gpu_recorder_new failed")

    def close(self):
        if self.h:
            self.lib.dav1d_gpu_recorder_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def block(self, rb):
        rc = self.lib.dav1d_gpu_rec_block(self.h, ctypes.byref(rb))
        if rc:
            raise ValueError(f"dav1d_gpu_rec_block: {rc}")

    def block_aux(self, rb, data):
        """dav1d_gpu_rec_block_aux: a block with its kind's data (bytes or None)."""
        buf = None if data is None else ctypes.create_string_buffer(bytes(data), len(data))
        rc = self.lib.dav1d_gpu_rec_block_aux(self.h, ctypes.byref(rb), buf, 0 if data is None else len(data))
        if rc:
            raise ValueError(f"dav1d_gpu_rec_block_aux: {rc}")

    def residual(self, plane, x, y, tx, txtp, eob, coef):
        c = np.ascontiguousarray(coef, dtype=np.int16 if self.bpc == 8 else np.int32)
        rc = self.lib.dav1d_gpu_rec_residual(self.h, plane, x, y, tx, txtp, eob, c.ctypes.data)
        if rc:
            raise ValueError(f"dav1d_gpu_rec_residual: {rc}")

    def flush(self, dst, refs, stream):
        """dst: 3 device tensors (h, w); refs: list of [3 device tensors] with
        their picture origin offsets as (tensor, origin_px) pairs, or None."""
        bpp = 1 if self.bpc == 8 else 2
        d = (abi.Plane * 3)()
        for p, t in enumerate(dst):
            d[p].data, d[p].stride, d[p].w, d[p].h = t.data_ptr(), t.shape[1] * bpp, t.shape[1], t.shape[0]
        r = ((abi.Plane * 3) * abi.MAX_REFS)()
        for k, rp in enumerate(refs or []):
            for p, (t, org, w, h) in enumerate(rp):
                r[k][p].data, r[k][p].stride, r[k][p].w, r[k][p].h = t.data_ptr() + org * bpp, t.shape[1] * bpp, w, h
        rc = self.lib.dav1d_gpu_recorder_flush(self.h, ctypes.byref(d), ctypes.byref(r),
                                               ctypes.c_void_p(stream.cuda_stream))
        if rc:
            raise RuntimeError(f"dav1d_gpu_recorder_flush: {rc}")

    def set_top_edge(self, tops, sb128=False):
        """dav1d_gpu_recorder_set_top_edge: 3 device tensors (sb rows - 1 or
        more, superblock-aligned width) the flushes back superblock-bottom
        rows up to and read superblock-top rows from; None turns it off."""
        if tops is None:
            rc = self.lib.dav1d_gpu_recorder_set_top_edge(self.h, None, int(sb128))
        else:
            bpp = 1 if self.bpc == 8 else 2
            t = (abi.Plane * 3)()
            for p, a in enumerate(tops):
                t[p].data, t[p].stride, t[p].w, t[p].h = a.data_ptr(), a.shape[1] * bpp, a.shape[1], a.shape[0]
            rc = self.lib.dav1d_gpu_recorder_set_top_edge(self.h, ctypes.byref(t), int(sb128))
        if rc:
            raise ValueError(f"dav1d_gpu_recorder_set_top_edge: {rc}")

    def status(self):
        """The last flush's outcome (dav1d_gpu_recorder_status): 0, -6 (its
        wavefront gave up waiting: incomplete picture) or -3."""
        return self.lib.dav1d_gpu_recorder_status(self.h)

    def flush_rc(self, dst, refs, stream):
        """flush() returning the library's code instead of raising."""
        try:
            self.flush(dst, refs, stream)
            return 0
        except RuntimeError as e:
            return int(str(e).rsplit(":", 1)[1])

    def stats(self):
        n, lv = ctypes.c_int32(), ctypes.c_int32()
        self.lib.dav1d_gpu_recorder_stats(self.h, ctypes.byref(n), ctypes.byref(lv))
        return n.value, lv.value

    def prep_ms(self):
        """Device time of the last flush's prep (upload, cut, levels, sort,
        scatter on the recorder's own stream), ms."""
        ms = ctypes.c_float()
        self.lib.dav1d_gpu_recorder_prep_ms(self.h, ctypes.byref(ms))
        return ms.value


def replay(rec, fr, rows=None):
    """Feed an IntraFrame's blocks and residuals to a Recorder, in decode
    order, the way recon_b_* would (coefficients expanded to the reference's
    inv_txfm_add layout: column-major, min(h,32) rows).  rows=(y0, y1): only
    the blocks (and their residuals) of luma superblock rows [y0, y1) in
    pixels (chroma: the co-located half), for flushes per superblock row."""
    def inside(p, y):
        if rows is None:
            return True
        s = 1 if p else 0
        return (rows[0] >> s) <= y < (rows[1] >> s)
    bx = getattr(fr, "block_aux", None) or [False] * len(fr.blocks)
    for t, data in zip(fr.blocks, bx):
        if not inside(t[0], t[2]):
            continue
        rb = abi.RecBlock()
        (rb.plane, rb.x, rb.y, rb.w, rb.h, rb.tx, rb.kind, rb.tile_x0, rb.tile_y0, rb.tile_x1, rb.tile_y1,
         rb.mvx[0], rb.mvx[1], rb.mvy[0], rb.mvy[1], rb.ref[0], rb.ref[1], rb.filter2d, rb.weight, rb.mode,
         rb.angle, rb.cfl_alpha, rb.flags) = t
        if data is False:
            rec.block(rb)
        else:
            rec.block_aux(rb, data)
    u = fr.dec_units
    for i in np.nonzero(u["txtp"] != abi.NO_RESIDUAL)[0]:
        p = int(u["plane"][i])
        w = fr.plane_wh[p][0] + getattr(fr, "dst_pad", 0)   # dst_off's row pitch
        y, x = divmod(int(u["dst_off"][i]), w)
        if not inside(p, y):
            continue
        tw, th = abi.TX_WH[int(u["tx"][i])]
        sw, sh = min(tw, 32), min(th, 32)
        cf = np.zeros(sw * sh, np.int64)
        nzw, nzh, o = int(u["nzw"][i]), int(u["nzh"][i]), int(u["coef_off"][i])
        if nzw == 0:
            cf[0] = fr.coefs[o]
            eob = 0 if int(u["txtp"][i]) == abi.DCT_DCT else 1
        else:
            reg = fr.coefs[o:o + nzw * nzh].reshape(nzw, nzh)   # [x][y]
            for xx in range(nzw):
                cf[xx * sh:xx * sh + nzh] = reg[xx]
            eob = 1
        rec.residual(p, x, y, int(u["tx"][i]), int(u["txtp"][i]), eob, cf)
