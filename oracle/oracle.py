"""ctypes front-end of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product.  See dsp_ref.c's header
for what this restates and why parity is unpinned against the reference
binary.
"""
import ctypes
import os
import sys
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _abi():
    pkg = sys.modules.get("dav1d_mirror_amd")
    if pkg is None:
        raise RuntimeError("load the dav1d_mirror_amd package first (tests/conftest.py does)")
    return pkg.abi


def load():
    global _LIB
    if _LIB is None:
        p = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(p):
            raise RuntimeError(f"{p} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(p)
        abi = _abi()
        for bpc in (8, 16):
            f = getattr(L, f"oracle_recon_units_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(abi.FrameBatch), ctypes.c_int, ctypes.c_int]
            f.restype = ctypes.c_int
            f = getattr(L, f"oracle_recon_tiles_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(abi.TileBatch), ctypes.c_int, ctypes.c_int]
            f.restype = ctypes.c_int
            f = getattr(L, f"oracle_prepare_intra_edges_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(abi.IntraEdgeBatch)]
            f.restype = ctypes.c_int
            f = getattr(L, f"oracle_backup_ipred_edge_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(abi.IntraEdgeBatch), ctypes.c_void_p, ctypes.c_int]
            f.restype = ctypes.c_int
            f = getattr(L, f"oracle_recon_intra_frame_{bpc}bpc")
            f.argtypes = [ctypes.POINTER(abi.FrameBatch), ctypes.POINTER(abi.IntraEdgeBatch), ctypes.c_void_p,
                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
            f.restype = ctypes.c_int
        _LIB = L
    return _LIB


class HostFrame:
    """The same FrameData reconstructed on the CPU by the oracle."""

    def __init__(self, fd):
        abi = _abi()
        self.fd = fd
        pdt = fd.cfg.pixel_dtype
        if getattr(fd, "dst_init", None) is not None:
            self.dst = [a.copy() for a in fd.dst_init]
        else:
            self.dst = [np.zeros((h, w), pdt) for (w, h) in fd.plane_wh]
        self.units = np.ascontiguousarray(fd.units)
        self.coefs = fd.coefs.copy()
        self.edges = np.ascontiguousarray(fd.edges)
        self.refs = fd.refs
        bpp = 1 if fd.cfg.bpc == 8 else 2
        b = abi.FrameBatch()
        for p in range(3):
            w, h = fd.plane_wh[p]
            b.dst[p].data = self.dst[p].ctypes.data
            b.dst[p].stride = w * bpp
            b.dst[p].w, b.dst[p].h = w, h
            for r in range(len(self.refs)):
                a = self.refs[r][p]
                b.ref[r][p].data = a.ctypes.data + fd.ref_origin_offset(p) * bpp
                b.ref[r][p].stride = a.shape[1] * bpp
                b.ref[r][p].w, b.ref[r][p].h = w, h
        b.units = self.units.ctypes.data
        b.n_units = fd.n_units
        for i in range(abi.N_TX + 1):
            b.class_start[i] = int(fd.class_start[i])
        b.coef = self.coefs.ctypes.data
        b.edges = self.edges.ctypes.data
        b.bitdepth_max = fd.cfg.bitdepth_max if fd.cfg.bpc == 16 else 255
        b.zero_coefs = 0
        self.cfl_luma = np.ascontiguousarray(fd.cfl_luma)
        b.cfl_luma.data = self.cfl_luma.ctypes.data
        b.cfl_luma.stride = self.cfl_luma.shape[1] * bpp
        b.cfl_luma.w, b.cfl_luma.h = fd.plane_wh[0]
        b.cfl_ss = 3
        self.aux = self.aux_pool = None
        if getattr(fd, "aux", None) is not None:
            self.aux = np.ascontiguousarray(fd.aux, dtype=np.int32)
            self.aux_pool = np.ascontiguousarray(fd.aux_pool, dtype=np.uint8)
            b.aux = self.aux.ctypes.data
            b.aux_pool = self.aux_pool.ctypes.data
        if getattr(fd, "class_warp", None) is not None:
            for i in range(abi.N_TX):
                b.class_warp[i] = int(fd.class_warp[i])
        self.batch = b

    def run(self, u0=0, u1=None, threads=1):
        """Reconstruct units [u0, u1); `threads` > 1 splits the range over
        OS threads (ctypes releases the GIL during the call)."""
        L = load()
        fn = L.oracle_recon_units_8bpc if self.fd.cfg.bpc == 8 else L.oracle_recon_units_16bpc
        if u1 is None:
            u1 = self.fd.n_units
        # INTER_WMASK units write the seg masks their blocks' chroma units
        # read: run them first (re-running them below is idempotent)
        for i in np.nonzero(self.units["pred"][u0:u1] == _abi().PRED_INTER_WMASK)[0]:
            fn(ctypes.byref(self.batch), int(u0 + i), int(u0 + i + 1))
        if threads <= 1:
            fn(ctypes.byref(self.batch), u0, u1)
            return
        bounds = np.linspace(u0, u1, threads + 1).astype(int)
        ts = [threading.Thread(target=fn, args=(ctypes.byref(self.batch), int(bounds[i]),
                                                int(bounds[i + 1]))) for i in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()


class HostTiles:
    """A TileData (dav1d_mirror_amd.tiles.build_tiles) reconstructed on the
    CPU by the oracle's tile walker: per tile, the reference's DSP calls for
    each pred (mc with recon_tmpl.c's emu_edge condition, intra, CfL, pal,
    warp, inter-intra) and each transform block."""

    def __init__(self, fd, td, zero_coefs=False):
        abi = _abi()
        self.fd, self.td = fd, td
        pdt = fd.cfg.pixel_dtype
        if getattr(fd, "dst_init", None) is not None:
            self.dst = [a.copy() for a in fd.dst_init]
        else:
            self.dst = [np.zeros((h, w), pdt) for (w, h) in fd.plane_wh]
        self.tiles = np.ascontiguousarray(td.tiles)
        self.preds = np.ascontiguousarray(td.preds)
        self.txs = np.ascontiguousarray(td.txs)
        self.coefs = td.coefs.copy()
        self.edges = np.ascontiguousarray(td.edges)
        self.aux_pool = None if td.aux_pool is None else np.ascontiguousarray(td.aux_pool)
        self.refs = fd.refs
        self.cfl_luma = np.ascontiguousarray(fd.cfl_luma)
        bpp = 1 if fd.cfg.bpc == 8 else 2
        b = abi.TileBatch()
        for p in range(3):
            w, h = fd.plane_wh[p]
            b.dst[p].data = self.dst[p].ctypes.data
            b.dst[p].stride = w * bpp
            b.dst[p].w, b.dst[p].h = w, h
            for r in range(len(self.refs)):
                a = self.refs[r][p]
                b.ref[r][p].data = a.ctypes.data + fd.ref_origin_offset(p) * bpp
                b.ref[r][p].stride = a.shape[1] * bpp
                b.ref[r][p].w, b.ref[r][p].h = w, h
        b.tiles = self.tiles.ctypes.data
        b.n_tiles = len(self.tiles)
        b.n_tiles_huge = td.n_tiles_huge
        b.bitdepth_max = fd.cfg.bitdepth_max if fd.cfg.bpc == 16 else 255
        b.preds = self.preds.ctypes.data
        b.txs = self.txs.ctypes.data
        b.coef = self.coefs.ctypes.data
        b.edges = self.edges.ctypes.data
        b.aux_pool = None if self.aux_pool is None else self.aux_pool.ctypes.data
        b.cfl_luma.data = self.cfl_luma.ctypes.data
        b.cfl_luma.stride = self.cfl_luma.shape[1] * bpp
        b.cfl_luma.w, b.cfl_luma.h = fd.plane_wh[0]
        b.cfl_ss = 3
        b.zero_coefs = 1 if zero_coefs else 0
        self.batch = b

    def run(self, threads=1):
        L = load()
        fn = L.oracle_recon_tiles_8bpc if self.fd.cfg.bpc == 8 else L.oracle_recon_tiles_16bpc
        n = len(self.tiles)
        if threads <= 1:
            fn(ctypes.byref(self.batch), 0, n)
            return
        bounds = np.linspace(0, n, threads + 1).astype(int)
        ts = [threading.Thread(target=fn, args=(ctypes.byref(self.batch), int(bounds[i]), int(bounds[i + 1])))
              for i in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()


# ---------------------------------------------------------------------------
# Direct access to the oracle's DSP tables (same layouts as dav1d_gpu.h) for
# property tests.
class _MC(ctypes.Structure):
    _fields_ = [("mc", ctypes.c_void_p * 10), ("mc_scaled", ctypes.c_void_p * 10),
                ("mct", ctypes.c_void_p * 10), ("mct_scaled", ctypes.c_void_p * 10),
                ("avg", ctypes.c_void_p), ("w_avg", ctypes.c_void_p), ("mask", ctypes.c_void_p),
                ("w_mask", ctypes.c_void_p * 3), ("blend", ctypes.c_void_p),
                ("blend_v", ctypes.c_void_p), ("blend_h", ctypes.c_void_p),
                ("warp8x8", ctypes.c_void_p), ("warp8x8t", ctypes.c_void_p),
                ("emu_edge", ctypes.c_void_p), ("resize", ctypes.c_void_p)]


class _ITX(ctypes.Structure):
    _fields_ = [("itxfm_add", (ctypes.c_void_p * 17) * 19)]


def mc_table(bpc):
    L = load()
    t = _MC()
    getattr(L, f"oracle_mc_dsp_init_{bpc}bpc")(ctypes.byref(t))
    return t


def itx_table(bpc, bits=None):
    L = load()
    t = _ITX()
    getattr(L, f"oracle_itx_dsp_init_{bpc}bpc")(ctypes.byref(t), bits or (8 if bpc == 8 else 10))
    return t


def call_put(tbl, f, dst, src, src_off, w, h, mx, my, bdmax=None):
    """mc[f](dst, dst_stride, src + src_off, src_stride, w, h, mx, my[, bdmax])."""
    hbd = dst.dtype == np.uint16
    args = [ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p, ctypes.c_ssize_t] + [ctypes.c_int] * 4
    if hbd:
        args.append(ctypes.c_int)
    fn = ctypes.CFUNCTYPE(None, *args)(tbl.mc[f])
    a = [dst.ctypes.data, dst.strides[0], src.ctypes.data + src_off * src.itemsize, src.strides[0],
         w, h, mx, my]
    if hbd:
        a.append(bdmax)
    fn(*a)


def call_prep(tbl, f, tmp, src, src_off, w, h, mx, my, bdmax=None):
    hbd = src.dtype == np.uint16
    args = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ssize_t] + [ctypes.c_int] * 4
    if hbd:
        args.append(ctypes.c_int)
    fn = ctypes.CFUNCTYPE(None, *args)(tbl.mct[f])
    a = [tmp.ctypes.data, src.ctypes.data + src_off * src.itemsize, src.strides[0], w, h, mx, my]
    if hbd:
        a.append(bdmax)
    fn(*a)


def call_itx(tbl, tx, tp, dst, coef, eob, bdmax=None):
    hbd = dst.dtype == np.uint16
    args = [ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p, ctypes.c_int]
    if hbd:
        args.append(ctypes.c_int)
    fn = ctypes.CFUNCTYPE(None, *args)(tbl.itxfm_add[tx][tp])
    a = [dst.ctypes.data, dst.strides[0], coef.ctypes.data, eob]
    if hbd:
        a.append(bdmax)
    fn(*a)


def prepare_intra_edges(case):
    """An intra.EdgeCase through the oracle's dav1d_prepare_intra_edges
    restatement; returns the (units, edge pool) it leaves."""
    import dav1d_mirror_amd.intra as intra
    abi = _abi()
    L = load()
    pics = [np.ascontiguousarray(a) for a in case.pics]
    tops = [np.ascontiguousarray(a) for a in case.top_edge]
    units = case.units.copy()
    edges = case.edges.copy()
    recs = np.ascontiguousarray(case.recs)
    b = intra.fill_batch(abi.IntraEdgeBatch(), case, [a.ctypes.data for a in pics],
                         [a.ctypes.data for a in tops], units.ctypes.data, edges.ctypes.data,
                         recs.ctypes.data)
    fn = getattr(L, f"oracle_prepare_intra_edges_{8 if case.bpc == 8 else 16}bpc")
    rc = fn(ctypes.byref(b))
    assert rc == 0
    return units, edges


class HostIntraFrame:
    """An intra.IntraFrame reconstructed by the oracle in the decoder's own
    order: per transform block prepare_intra_edges then the DSP calls, the
    top_edge backup at each superblock-row end (oracle_recon_intra_frame)."""

    def __init__(self, fr, top_fill=0x5A):
        import dav1d_mirror_amd.intra as intra
        abi = _abi()
        self.fr = fr
        pdt = fr.cfg.pixel_dtype
        pad = getattr(fr, "dst_pad", 0)   # room for transform blocks overhanging the picture
        self._dst = [np.zeros((h + pad, w + pad), pdt) for (w, h) in fr.plane_wh]
        self.dst = [a[:h, :w] for a, (w, h) in zip(self._dst, fr.plane_wh)]
        self.top = [np.full(s, top_fill, pdt) for s in fr.top_rows]
        self.units = fr.units.copy()
        self.coefs = fr.coefs.copy()
        self.edges = fr.edges.copy()
        self.recs = np.ascontiguousarray(fr.recs)
        self.steps = np.ascontiguousarray(fr.steps, dtype=np.int32)
        self.unit_rec = np.ascontiguousarray(fr.unit_rec, dtype=np.int32)
        self.oruns = np.ascontiguousarray(fr.oracle_runs) if len(fr.oracle_runs) else np.zeros(1, abi.EDGE_BACKUP_DTYPE)
        d = [a.ctypes.data for a in self._dst]
        # recorder kinds with block data: per-unit aux offsets and a writable
        # pool (INTER_WMASK units write the seg mask their chroma units read)
        self.aux = None if getattr(fr, "aux", None) is None else np.ascontiguousarray(fr.aux, dtype=np.int32)
        self.aux_pool = None if self.aux is None else np.ascontiguousarray(fr.aux_pool, dtype=np.uint8).copy()
        self.rb = intra.frame_batch(fr, d, self.units.ctypes.data, self.coefs.ctypes.data, self.edges.ctypes.data,
                                    [[a.ctypes.data for a in rp] for rp in (fr.refs or [])],
                                    None if self.aux is None else self.aux.ctypes.data,
                                    None if self.aux is None else self.aux_pool.ctypes.data)
        self.eb = intra.edge_batch(fr, d, [a.ctypes.data for a in self.top], self.units.ctypes.data,
                                   self.edges.ctypes.data, self.recs.ctypes.data)

    def run(self):
        fn = getattr(load(), f"oracle_recon_intra_frame_{8 if self.fr.cfg.bpc == 8 else 16}bpc")
        rc = fn(ctypes.byref(self.rb), ctypes.byref(self.eb), self.steps.ctypes.data, len(self.steps),
                self.unit_rec.ctypes.data, self.oruns.ctypes.data)
        assert rc == 0

    def run_levels(self):
        """The same frame in the wavefront's level order (edges, units, then
        backup runs per level), on the CPU: checks the schedule itself."""
        abi = _abi()
        fr = self.fr
        L = load()
        sfx = 8 if fr.cfg.bpc == 8 else 16
        prep = getattr(L, f"oracle_prepare_intra_edges_{sfx}bpc")
        recon = getattr(L, f"oracle_recon_units_{sfx}bpc")
        backup = getattr(L, f"oracle_backup_ipred_edge_{sfx}bpc")
        runs = np.ascontiguousarray(fr.runs) if len(fr.runs) else np.zeros(1, abi.EDGE_BACKUP_DTYPE)
        rec_sz = fr.recs.dtype.itemsize
        run_sz = runs.dtype.itemsize
        e = abi.IntraEdgeBatch.from_buffer_copy(self.eb)
        for lv in range(fr.n_levels):
            r0, r1 = int(fr.rec_start[lv]), int(fr.rec_start[lv + 1])
            e.recs = self.recs.ctypes.data + r0 * rec_sz
            e.n_recs = r1 - r0
            prep(ctypes.byref(e))
            recon(ctypes.byref(self.rb), int(fr.unit_start[lv]), int(fr.unit_start[lv + 1]))
            b0, b1 = int(fr.run_start[lv]), int(fr.run_start[lv + 1])
            backup(ctypes.byref(self.eb), runs.ctypes.data + b0 * run_sz, b1 - b0)


    def run_dataflow(self, seed=0):
        """Unit by unit in a random order that respects only the producer
        lists (fr.dep_start / fr.deps): what the persistent kernel's
        dataflow waits allow.  A unit that ends a superblock row backs its
        bottom row up right after it, as the fused kernel does."""
        import heapq
        abi = _abi()
        fr = self.fr
        L = load()
        sfx = 8 if fr.cfg.bpc == 8 else 16
        prep = getattr(L, f"oracle_prepare_intra_edges_{sfx}bpc")
        recon = getattr(L, f"oracle_recon_units_{sfx}bpc")
        backup = getattr(L, f"oracle_backup_ipred_edge_{sfx}bpc")
        n = len(fr.units)
        ds, dp = fr.dep_start, fr.deps
        users = [[] for _ in range(n)]
        waiting = np.diff(ds).astype(np.int64)
        for u in range(n):
            for q in dp[ds[u]:ds[u + 1]]:
                users[int(q)].append(u)
        rng = np.random.default_rng(seed)
        pri = rng.random(n)
        ready = [(pri[u], u) for u in range(n) if waiting[u] == 0]
        heapq.heapify(ready)
        rec_sz = fr.recs.dtype.itemsize
        e = abi.IntraEdgeBatch.from_buffer_copy(self.eb)
        run = np.zeros(1, abi.EDGE_BACKUP_DTYPE)
        done = 0
        while ready:
            _, u = heapq.heappop(ready)
            done += 1
            if fr.unit_rec[u] >= 0:
                e.recs = self.recs.ctypes.data + int(fr.unit_rec[u]) * rec_sz
                e.n_recs = 1
                prep(ctypes.byref(e))
            recon(ctypes.byref(self.rb), u, u + 1)
            un = fr.units[u]
            p = int(un["plane"])
            w = fr.plane_wh[p][0]
            tw, th = abi.TX_WH[un["tx"]]
            y, x = divmod(int(un["dst_off"]), w)
            sh = 1 << fr.sb_log2[p]
            if fr.cfg.sb_edge_backup and (y + th) % sh == 0 and y + th < fr.plane_wh[p][1]:
                run[0] = (p, (y + th) // sh - 1, x, tw)
                backup(ctypes.byref(self.eb), run.ctypes.data, 1)
            for v in users[u]:
                waiting[v] -= 1
                if waiting[v] == 0:
                    heapq.heappush(ready, (pri[v], v))
        assert done == n   # the producer graph is acyclic


def apply_grain(case):
    """A grain.GrainCase through the oracle's dav1d_apply_grain restatement:
    returns (output planes, grain LUTs [3][73][82], scaling LUTs [3][4096])."""
    import dav1d_mirror_amd.grain as grain
    abi = _abi()
    L = load()
    sfx = 8 if case.bpc == 8 else 16
    ins = [np.ascontiguousarray(a) for a in case.planes]
    outs = [np.zeros_like(a) for a in ins]
    b = grain.fill_batch(abi.FilmGrainBatch(), case, [(a.ctypes.data, a.shape[1]) for a in ins],
                         [(a.ctypes.data, a.shape[1]) for a in outs], None)
    fn = getattr(L, f"oracle_apply_grain_{sfx}bpc")
    fn.argtypes = [ctypes.POINTER(abi.FilmGrainBatch)]
    fn.restype = ctypes.c_int
    assert fn(ctypes.byref(b)) == 0
    g = np.zeros((3, abi.GRAIN_H, abi.GRAIN_W), np.int16)
    sc = np.zeros((3, 4096), np.uint8)
    prep = getattr(L, f"oracle_prep_grain_{sfx}bpc")
    prep.argtypes = [ctypes.POINTER(abi.FilmGrainData), ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    prep.restype = ctypes.c_int
    d = abi.FilmGrainData.from_buffer_copy(case.data)
    assert prep(ctypes.byref(d), case.layout, case.bitdepth_max, g.ctypes.data, sc.ctypes.data) == 0
    return outs, g, sc


def cdef_frame(case, sb128=0):
    """A cdef.CdefCase through the oracle's dav1d_filter_sbrow_cdef /
    dav1d_cdef_brow restatement (in place on a copy, with the reference's
    line and column backups); returns the output planes over the 8x8 grid."""
    import dav1d_mirror_amd.cdef as cdef
    abi = _abi()
    L = load()
    sfx = 8 if case.bpc == 8 else 16
    ins = [np.ascontiguousarray(a) for a in case.planes]
    outs = [np.zeros_like(a) for a in ins]
    idx = np.ascontiguousarray(case.cdef_idx, np.int8)
    nsk = np.ascontiguousarray(case.noskip, np.uint8)
    f = cdef.fill_frame(abi.CdefFrame(), case, [(a.ctypes.data, a.shape[1]) for a in ins],
                        [(a.ctypes.data, a.shape[1]) for a in outs], idx.ctypes.data, nsk.ctypes.data)
    fn = getattr(L, f"oracle_cdef_frame_{sfx}bpc")
    fn.argtypes = [ctypes.POINTER(abi.CdefFrame), ctypes.c_int]
    fn.restype = ctypes.c_int
    assert fn(ctypes.byref(f), sb128) == 0
    return outs


def cdef_dsp(bpc):
    """(dir, fb[3]) of the oracle's bitfn(dav1d_cdef_dsp_init) as ctypes callables."""
    L = load()
    hbd = [] if bpc == 8 else [ctypes.c_int]
    dir_t = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_ssize_t, ctypes.POINTER(ctypes.c_uint), *hbd)
    fb_t = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, *hbd)

    class Ctx(ctypes.Structure):
        _fields_ = [("dir", dir_t), ("fb", fb_t * 3)]
    c = Ctx()
    getattr(L, f"oracle_cdef_dsp_init_{bpc}bpc")(ctypes.byref(c))
    return c


def loopfilter_frame(case):
    """An lpf.LpfCase through the oracle's dav1d_loopfilter_sbrow_cols /
    _rows restatement, superblock row by superblock row; returns the planes."""
    import dav1d_mirror_amd.lpf as lpf
    abi = _abi()
    L = load()
    sfx = 8 if case.bpc == 8 else 16
    pics = [np.ascontiguousarray(a).copy() for a in case.planes]
    masks = np.ascontiguousarray(case.masks)
    level = np.ascontiguousarray(case.level)
    f = lpf.fill_frame(abi.LoopFilterFrame(), case, [(a.ctypes.data, a.shape[1]) for a in pics],
                       masks.ctypes.data, level.ctypes.data)
    fn = getattr(L, f"oracle_loopfilter_frame_{sfx}bpc")
    fn.argtypes = [ctypes.POINTER(abi.LoopFilterFrame), ctypes.c_int]
    fn.restype = ctypes.c_int
    assert fn(ctypes.byref(f), case.sb128) == 0
    return pics


def lr_dsp(bpc, bitdepth=None):
    """wiener[2] + sgr[3] of the oracle's bitfn(dav1d_loop_restoration_dsp_init) as ctypes callables."""
    abi = _abi()
    L = load()
    hbd = [] if bpc == 8 else [ctypes.c_int]
    fn_t = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                            ctypes.c_int, ctypes.POINTER(abi.LrParams), ctypes.c_int, *hbd)

    class Ctx(ctypes.Structure):
        _fields_ = [("wiener", fn_t * 2), ("sgr", fn_t * 3)]
    c = Ctx()
    getattr(L, f"oracle_loop_restoration_dsp_init_{bpc}bpc")(ctypes.byref(c), bitdepth or bpc)
    return c


def lr_frame(case):
    """An lr.LrCase through the oracle's dav1d_lr_sbrow restatement; returns the planes."""
    import dav1d_mirror_amd.lr as lr
    abi = _abi()
    L = load()
    sfx = 8 if case.bpc == 8 else 16
    ins = [np.ascontiguousarray(a) for a in case.ins]
    lpfs = [np.ascontiguousarray(a) for a in case.lpfs]
    outs = [np.zeros_like(a) for a in ins]
    f = lr.fill_frame(abi.LrFrame(), case, [(a.ctypes.data, a.shape[1]) for a in ins],
                      [(a.ctypes.data, a.shape[1]) for a in lpfs], [(a.ctypes.data, a.shape[1]) for a in outs],
                      [ctypes.addressof(u) for (u, _, _) in case.units])
    fn = getattr(L, f"oracle_lr_frame_{sfx}bpc")
    fn.argtypes = [ctypes.POINTER(abi.LrFrame)]
    fn.restype = ctypes.c_int
    assert fn(ctypes.byref(f)) == 0
    return outs


def resize_frame(case):
    """A superres.ResizeCase through the oracle's dav1d_filter_sbrow_resize
    walk (per superblock row); returns the upscaled planes."""
    import dav1d_mirror_amd.superres as sr
    abi = _abi()
    L = load()
    ins = [np.ascontiguousarray(a) for a in case.ins]
    outs = [np.zeros(sh, dtype=case.dtype) for sh in sr.out_shapes(case)]
    f = sr.fill(case, [(a.ctypes.data, a.shape[1]) for a in ins], [(a.ctypes.data, a.shape[1]) for a in outs])
    fn = getattr(L, f"oracle_resize_frame_{8 if case.bpc == 8 else 16}bpc")
    fn.argtypes = [ctypes.POINTER(abi.ResizeFrame)]
    fn.restype = ctypes.c_int
    assert fn(ctypes.byref(f)) == 0
    return [o[:, :case.dst_w[p]] for p, o in enumerate(outs)]
