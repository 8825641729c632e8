"""Superblock-tile batches (Dav1dGpuTileBatch, include/dav1d_gpu.h) built
from a FrameData.

This is the producer side of the tile ABI -- what a batch recorder at
recon_b_inter / recon_b_intra (src/recon_tmpl.c:1598, :1195) emits per
superblock: one Dav1dGpuPred per prediction block (one mc call per block and
reference, as recon_tmpl.c's mc() makes; intra / CfL / palette / warp /
inter-intra per transform block as in the unit batch), one Dav1dGpuTx per
transform block with a residual, the coefficients and intra edges laid out
tile by tile, and the per-tile lane bases the kernel's lane maps use.

Tiles: luma 64x64 (a superblock), chroma 32x32 (its 4:2:0 chroma), in
superblock raster order with the three planes of a superblock together;
tiles holding 64-point transforms go last (n_tiles_huge).

Host-side numpy only; nothing here is timed.
"""
from dataclasses import dataclass

import numpy as np

from . import abi

TILE_DTYPE = np.dtype({
    "names": ["x", "y", "plane", "w4", "h4", "flags", "pred0", "tx0", "coef0", "edge0",
              "n_pred", "n_tx", "n_coef", "n_edge", "lanes_tx", "lanes_coop", "lanes_task",
              "lanes_coop_used", "reserved0", "reserved1"],
    "formats": ["<i2", "<i2", "u1", "u1", "u1", "u1", "<i4", "<i4", "<i4", "<i4",
                "<u2", "<u2", "<u2", "<u2", "<u2", "<u2", "<u2", "<u2", "<i4", "<i4"],
    "offsets": [0, 2, 4, 5, 6, 7, 8, 12, 16, 20, 24, 26, 28, 30, 32, 34, 36, 38, 40, 44],
    "itemsize": 48,
})

# Dav1dGpuPred: header, then the inter / intra union at offset 12 (every byte
# belongs to some field, so copies never carry uninitialised padding)
PRED_DTYPE = np.dtype({
    "names": ["kind", "x4", "y4", "w4", "h4", "bw4", "bh4", "lanes_log2", "lane0", "pad0",
              "src_x0", "src_x1", "src_y0", "src_y1", "mx0", "mx1", "my0", "my1", "filter2d",
              "ref0", "ref1", "weight", "aux",
              "edge_off", "angle", "mode", "alpha", "max_w", "max_h", "cfl_pad_wh", "pad2", "pad3"],
    "formats": ["u1", "u1", "u1", "u1", "u1", "u1", "u1", "u1", "<u2", "<u2",
                "<i2", "<i2", "<i2", "<i2", "u1", "u1", "u1", "u1", "u1",
                "u1", "u1", "u1", "<i4",
                "<i4", "<u2", "u1", "i1", "<u2", "<u2", "u1", "u1", "<u2"],
    "offsets": [0, 1, 2, 3, 4, 5, 6, 7, 8, 10,
                12, 14, 16, 18, 20, 21, 22, 23, 24,
                25, 26, 27, 28,
                12, 16, 18, 19, 20, 22, 24, 25, 26],
    "itemsize": 32,
})

TX_DTYPE = np.dtype([("w0", "<u4"), ("w1", "<u4")])

MAX_EDGE = 4608            # DGPU_TILE_MAX_EDGE
COOP_KINDS = (abi.PRED_INTRA, abi.PRED_CFL)
BLOCK_KINDS = abi.INTER_KINDS   # one pred per prediction block (mc once per block and reference)


def coop_lanes(w, h):
    """Group size of a cooperative pred: one 4x2 task per lane up to the
    1-D extent, 2..64 (the batch kernel's lanes_per_unit)."""
    w = np.asarray(w, np.int64)
    h = np.asarray(h, np.int64)
    g = np.minimum(w * h // 8, np.maximum(w, np.minimum(h, 32)))
    g = np.clip(g, 2, 64)
    return np.where(w * h >= 1024, 64, g)


def tx_lanes(w, h):
    return np.maximum(w, np.minimum(h, 32))


def task_rows(h, bpc):
    """R of the independent 4 x R tasks: 8 at 8 bpc when the pred is >= 8
    high, else 4."""
    return np.where((bpc == 8) & (np.asarray(h) >= 8), 8, 4)


def _seg_excl_cumsum(v, starts, lengths):
    """Exclusive cumsum of v restarting at every segment start."""
    cs = np.cumsum(v) - v
    return cs - np.repeat(cs[starts], lengths)


def _gather_ranges(src_start, n):
    """Concatenated index ranges [src_start[i], src_start[i] + n[i])."""
    n = np.asarray(n, np.int64)
    tot = int(n.sum())
    if tot == 0:
        return np.zeros(0, np.int64)
    dst_start = np.cumsum(n) - n
    return np.repeat(np.asarray(src_start, np.int64) - dst_start, n) + np.arange(tot)


@dataclass
class TileData:
    cfg: object
    tiles: np.ndarray
    preds: np.ndarray
    txs: np.ndarray
    coefs: np.ndarray
    edges: np.ndarray
    aux_pool: np.ndarray
    n_tiles_huge: int
    stats: dict


def build_tiles(fd):
    """The Dav1dGpuTileBatch arrays of frame `fd` (same pixels as its unit
    batch: same blocks, predictions and residuals)."""
    cfg = fd.cfg
    bpc = cfg.bpc
    u = fd.units
    n = len(u)
    pw = np.array([fd.plane_wh[p][0] for p in range(3)], np.int64)
    ph = np.array([fd.plane_wh[p][1] for p in range(3)], np.int64)
    plane = u["plane"].astype(np.int64)
    ux = u["dst_off"] % pw[plane]
    uy = u["dst_off"] // pw[plane]
    tw = np.array([abi.TX_WH[t][0] for t in range(abi.N_TX)], np.int64)[u["tx"]]
    th = np.array([abi.TX_WH[t][1] for t in range(abi.N_TX)], np.int64)[u["tx"]]
    bw = u["bw4"].astype(np.int64) * 4
    bh = u["bh4"].astype(np.int64) * 4
    pk = u["pred"].astype(np.int64)
    assert fd.src_xy is not None, "FrameData without src_xy (make_frame records it)"

    # tile of each unit: luma 64, chroma 32 (4:2:0), superblock raster order
    ts = np.array([64, 32, 32], np.int64)
    ncol = -(-pw[0] // 64)
    nrow = -(-ph[0] // 64)
    tcol = ux // ts[plane]
    trow = uy // ts[plane]
    tid = (trow * ncol + tcol) * 3 + plane
    n_tiles_all = int(nrow * ncol * 3)

    # ---- preds: one per block for the mc kinds, one per unit otherwise ----
    is_blk = np.isin(pk, BLOCK_KINDS)
    bx = (ux // bw) * bw
    by = (uy // bh) * bh
    rep = is_blk & (ux == bx) & (uy == by)        # the unit at the block's origin
    pred_of_unit = ~is_blk | rep
    pu = np.nonzero(pred_of_unit)[0]              # unit index representing each pred
    npred = len(pu)
    P = np.zeros(npred, PRED_DTYPE)
    kind = pk[pu]
    blkp = is_blk[pu]
    pwid = np.where(blkp, bw[pu], tw[pu])
    phei = np.where(blkp, bh[pu], th[pu])
    ptile = tid[pu]
    tile_x = tcol[pu] * ts[plane[pu]]
    tile_y = trow[pu] * ts[plane[pu]]
    P["kind"] = kind
    P["x4"] = (ux[pu] - tile_x) // 4
    P["y4"] = (uy[pu] - tile_y) // 4
    P["w4"] = pwid // 4
    P["h4"] = phei // 4
    P["bw4"] = u["bw4"][pu]
    P["bh4"] = u["bh4"][pu]
    assert np.all(P["x4"].astype(np.int64) * 4 + pwid <= ts[plane[pu]]), "pred crosses its tile"
    assert np.all(P["y4"].astype(np.int64) * 4 + phei <= ts[plane[pu]]), "pred crosses its tile"
    inter = np.isin(kind, abi.INTER_KINDS + (abi.PRED_INTER_INTRA, abi.PRED_WARP))
    sxy = fd.src_xy[pu]
    for k in range(2):
        P[f"src_x{k}"] = np.where(inter, sxy[:, k, 0], 0)
        P[f"src_y{k}"] = np.where(inter, sxy[:, k, 1], 0)
        P[f"mx{k}"] = np.where(inter, u[f"mx{k}"][pu], 0)
        P[f"my{k}"] = np.where(inter, u[f"my{k}"][pu], 0)
        P[f"ref{k}"] = np.where(inter, u[f"ref{k}"][pu], 0)
    P["filter2d"] = np.where(inter, u["filter2d"][pu], 0)
    P["weight"] = np.where(inter, u["weight"][pu], 0)
    aux_u = fd.aux if fd.aux is not None else np.zeros(n, np.int32)
    P["aux"] = np.where(inter, aux_u[pu], 0)

    # ---- order inside each tile: cooperative groups (largest first, then
    # mode), then the independent tasks (by kind) ----
    coop = np.isin(kind, COOP_KINDS)
    G = np.where(coop, coop_lanes(pwid, phei), 0)
    R = task_rows(phei, bpc)
    ntask = np.where(coop, 0, (pwid // 4) * (phei // R))
    mode_key = np.where(coop, u["mode"][pu], 0)
    # tasks: by row count R, then by kind (a wave then runs one mc path)
    rkey = np.where(coop, 0, R)
    order = np.lexsort((u["txtp"][pu], mode_key, kind, rkey, -G, ~coop, ptile))
    pu, P, kind, pwid, phei, ptile, coop, G, ntask = (pu[order], P[order], kind[order], pwid[order], phei[order],
                                                      ptile[order], coop[order], G[order], ntask[order])
    tile_pred_count = np.bincount(ptile, minlength=n_tiles_all)
    pred0 = np.cumsum(tile_pred_count) - tile_pred_count
    starts = pred0[tile_pred_count > 0]
    lengths = tile_pred_count[tile_pred_count > 0]
    coop_base = _seg_excl_cumsum(G, starts, lengths)
    task_base = _seg_excl_cumsum(ntask, starts, lengths)
    P["lane0"] = np.where(coop, coop_base, task_base)
    P["lanes_log2"] = np.where(coop, np.log2(np.maximum(G, 1)).astype(np.int64), 0)
    coop_used = np.bincount(ptile, weights=G, minlength=n_tiles_all).astype(np.int64)
    task_used = np.bincount(ptile, weights=ntask, minlength=n_tiles_all).astype(np.int64)
    assert np.all(coop_base[coop] % G[coop] == 0), "cooperative groups must be aligned"

    # intra-side fields (union view); edges laid out tile by tile in pred order
    cu = pu[coop]
    P["edge_off"][coop] = 0   # filled below
    iv = P[coop]
    iv["angle"] = u["angle"][cu]
    iv["mode"] = u["mode"][cu]
    iv["max_w"] = u["max_w"][cu]
    iv["max_h"] = u["max_h"][cu]
    iscfl = kind[coop] == abi.PRED_CFL
    iv["alpha"] = np.where(iscfl, u["cfl_alpha"][cu], 0)
    iv["cfl_pad_wh"] = np.where(iscfl, u["cfl_pad_wh"][cu], 0)
    iv["aux"] = np.where(iscfl, u["cfl_luma_off"][cu], 0)
    iv["pad2"] = 0
    iv["pad3"] = 0
    elen = 2 * pwid[coop] + 2 * phei[coop] + 1
    esrc = u["edge_off"][cu].astype(np.int64) - 2 * phei[coop]
    ctile = ptile[coop]
    tile_edge_n = np.bincount(ctile, weights=elen, minlength=n_tiles_all).astype(np.int64)
    assert tile_edge_n.max(initial=0) <= MAX_EDGE, "tile edge pool over DGPU_TILE_MAX_EDGE"
    edge0 = np.cumsum(tile_edge_n) - tile_edge_n
    e_dst = np.cumsum(elen) - elen                     # global position in the new pool
    iv["edge_off"] = e_dst - edge0[ctile] + 2 * phei[coop]
    P[coop] = iv
    edges_main = fd.edges[_gather_ranges(esrc, elen)] if len(elen) else np.zeros(0, fd.edges.dtype)
    pal = kind == abi.PRED_PAL
    pv = P[pal]
    pv["aux"] = aux_u[pu[pal]]
    pv["edge_off"] = 0
    pv["angle"] = 0
    P[pal] = pv

    # inter-intra: its record's edge array moves to the new pool (after the
    # tiles' staged edges; the kernel reads it from memory)
    aux_pool = None if fd.aux_pool is None else fd.aux_pool.copy()
    edges_ii = np.zeros(0, fd.edges.dtype)
    iiu = np.nonzero(kind == abi.PRED_INTER_INTRA)[0]
    if len(iiu):
        recs = P["aux"][iiu].astype(np.int64)
        old = np.frombuffer(aux_pool.tobytes(), np.uint8)
        eo = np.array([int(np.frombuffer(old[r:r + 4].tobytes(), "<i4")[0]) for r in recs], np.int64)
        ilen = 2 * pwid[iiu] + 2 * phei[iiu] + 1
        edges_ii = fd.edges[_gather_ranges(eo - 2 * phei[iiu], ilen)]
        new_eo = len(edges_main) + np.cumsum(ilen) - ilen + 2 * phei[iiu]
        for r, e in zip(recs, new_eo):
            aux_pool[r:r + 4] = np.array([e], "<i4").view(np.uint8)
    edges = np.concatenate([edges_main, edges_ii]) if len(edges_ii) else edges_main
    if len(edges) == 0:
        edges = np.zeros(1, fd.edges.dtype)

    # ---- transform blocks with a residual ----
    has_res = u["txtp"] != abi.NO_RESIDUAL
    xu = np.nonzero(has_res)[0]
    xl = tx_lanes(tw[xu], th[xu])
    xtile = tid[xu]
    # inside a lane-count group: by width, height, then the 1-D kinds (ADST
    # and FLIPADST share a body), so a wave's lanes mostly run one row path
    # and one column path
    kc = np.array([0, 1, 1, 2])   # DCT, ADST, FLIPADST, IDENTITY -> body
    kh = kc[(0xb73da850 >> (2 * u["txtp"][xu].astype(np.int64))) & 3]
    kv = kc[(0xedce6244 >> (2 * u["txtp"][xu].astype(np.int64))) & 3]
    xorder = np.lexsort((u["txtp"][xu], kv, kh, th[xu], tw[xu], -xl, xtile))
    xu, xl, xtile = xu[xorder], xl[xorder], xtile[xorder]
    tile_tx_count = np.bincount(xtile, minlength=n_tiles_all)
    tx0 = np.cumsum(tile_tx_count) - tile_tx_count
    xs = tx0[tile_tx_count > 0]
    xlen = tile_tx_count[tile_tx_count > 0]
    lane0 = _seg_excl_cumsum(xl, xs, xlen)
    lanes_tx = np.bincount(xtile, weights=xl, minlength=n_tiles_all).astype(np.int64)
    assert np.all(lane0 % xl == 0)
    nzw = u["nzw"][xu].astype(np.int64)
    nzh = u["nzh"][xu].astype(np.int64)
    ncoef = np.where(nzw == 0, 1, nzw * nzh)
    tile_coef_n = np.bincount(xtile, weights=ncoef, minlength=n_tiles_all).astype(np.int64)
    coef0 = np.cumsum(tile_coef_n) - tile_coef_n
    c_dst = np.cumsum(ncoef) - ncoef
    coef_rel = c_dst - coef0[xtile]
    coefs = fd.coefs[_gather_ranges(u["coef_off"][xu], ncoef)] if len(xu) else np.zeros(0, fd.coefs.dtype)
    if len(coefs) == 0:
        coefs = np.zeros(1, fd.coefs.dtype)
    ttx = tcol[xu] * ts[plane[xu]]
    tty = trow[xu] * ts[plane[xu]]
    X = np.zeros(len(xu), TX_DTYPE)
    X["w0"] = (((ux[xu] - ttx) // 4) | (((uy[xu] - tty) // 4) << 4) | (u["tx"][xu].astype(np.int64) << 8)
               | (u["txtp"][xu].astype(np.int64) << 13) | (nzw << 18) | (nzh << 24))
    X["w1"] = coef_rel | (lane0 << 16)
    assert coef_rel.max(initial=0) < 65536 and lanes_tx.max(initial=0) <= 1024

    # ---- tiles ----
    T = np.zeros(n_tiles_all, TILE_DTYPE)
    tt = np.arange(n_tiles_all)
    tp_ = tt % 3
    sb = tt // 3
    T["plane"] = tp_
    T["x"] = (sb % ncol) * ts[tp_]
    T["y"] = (sb // ncol) * ts[tp_]
    T["w4"] = np.minimum(ts[tp_], pw[tp_] - T["x"]) // 4
    T["h4"] = np.minimum(ts[tp_], ph[tp_] - T["y"]) // 4
    T["pred0"] = pred0
    T["n_pred"] = tile_pred_count
    T["tx0"] = tx0
    T["n_tx"] = tile_tx_count
    T["coef0"] = coef0
    T["n_coef"] = tile_coef_n
    T["edge0"] = edge0
    T["n_edge"] = tile_edge_n
    T["lanes_tx"] = lanes_tx
    T["lanes_coop"] = (coop_used + 63) // 64 * 64
    T["lanes_coop_used"] = coop_used
    T["lanes_task"] = task_used
    T["flags"] = (np.bincount(ptile, weights=(kind == abi.PRED_WARP), minlength=n_tiles_all) > 0).astype(np.uint8)
    assert tile_pred_count.max(initial=0) <= 256 and tile_tx_count.max(initial=0) <= 256
    assert (T["lanes_coop"].astype(np.int64) + T["lanes_task"]).max(initial=0) <= 1024
    # every pixel of a tile is covered by exactly one pred
    cover = np.bincount(ptile, weights=pwid * phei, minlength=n_tiles_all)
    assert np.array_equal(cover.astype(np.int64), T["w4"].astype(np.int64) * T["h4"] * 16), "tile coverage"
    # the tiles with 64-point transforms go last (their own kernel)
    huge_tx = (tw[xu] == 64) | (th[xu] == 64)
    is_huge = np.bincount(xtile, weights=huge_tx, minlength=n_tiles_all) > 0
    torder = np.concatenate([np.nonzero(~is_huge)[0], np.nonzero(is_huge)[0]])
    T = T[torder]

    stats = dict(fd.stats)
    desc = n_tiles_all * TILE_DTYPE.itemsize + npred * PRED_DTYPE.itemsize + len(xu) * TX_DTYPE.itemsize
    stats["desc_bytes"] = desc   # the tile / pred / tx records: not in total_bytes (algorithmic)
    stats["n_tiles"] = n_tiles_all
    stats["n_preds"] = npred
    stats["n_txs"] = len(xu)
    return TileData(cfg=cfg, tiles=T, preds=P, txs=X, coefs=coefs, edges=edges, aux_pool=aux_pool,
                    n_tiles_huge=int(is_huge.sum()), stats=stats)
