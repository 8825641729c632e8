"""CPU tests of intra edge preparation: the C layout of
Dav1dGpuIntraEdge / Dav1dGpuIntraEdgeBatch against the Python mirrors, the
oracle's restatement (oracle/dsp_ref.c, oracle_prepare_intra_edges) against
a second, independent pure-Python restatement that follows the reference's
own control flow (src/ipred_prepare_tmpl.c:76-204: copy px_have pixels,
then pixel_set the rest) on small random batches, hand-checked cases, and
the launch's validation paths.

Parity unpinned against the reference binary (it is not buildable here,
DESIGN.md 'Parity'); the reference holds no fixtures for this function."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_LAYOUT_C = r"""
#include <stddef.h>
#include <stdio.h>
#include "dav1d_gpu.h"
#define P(s, f) printf(#s "." #f " %zu\n", offsetof(s, f))
int main(void) {
    printf("Dav1dGpuIntraEdge %zu\nDav1dGpuIntraEdgeBatch %zu\n", sizeof(Dav1dGpuIntraEdge),
           sizeof(Dav1dGpuIntraEdgeBatch));
    P(Dav1dGpuIntraEdge, unit); P(Dav1dGpuIntraEdge, x4); P(Dav1dGpuIntraEdge, y4);
    P(Dav1dGpuIntraEdge, w4); P(Dav1dGpuIntraEdge, h4); P(Dav1dGpuIntraEdge, mode);
    P(Dav1dGpuIntraEdge, angle); P(Dav1dGpuIntraEdge, flags);
    P(Dav1dGpuIntraEdgeBatch, pic); P(Dav1dGpuIntraEdgeBatch, top_edge); P(Dav1dGpuIntraEdgeBatch, sb_log2);
    P(Dav1dGpuIntraEdgeBatch, units); P(Dav1dGpuIntraEdgeBatch, edges); P(Dav1dGpuIntraEdgeBatch, recs);
    P(Dav1dGpuIntraEdgeBatch, n_recs); P(Dav1dGpuIntraEdgeBatch, bitdepth_max);
    return 0;
}
"""


def test_intra_edge_abi_layout(pkg, tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(_LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["cc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    c = {k: int(v) for k, v in (line.split() for line in out.splitlines())}
    abi = pkg.abi
    assert c["Dav1dGpuIntraEdge"] == abi.INTRA_EDGE_DTYPE.itemsize == 16
    for name in ("unit", "x4", "y4", "w4", "h4", "mode", "angle", "flags"):
        assert c[f"Dav1dGpuIntraEdge.{name}"] == abi.INTRA_EDGE_DTYPE.fields[name][1], name
    B = abi.IntraEdgeBatch
    assert c["Dav1dGpuIntraEdgeBatch"] == ctypes.sizeof(B)
    for name in ("pic", "top_edge", "sb_log2", "units", "edges", "recs", "n_recs", "bitdepth_max"):
        assert c[f"Dav1dGpuIntraEdgeBatch.{name}"] == getattr(B, name).offset, name


# ---- a second restatement, in the reference's own control-flow shape ----
_ANGLE = [90, 180, 45, 135, 113, 157, 203, 67]          # av1_mode_to_angle_map
# (needs_left, needs_top, needs_topleft, needs_topright, needs_bottomleft),
# av1_intra_prediction_edges, src/ipred_prepare_tmpl.c:50-75
_NEEDS = {0: (1, 1, 0, 0, 0), 1: (0, 1, 0, 0, 0), 2: (1, 0, 0, 0, 0), 3: (1, 0, 0, 0, 0),
          4: (0, 1, 0, 0, 0), 5: (0, 0, 0, 0, 0), 6: (0, 1, 1, 1, 0), 7: (1, 1, 1, 0, 0),
          8: (1, 0, 1, 0, 1), 9: (1, 1, 0, 0, 0), 10: (1, 1, 0, 0, 0), 11: (1, 1, 0, 0, 0),
          12: (1, 1, 1, 0, 0), 13: (1, 1, 1, 0, 0)}
# av1_mode_conv[mode][have_left][have_top] (:38-48) for DC (0) and PAETH (12)
_CONV = {0: [[5, 4], [3, 0]], 12: [[5, 1], [2, 12]]}


def _py_prepare(case, rec, units, edges):
    u = units[rec["unit"]]
    pl, tx = int(u["plane"]), int(u["tx"])
    tw, th = (d // 4 for d in __import__("dav1d_mirror_amd.abi", fromlist=["x"]).TX_WH[tx])
    pic = case.pics[pl].astype(np.int64)
    x, y, w, h = int(rec["x4"]), int(rec["y4"]), int(rec["w4"]), int(rec["h4"])
    fl = int(rec["flags"])
    have_left, have_top = bool(fl & 1), bool(fl & 2)
    bd = case.bitdepth_max.bit_length()
    px = lambda r, c: int(pic[y * 4 + r, x * 4 + c])                       # dst[r*stride + c]
    mode, angle = int(rec["mode"]), int(rec["angle"])
    if 1 <= mode <= 8:
        angle = _ANGLE[mode - 1] + 3 * angle
        if angle <= 90:
            mode = 6 if angle < 90 and have_top else 1
        elif angle < 180:
            mode = 7
        else:
            mode = 8 if angle > 180 and have_left else 2
    elif mode in _CONV:
        mode = _CONV[mode][have_left][have_top]
    nl, nt, ntl, ntr, nbl = _NEEDS[mode]
    if fl & 64:
        row = case.top_edge[pl][((y * 4) >> case.sb_log2[pl]) - 1].astype(np.int64)
        dst_top = lambda c: int(row[x * 4 + c])
    else:
        dst_top = lambda c: px(-1, c)
    E = {}
    o = int(u["edge_off"])
    if nl:
        sz = th * 4
        left = {}
        if have_left:
            ph = min(sz, (h - y) * 4)
            for i in range(ph):
                left[sz - 1 - i] = px(i, -1)
            for i in range(sz - ph):
                left[i] = left[sz - ph]
        else:
            for i in range(sz):
                left[i] = dst_top(0) if have_top else (1 << bd >> 1) + 1
        if nbl:
            hbl = have_left and y + th < h and (fl & 8)
            if hbl:
                ph = min(sz, (h - y - th) * 4)
                for i in range(ph):
                    left[-(i + 1)] = px(sz + i, -1)
                for i in range(sz - ph):
                    left[-sz + i] = left[-ph]
            else:
                for i in range(sz):
                    left[-sz + i] = left[0]
        for k, v in left.items():
            E[k - sz] = v
    if nt:
        sz = tw * 4
        top = {}
        if have_top:
            ph = min(sz, (w - x) * 4)
            for i in range(ph):
                top[i] = dst_top(i)
            for i in range(ph, sz):
                top[i] = top[ph - 1]
        else:
            for i in range(sz):
                top[i] = px(0, -1) if have_left else (1 << bd >> 1) - 1
        if ntr:
            htr = have_top and x + tw < w and (fl & 4)
            if htr:
                ph = min(sz, (w - x - tw) * 4)
                for i in range(ph):
                    top[sz + i] = dst_top(sz + i)
                for i in range(ph, sz):
                    top[sz + i] = top[sz + ph - 1]
            else:
                for i in range(sz):
                    top[sz + i] = top[sz - 1]
        for k, v in top.items():
            E[1 + k] = v
    if ntl:
        if have_left:
            t = dst_top(-1) if have_top else px(0, -1)
        else:
            t = dst_top(0) if have_top else 1 << bd >> 1
        if mode == 7 and tw + th >= 6 and (fl & 16):
            t = ((E[-1] + E[1]) * 5 + t * 6 + 8) >> 4
        E[0] = t
    for k, v in E.items():
        edges[o + k] = v
    units[rec["unit"]]["mode"] = mode
    if u["pred"] != 4:   # PRED_CFL: the DC source only, alpha / padding kept
        units[rec["unit"]]["angle"] = (angle & 511) | (512 if fl & 32 else 0) | (1024 if fl & 16 else 0)


@pytest.mark.parametrize("bpc,bdmax,seed", [(8, 255, 5), (16, 1023, 6), (16, 4095, 7)])
def test_oracle_matches_python_restatement(pkg, oracle, bpc, bdmax, seed):
    import dav1d_mirror_amd.intra as intra
    case = intra.make_edge_case(seed=seed, bpc=bpc, bitdepth_max=bdmax, n=400)
    units, edges = case.units.copy(), case.edges.copy()
    for r in case.recs:
        _py_prepare(case, r, units, edges)
    ou, oe = oracle.prepare_intra_edges(case)
    assert np.array_equal(ou, units)
    assert np.array_equal(oe, edges)
    # every implementation mode and every flag was exercised
    assert set(np.unique(units["mode"][case.recs["unit"]])) == set(range(14))
    for bit in (1, 2, 4, 8, 16, 32, 64):
        assert np.any(case.recs["flags"] & bit)
    cfl = units["pred"] == pkg.abi.PRED_CFL
    assert cfl.any() and np.array_equal(units["cfl_alpha"][cfl], case.units["cfl_alpha"][cfl])


def _one(pkg, pic, rec, tx, bpc=8, bdmax=255, top_edge=None):
    import dav1d_mirror_amd.intra as intra
    abi = pkg.abi
    pdt = np.uint8 if bpc == 8 else np.uint16
    tw, th = abi.TX_WH[tx]
    units = np.zeros(1, abi.UNIT_DTYPE)
    units["tx"], units["pred"], units["edge_off"] = tx, abi.PRED_INTRA, 2 * th
    small = np.zeros((4, 8), pdt)
    te = top_edge if top_edge is not None else np.zeros((2, pic.shape[1]), pdt)
    recs = np.array([rec], abi.INTRA_EDGE_DTYPE)
    edges = np.full(2 * th + 2 * tw + 1, 7, pdt)
    return intra.EdgeCase(bpc, bdmax, [pic, small, small], [te, small, small], (6, 5, 5), units, recs, edges)


def test_oracle_hand_cases(pkg, oracle):
    """Known answers read off src/ipred_prepare_tmpl.c by hand."""
    abi = pkg.abi
    pic = np.arange(64 * 64, dtype=np.int64).reshape(64, 64).astype(np.uint8)
    tx8 = abi.TX_INDEX[(8, 8)]
    # DC with no neighbours: DC_128, nothing read or written (:107-110 needs nothing)
    u, e = oracle.prepare_intra_edges(_one(pkg, pic, (0, 2, 2, 16, 16, 0, 0, 0, 0), tx8))
    assert u["mode"][0] == abi.DC_128_PRED and np.all(e == 7)
    # V_PRED without top, with left: top row = dst[-1] (:163-164)
    u, e = oracle.prepare_intra_edges(_one(pkg, pic, (0, 2, 2, 16, 16, 1, 0, abi.IE_HAVE_LEFT, 0), tx8))
    assert u["mode"][0] == abi.VERT_PRED and u["angle"][0] == 90
    assert np.all(e[17:25] == pic[8, 7]) and np.all(e[:17] == 7)
    # H_PRED without left, with top: left column = dst_top[0] (:131-132)
    u, e = oracle.prepare_intra_edges(_one(pkg, pic, (0, 2, 2, 16, 16, 2, 0, abi.IE_HAVE_TOP, 0), tx8))
    assert u["mode"][0] == abi.HOR_PRED and np.all(e[8:16] == pic[7, 8])
    # left column clipped by the tile end h4: rows past it repeat the last (:126-129)
    u, e = oracle.prepare_intra_edges(_one(pkg, pic, (0, 2, 2, 16, 3, 2, 0, abi.IE_HAVE_LEFT, 0), tx8))
    assert list(e[8:16][::-1]) == [pic[8 + i, 7] for i in range(4)] + [pic[11, 7]] * 4
    # D45 (angle 45 - 9 = 36): Z1; top-right from the picture when available
    fl = abi.IE_HAVE_LEFT | abi.IE_HAVE_TOP | abi.IE_TOP_HAS_RIGHT
    u, e = oracle.prepare_intra_edges(_one(pkg, pic, (0, 2, 2, 16, 16, 3, -3, fl, 0), tx8))
    assert u["mode"][0] == abi.Z1_PRED and u["angle"][0] == 36
    assert list(e[17:33]) == [pic[7, 8 + i] for i in range(16)] and e[16] == pic[7, 7]
    # the same without TOP_HAS_RIGHT: top-right repeats top[sz-1] (:183-184)
    u, e = oracle.prepare_intra_edges(_one(pkg, pic, (0, 2, 2, 16, 16, 3, -3, fl & ~4, 0), tx8))
    assert np.all(e[25:33] == pic[7, 15])
    # PAETH at a superblock top: top row and top-left from the top_edge row
    # (prefilter_toplevel_sb_edge, :117-120), left from the picture
    pic2 = (np.arange(128 * 64) % 251).astype(np.uint8).reshape(128, 64)
    te = (255 - np.arange(2 * 64) % 256).astype(np.uint8).reshape(2, 64)
    fl = abi.IE_HAVE_LEFT | abi.IE_HAVE_TOP | abi.IE_TOP_SB_EDGE
    u, e = oracle.prepare_intra_edges(_one(pkg, pic2, (0, 2, 16, 16, 32, 12, 0, fl, 0), tx8, top_edge=te))
    assert u["mode"][0] == abi.PAETH_PRED
    assert list(e[16:25]) == list(te[0, 7:16])
    assert list(e[8:16][::-1]) == [pic2[64 + i, 7] for i in range(8)]
    # Z2 with the edge filter on a 16x16: the top-left is smoothed (:197-200)
    tx16 = abi.TX_INDEX[(16, 16)]
    fl = abi.IE_HAVE_LEFT | abi.IE_HAVE_TOP | abi.IE_FILTER_EDGE
    u, e = oracle.prepare_intra_edges(_one(pkg, pic2, (0, 4, 4, 16, 32, 4, 0, fl, 0), tx16))
    assert u["mode"][0] == abi.Z2_PRED and u["angle"][0] == 135 | 1024
    l0, t0, tl = int(pic2[16, 15]), int(pic2[15, 16]), int(pic2[15, 15])
    assert e[32] == ((l0 + t0) * 5 + tl * 6 + 8) >> 4


def test_prepare_edges_launch_validation(pkg):
    L = pkg.abi.load_lib()
    for bpc in (8, 16):
        fn = getattr(L, f"dav1d_gpu_prepare_intra_edges_{bpc}bpc")
        assert fn(None, None) == -1
        b = pkg.abi.IntraEdgeBatch()
        b.n_recs = -1
        assert fn(ctypes.byref(b), None) == -1
        b.n_recs = 3
        assert fn(ctypes.byref(b), None) == -1                      # recs / units / edges NULL
        b.n_recs = 0
        assert fn(ctypes.byref(b), None) == 0                       # empty batch: nothing to do
