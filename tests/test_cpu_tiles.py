"""CPU-side tests of the superblock-tile batch (no GPU): the C layout of the
tile ABI against its Python mirror, the host-side tile builder's invariants,
the oracle's tile walker against the golden fixtures (the same pixels as
the unit walker), and the launch's validation paths."""
import ctypes
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_LAYOUT_C = r"""
#include <stddef.h>
#include <stdio.h>
#include "dav1d_gpu.h"
#define P(s, f) printf(#s "." #f " %zu\n", offsetof(s, f))
int main(void) {
    printf("Dav1dGpuTile %zu\nDav1dGpuPred %zu\nDav1dGpuTx %zu\nDav1dGpuTileBatch %zu\n",
           sizeof(Dav1dGpuTile), sizeof(Dav1dGpuPred), sizeof(Dav1dGpuTx), sizeof(Dav1dGpuTileBatch));
    P(Dav1dGpuTile, x); P(Dav1dGpuTile, plane); P(Dav1dGpuTile, flags); P(Dav1dGpuTile, pred0);
    P(Dav1dGpuTile, tx0); P(Dav1dGpuTile, coef0); P(Dav1dGpuTile, edge0); P(Dav1dGpuTile, n_pred);
    P(Dav1dGpuTile, n_coef); P(Dav1dGpuTile, n_edge); P(Dav1dGpuTile, lanes_tx); P(Dav1dGpuTile, lanes_coop);
    P(Dav1dGpuTile, lanes_task); P(Dav1dGpuTile, lanes_coop_used);
    P(Dav1dGpuPred, lanes_log2); P(Dav1dGpuPred, lane0); P(Dav1dGpuPred, p.inter.src_x);
    P(Dav1dGpuPred, p.inter.src_y); P(Dav1dGpuPred, p.inter.mx); P(Dav1dGpuPred, p.inter.my);
    P(Dav1dGpuPred, p.inter.filter2d); P(Dav1dGpuPred, p.inter.ref); P(Dav1dGpuPred, p.inter.weight);
    P(Dav1dGpuPred, p.inter.aux); P(Dav1dGpuPred, p.intra.edge_off); P(Dav1dGpuPred, p.intra.angle);
    P(Dav1dGpuPred, p.intra.mode); P(Dav1dGpuPred, p.intra.alpha); P(Dav1dGpuPred, p.intra.max_w);
    P(Dav1dGpuPred, p.intra.max_h); P(Dav1dGpuPred, p.intra.cfl_pad_wh); P(Dav1dGpuPred, p.intra.aux);
    P(Dav1dGpuTileBatch, tiles); P(Dav1dGpuTileBatch, n_tiles); P(Dav1dGpuTileBatch, n_tiles_huge);
    P(Dav1dGpuTileBatch, bitdepth_max); P(Dav1dGpuTileBatch, preds); P(Dav1dGpuTileBatch, txs);
    P(Dav1dGpuTileBatch, coef); P(Dav1dGpuTileBatch, edges); P(Dav1dGpuTileBatch, aux_pool);
    P(Dav1dGpuTileBatch, cfl_luma); P(Dav1dGpuTileBatch, cfl_ss); P(Dav1dGpuTileBatch, zero_coefs);
    return 0;
}
"""


def _c_layout(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(_LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["cc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    return {k: int(v) for k, v in (line.split() for line in out.splitlines())}


def test_tile_abi_layout(pkg, tmp_path):
    """include/dav1d_gpu.h's tile structs == the numpy / ctypes mirrors."""
    import dav1d_mirror_amd.tiles as tl
    c = _c_layout(tmp_path)
    assert c["Dav1dGpuTile"] == tl.TILE_DTYPE.itemsize == 48
    assert c["Dav1dGpuPred"] == tl.PRED_DTYPE.itemsize == 32
    assert c["Dav1dGpuTx"] == tl.TX_DTYPE.itemsize == 8
    f = tl.TILE_DTYPE.fields
    for name in ("x", "plane", "flags", "pred0", "tx0", "coef0", "edge0", "n_pred", "n_coef", "n_edge",
                 "lanes_tx", "lanes_coop", "lanes_task", "lanes_coop_used"):
        assert c[f"Dav1dGpuTile.{name}"] == f[name][1], name
    f = tl.PRED_DTYPE.fields
    pairs = {"lanes_log2": "lanes_log2", "lane0": "lane0", "p.inter.src_x": "src_x0", "p.inter.src_y": "src_y0",
             "p.inter.mx": "mx0", "p.inter.my": "my0", "p.inter.filter2d": "filter2d", "p.inter.ref": "ref0",
             "p.inter.weight": "weight", "p.inter.aux": "aux", "p.intra.edge_off": "edge_off",
             "p.intra.angle": "angle", "p.intra.mode": "mode", "p.intra.alpha": "alpha", "p.intra.max_w": "max_w",
             "p.intra.max_h": "max_h", "p.intra.cfl_pad_wh": "cfl_pad_wh", "p.intra.aux": "aux"}
    for cname, npname in pairs.items():
        assert c[f"Dav1dGpuPred.{cname}"] == f[npname][1], cname
    tb = pkg.abi.TileBatch
    assert c["Dav1dGpuTileBatch"] == ctypes.sizeof(tb)
    for name in ("tiles", "n_tiles", "n_tiles_huge", "bitdepth_max", "preds", "txs", "coef", "edges",
                 "aux_pool", "cfl_luma", "cfl_ss", "zero_coefs"):
        assert c[f"Dav1dGpuTileBatch.{name}"] == getattr(tb, name).offset, name


def test_tile_walker_golden(pkg, oracle):
    """The oracle's tile walker (per-block mc with recon_tmpl.c's emu_edge
    condition) reproduces the golden planes of the unit walker, including
    MVs far past the picture on edge-replicated references."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_golden
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.tiles as tl
    g = np.load(os.path.join(ROOT, "tests", "golden", "recon_golden.npz"))
    for name, kw in gen_golden.CASES:
        fd = wl.make_frame(wl.FrameConfig(**kw))
        ht = oracle.HostTiles(fd, tl.build_tiles(fd))
        ht.run()
        for p, a in enumerate(ht.dst):
            h = np.frombuffer(hashlib.sha256(a.tobytes()).digest(), np.uint8)
            assert np.array_equal(h, g[f"{name}_p{p}_sha256"]), (name, p)


@pytest.mark.parametrize("kind", ["full", "ext", "mc", "ipred", "itx"])
def test_tile_builder_invariants(pkg, kind):
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.tiles as tl
    abi = pkg.abi
    fd = wl.make_frame(wl.FrameConfig(width=512, height=256, seed=41, kind=kind, tx64=(kind == "full")))
    td = tl.build_tiles(fd)
    T, P, X = td.tiles, td.preds, td.txs
    # every transform block with a residual appears once, with its coefficients
    has_res = fd.units["txtp"] != abi.NO_RESIDUAL
    assert len(X) == int(has_res.sum())
    assert int(T["n_tx"].sum()) == len(X) and int(T["n_pred"].sum()) == len(P)
    assert int(T["n_coef"].sum()) == (len(td.coefs) if len(X) else 0)
    huge_seen = False
    for i, t in enumerate(T):
        x = X[t["tx0"]:t["tx0"] + t["n_tx"]]
        tx = (x["w0"] >> 8) & 31
        lanes = np.array([tl.tx_lanes(*abi.TX_WH[k]) for k in tx], np.int64)
        lane0 = (x["w1"] >> 16).astype(np.int64)
        if len(x):
            assert np.all(np.diff(lanes) <= 0)                     # largest groups first
            assert np.all(lane0 % lanes == 0)                      # aligned groups
            assert lane0[-1] + lanes[-1] == t["lanes_tx"] <= 1024
        has64 = any(max(abi.TX_WH[k]) == 64 for k in tx)
        assert has64 == (i >= len(T) - td.n_tiles_huge)           # 64-point tiles go last
        huge_seen |= has64
        p = P[t["pred0"]:t["pred0"] + t["n_pred"]]
        cov = np.zeros((t["h4"] * 4, t["w4"] * 4), np.int32)
        for q in p:
            cov[q["y4"] * 4:(q["y4"] + q["h4"]) * 4, q["x4"] * 4:(q["x4"] + q["w4"]) * 4] += 1
        assert np.all(cov == 1)                                    # one pred per pixel
        coop = np.isin(p["kind"], tl.COOP_KINDS)
        assert np.all(np.diff(coop.astype(int)) <= 0)              # cooperative preds first
        g = 1 << p["lanes_log2"][coop].astype(np.int64)
        l0 = p["lane0"][coop].astype(np.int64)
        assert np.all(l0 % g == 0) and int(g.sum()) == t["lanes_coop_used"] <= t["lanes_coop"]
        assert t["lanes_coop"] % 64 == 0 and t["n_edge"] <= tl.MAX_EDGE
    assert huge_seen == (kind == "full")


def test_tile_zero_coefs_oracle(pkg, oracle):
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.tiles as tl
    fd = wl.make_frame(wl.FrameConfig(width=256, height=128, seed=43))
    td = tl.build_tiles(fd)
    assert np.any(td.coefs)
    ht = oracle.HostTiles(fd, td, zero_coefs=True)
    ht.run()
    assert not np.any(ht.coefs)


def test_tiles_launch_validation(pkg):
    """dav1d_gpu_recon_tiles_* reject malformed batches before touching a
    device: NULL, negative / inconsistent counts, misaligned planes."""
    L = pkg.abi.load_lib()
    for bpc in (8, 16):
        fn = getattr(L, f"dav1d_gpu_recon_tiles_{bpc}bpc")
        assert fn(None, None) == -1
        b = pkg.abi.TileBatch()
        b.n_tiles = -1
        assert fn(ctypes.byref(b), None) == -1
        b.n_tiles, b.n_tiles_huge = 4, 5
        assert fn(ctypes.byref(b), None) == -1
        b.n_tiles, b.n_tiles_huge = 4, 0
        assert fn(ctypes.byref(b), None) == -1                      # tiles / preds NULL
        b.n_tiles = 0
        b.dst[0].data, b.dst[0].stride = 16, 24                     # stride not a multiple of 16
        assert fn(ctypes.byref(b), None) == -4
        b.dst[0].stride = 32
        b.ref[0][0].data, b.ref[0][0].stride = 18, 64               # reference not dword aligned
        assert fn(ctypes.byref(b), None) == -4
        b.ref[0][0].data = 16
        assert fn(ctypes.byref(b), None) == 0                       # empty batch: nothing to do


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
def test_tile_walker_lossless(pkg, oracle, bpc, bdmax):
    """WHT_WHT (lossless 4x4) blocks with full-range coefficients: the tile
    walker (per tile, transform records) and the unit walker (per unit)
    give the same planes, and the frame generator marks only 4x4 units
    without moving any coefficient region."""
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.tiles as tl
    kw = dict(width=256, height=128, seed=95, bpc=bpc, bitdepth_max=bdmax)
    base = wl.make_frame(wl.FrameConfig(**kw))
    fd = wl.make_frame(wl.FrameConfig(lossless=0.6, **kw))
    # the same units (the batch's sort puts them in another order)
    ua = fd.units[np.lexsort((fd.units["dst_off"], fd.units["plane"]))]
    ub = base.units[np.lexsort((base.units["dst_off"], base.units["plane"]))]
    wht = ua["txtp"] == pkg.abi.WHT_WHT
    assert wht.sum() > 20 and np.all(ua["tx"][wht] == 0)
    assert np.array_equal(ua["coef_off"], ub["coef_off"])
    assert np.array_equal(ua[~wht], ub[~wht])
    ht = oracle.HostTiles(fd, tl.build_tiles(fd))
    ht.run()
    hf = oracle.HostFrame(fd)
    hf.run(threads=2)
    for p in range(3):
        assert np.array_equal(ht.dst[p], hf.dst[p]), p
