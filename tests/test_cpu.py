"""CPU-side tests (no GPU): the C-ABI library loads and exports what
include/dav1d_gpu.h declares, the oracle against its golden fixtures and
against properties the reference's algorithms guarantee, and the host-side
batch builder.  Fixtures are oracle-generated (parity unpinned vs the
reference binary, which cannot be built here)."""
import ctypes
import hashlib
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------------ C ABI --

def test_header_symbols_exported(pkg):
    hdr = open(os.path.join(ROOT, "include", "dav1d_gpu.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    declared = set(re.findall(r"^\s*(?:int|int64_t|void|const char \*|Dav1dGpuRecorder \*)\s*(dav1d_\w+)\s*\(", hdr, flags=re.M))
    assert len(declared) >= 17
    assert declared == set(pkg.abi.EXPORTED_SYMBOLS)
    lib = ctypes.CDLL(pkg.abi.lib_path())   # loads without touching a device
    for name in sorted(declared):
        assert hasattr(lib, name), name


def test_abi_struct_sizes(pkg):
    assert pkg.abi.UNIT_DTYPE.itemsize == 32
    fb = pkg.abi.FrameBatch
    # 3 + 8*3 planes of 24 bytes, then pointers / ints as in dav1d_gpu.h
    assert ctypes.sizeof(pkg.abi.Plane) == 24
    assert fb.units.offset == 27 * 24


def test_recon_batch_validation(pkg):
    """dav1d_gpu_recon_* reject malformed batches before touching a device
    (no GPU needed): NULL, non-monotonic class ranges, WARP ranges in classes
    narrower than 8 or longer than the class, misaligned output planes; an
    empty batch is a no-op."""
    abi = pkg.abi
    L = abi.load_lib()
    assert L.dav1d_gpu_recon_8bpc(None, None) == -1

    def batch(n):
        b = abi.FrameBatch()
        b.units = 64          # never dereferenced on these paths
        b.n_units = n
        for i in range(abi.N_TX + 1):
            b.class_start[i] = 0 if i <= 1 else n   # all units in class 1 (8x8)
        return b

    for fn in (L.dav1d_gpu_recon_8bpc, L.dav1d_gpu_recon_16bpc):
        assert fn(ctypes.byref(batch(0)), None) == 0
        b = batch(5)
        b.class_start[3] = 2   # not monotonic
        assert fn(ctypes.byref(b), None) == -2
        b = batch(5)
        b.class_start[abi.N_TX] = 4   # last bound != n_units
        assert fn(ctypes.byref(b), None) == -2
        b = batch(5)
        for i in range(abi.N_TX + 1):
            b.class_start[i] = 0 if i <= 4 else 5   # all units in class 4 (64x64)
        b.class_warp[4] = 1   # 64-point classes have no second launch
        assert fn(ctypes.byref(b), None) == -2
        b = batch(5)
        b.class_warp[1] = 6   # more WARP units than the class has
        assert fn(ctypes.byref(b), None) == -2
        b = batch(5)
        b.dst[0].data = 8     # not 16-byte aligned
        assert fn(ctypes.byref(b), None) == -4
        b = batch(5)
        b.dst[1].stride = 1 << 23   # row offsets are 24-bit multiplies: strides in [0, 2^23)
        assert fn(ctypes.byref(b), None) == -4
        b = batch(5)
        b.ref[0][0].data = 4096
        b.ref[0][0].stride = -4096   # negative reference strides too
        assert fn(ctypes.byref(b), None) == -4
    assert L.dav1d_gpu_recon_lds_bytes(8, 3) > L.dav1d_gpu_recon_lds_bytes(8, 2) - 65536
    assert L.dav1d_gpu_recon_lds_bytes(8, 9) == -1


def test_itx_table_matches_reference_count(pkg, oracle):
    L = oracle.load()
    for bpc in (8, 16):
        t = oracle.itx_table(bpc)
        n = sum(1 for tx in range(19) for tp in range(17) if t.itxfm_add[tx][tp])
        assert n == 156, (bpc, n)        # tests/checkasm/itx.c:313-314 table density
        ours = sum(1 for tx in range(19) for tp in range(17) if pkg.abi.itx_supported(tx, tp))
        assert ours == 156
    assert L.oracle_itx_supported_8bpc(4, 0) == 1


# ---------------------------------------------------------------- oracle ---

def test_oracle_golden(pkg, oracle):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_golden
    g = np.load(os.path.join(ROOT, "tests", "golden", "recon_golden.npz"))
    for name, kw in gen_golden.CASES:
        fd, planes = gen_golden.run_case(kw)
        assert int(g[f"{name}_units"][0]) == fd.n_units, name
        for p, a in enumerate(planes):
            h = np.frombuffer(hashlib.sha256(a.tobytes()).digest(), np.uint8)
            assert np.array_equal(h, g[f"{name}_p{p}_sha256"]), (name, p)
            if name == "full8_s1":
                assert np.array_equal(a, g[f"{name}_p{p}"])


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_mc_constant_image_is_preserved(oracle, bpc, bdmax):
    """Every 8-tap / bilinear kernel has unit DC gain (taps sum to 64), so a
    flat picture stays flat through put for all sub-pel positions
    (src/mc_tmpl.c:113-171, :395-450)."""
    tbl = oracle.mc_table(bpc)
    pdt = np.uint8 if bpc == 8 else np.uint16
    rng = np.random.default_rng(bpc + bdmax)
    for f in range(10):
        for w, h in ((4, 4), (8, 8), (16, 32), (2, 8)):
            c = int(rng.integers(0, bdmax + 1))
            src = np.full((h + 8, w + 8), c, pdt)
            dst = np.zeros((h, w), pdt)
            mx, my = int(rng.integers(0, 16)), int(rng.integers(0, 16))
            oracle.call_put(tbl, f, dst, src, 3 * (w + 8) + 3, w, h, mx, my, bdmax)
            assert (dst == c).all(), (f, w, h, mx, my)


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
def test_prep_copy_then_avg_equals_put(oracle, bpc, bdmax):
    """Integer-position compound: avg(prep(x), prep(x)) == put(x) (the
    intermediate scaling/bias of src/mc_tmpl.c:39-49 cancels exactly)."""
    tbl = oracle.mc_table(bpc)
    pdt = np.uint8 if bpc == 8 else np.uint16
    rng = np.random.default_rng(3)
    w = h = 16
    src = rng.integers(0, bdmax + 1, (h + 8, w + 8)).astype(pdt)
    tmp = np.zeros(w * h, np.int16)
    oracle.call_prep(tbl, 0, tmp, src, 3 * (w + 8) + 3, w, h, 0, 0, bdmax)
    ib = 4 if bpc == 8 else 14 - int(np.log2(bdmax + 1))
    pb = 0 if bpc == 8 else 8192
    avg = np.clip((2 * tmp.astype(np.int32) + (1 << ib) + 2 * pb) >> (ib + 1), 0, bdmax)
    assert np.array_equal(avg.reshape(h, w), src[3:3 + h, 3:3 + w])


@pytest.mark.parametrize("bpc", [8, 16])
def test_itx_dc_only_shortcut_matches_full_path(oracle, pkg, bpc):
    """The eob==0 DC-only shortcut of dct_dct (src/itx_tmpl.c:53-65) equals
    the full separable path on a DC-only block for in-range DC values."""
    tbl = oracle.itx_table(bpc)
    pdt = np.uint8 if bpc == 8 else np.uint16
    cdt = np.int16 if bpc == 8 else np.int32
    bdmax = 255 if bpc == 8 else 1023
    rng = np.random.default_rng(bpc)
    for tx, (w, h) in enumerate(pkg.abi.TX_WH):
        for _ in range(4):
            dc = int(rng.integers(-2000, 2000))
            base = rng.integers(0, bdmax + 1, (h, w)).astype(pdt)
            d0, d1 = base.copy(), base.copy()
            c0 = np.zeros(32 * 32, cdt)
            c1 = np.zeros(32 * 32, cdt)
            c0[0] = c1[0] = dc
            oracle.call_itx(tbl, tx, 0, d0, c0, 0, bdmax)
            oracle.call_itx(tbl, tx, 0, d1, c1, 1, bdmax)
            assert np.array_equal(d0, d1), (w, h, dc)
            assert not c0.any() and not c1.any()       # coefficient zeroing contract


# ------------------------------------------------------------- workload ---

def test_workload_covers_every_pixel_once(pkg):
    import dav1d_mirror_amd.workload as wl
    for kind in ("full", "mc", "ipred", "itx", "ext"):
        fd = wl.make_frame(wl.FrameConfig(width=512, height=256, kind=kind, seed=3))
        u = fd.units
        assert np.array_equal(fd.class_start, np.concatenate(
            [[0], np.cumsum(np.bincount(u["tx"], minlength=19))]))
        assert (np.diff(u["tx"].astype(int)) >= 0).all()        # sorted by class
        for p, (w, h) in enumerate(fd.plane_wh):
            cover = np.zeros(h * w, np.int32)
            for t in range(19):
                sel = u[(u["plane"] == p) & (u["tx"] == t)]
                tw, th = pkg.abi.TX_WH[t]
                for off in sel["dst_off"]:
                    y, x = divmod(int(off), w)
                    cover.reshape(h, w)[y:y + th, x:x + tw] += 1
            assert (cover == 1).all(), (kind, p)


def test_workload_family_kinds(pkg, oracle):
    """Bench breakdown frames: every unit of an "ipred" frame is intra / CfL
    without residual, every unit of an "itx" frame is PRED_NONE with one,
    and the oracle adds the residual onto the starting picture."""
    import dav1d_mirror_amd.workload as wl
    abi = pkg.abi
    fi = wl.make_frame(wl.FrameConfig(width=256, height=128, kind="ipred", seed=8))
    assert np.isin(fi.units["pred"], [abi.PRED_INTRA, abi.PRED_CFL]).all()
    assert (fi.units["txtp"] == abi.NO_RESIDUAL).all()
    fx = wl.make_frame(wl.FrameConfig(width=256, height=128, kind="itx", seed=8))
    assert (fx.units["pred"] == abi.PRED_NONE).all() and (fx.units["txtp"] != abi.NO_RESIDUAL).all()
    assert fx.stats["dst_read_bytes"] == fx.stats["dst_bytes"]
    hf = oracle.HostFrame(fx)
    hf.run()
    assert any(not np.array_equal(hf.dst[p], fx.dst_init[p]) for p in range(3))


def test_mc_split_prediction_is_exact(pkg, oracle):
    """Cutting a prediction-only block into smaller units (mc_split) leaves
    the picture unchanged: the batch tier may do it to keep 64-wide blocks
    out of the 64-point class group."""
    import dav1d_mirror_amd.workload as wl
    a = wl.make_frame(wl.FrameConfig(width=256, height=128, kind="mc", seed=3, mc_split=64))
    b = wl.make_frame(wl.FrameConfig(width=256, height=128, kind="mc", seed=3, mc_split=16))
    assert b.n_units > a.n_units
    ha, hb = oracle.HostFrame(a), oracle.HostFrame(b)
    ha.run()
    hb.run()
    assert all(np.array_equal(ha.dst[p], hb.dst[p]) for p in range(3))
    assert a.stats["ref_bytes"] == b.stats["ref_bytes"]


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023)])
def test_oracle_wavg8_and_mask32_equal_avg(pkg, oracle, bpc, bdmax):
    """w_avg with weight 8 and mask_c with a flat 32 mask are avg_c exactly
    (src/mc_tmpl.c:587-639): the batch's extra compound kinds reduce to the
    plain compound average."""
    import dav1d_mirror_amd.workload as wl
    abi = pkg.abi
    fd = wl.make_frame(wl.FrameConfig(width=256, height=128, kind="ext", bpc=bpc, bitdepth_max=bdmax, seed=9))
    u = fd.units.copy()
    wv, mk = u["pred"] == abi.PRED_INTER_WAVG, u["pred"] == abi.PRED_INTER_MASK
    assert wv.any() and mk.any()
    u["weight"][wv] = 8
    fd.units = u
    pool = fd.aux_pool.copy()
    for i in np.nonzero(mk)[0]:
        bw = int(u["bw4"][i]) * 4
        w, h = abi.TX_WH[int(u["tx"][i])]
        for y in range(h):
            o = int(fd.aux[i]) + y * bw
            pool[o:o + w] = 32
    fd.aux_pool = pool
    a = oracle.HostFrame(fd)
    a.run()
    u2 = u.copy()
    u2["pred"][wv | mk] = abi.PRED_INTER_AVG
    fd.units = u2
    b = oracle.HostFrame(fd)
    b.run()
    assert all(np.array_equal(a.dst[p], b.dst[p]) for p in range(3))


def test_workload_deterministic(pkg):
    import dav1d_mirror_amd.workload as wl
    a = wl.make_frame(wl.FrameConfig(width=256, height=128, seed=42))
    b = wl.make_frame(wl.FrameConfig(width=256, height=128, seed=42))
    assert a.units.tobytes() == b.units.tobytes()
    assert np.array_equal(a.coefs, b.coefs) and np.array_equal(a.edges, b.edges)


def test_workload_types_valid(pkg):
    import dav1d_mirror_amd.workload as wl
    fd = wl.make_frame(wl.FrameConfig(width=512, height=256, seed=8))
    u = fd.units
    for tx, tp in zip(u["tx"], u["txtp"]):
        assert pkg.abi.itx_supported(int(tx), int(tp))
    abi = pkg.abi
    inter = (u["pred"] == abi.PRED_INTER) | (u["pred"] == abi.PRED_INTER_AVG)
    intra = u["pred"] == abi.PRED_INTRA
    cfl = u["pred"] == abi.PRED_CFL
    assert (u["filter2d"][inter] < 9).all()
    assert (u["mode"][intra] < 14).all()
    # CfL: chroma only, whole square block <= 32, DC-family source, |alpha| 1..16
    assert cfl.any() and (u["plane"][cfl] > 0).all()
    assert np.isin(u["tx"][cfl], [0, 1, 2, 3]).all()
    assert np.isin(u["mode"][cfl], [abi.DC_PRED, abi.LEFT_DC_PRED, abi.TOP_DC_PRED, abi.DC_128_PRED]).all()
    al = np.abs(u["cfl_alpha"][cfl].astype(int))
    assert ((al >= 1) & (al <= 16)).all()


def test_oracle_cfl_flat_luma_is_dc(pkg, oracle):
    """cfl_ac of a flat luma block is all zero (mean removed), so CfL must
    reproduce the DC-family prediction of the same edges
    (src/ipred_tmpl.c:71-84, :657-703)."""
    import dav1d_mirror_amd.workload as wl
    abi = pkg.abi
    fd = wl.make_frame(wl.FrameConfig(width=256, height=128, seed=21))
    fd.cfl_luma[:] = 77
    a = oracle.HostFrame(fd)
    a.run()
    cfl = fd.units["pred"] == abi.PRED_CFL
    assert cfl.any()
    u2 = fd.units.copy()
    v = u2[cfl]
    v["pred"] = abi.PRED_INTRA
    v["angle"] = 0        # overwrites alpha / pad_wh (the union's intra view)
    v["max_w"] = 0
    v["max_h"] = 0
    u2[cfl] = v
    fd.units = u2
    b = oracle.HostFrame(fd)
    b.run()
    for p in range(3):
        assert np.array_equal(a.dst[p], b.dst[p])


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_ext2_kinds_cut_invariant(pkg, oracle, bpc, bdmax):
    """The second launch's w_mask / OBMC / scaled-reference units: the same
    blocks cut into transform-sized units and into whole prediction blocks
    (<= 32 px) give the same picture, so each unit's record (its part of the
    seg mask, its clipped OBMC overlaps with their mask offsets, its scaled
    phase and integer position) is the block's call restricted to it."""
    import dav1d_mirror_amd.workload as wl
    base = dict(width=256, height=128, bpc=bpc, bitdepth_max=bdmax, kind="ext2", seed=61, no_residual=True)
    a = wl.make_frame(wl.FrameConfig(**base))
    b = wl.make_frame(wl.FrameConfig(unit_split=32, **base))
    kinds = set(np.unique(a.units["pred"]).tolist())
    assert {pkg.abi.PRED_INTER_WMASK, pkg.abi.PRED_INTER_OBMC, pkg.abi.PRED_INTER_SCALED} <= kinds
    assert len(a.units) > len(b.units)
    ha, hb = oracle.HostFrame(a), oracle.HostFrame(b)
    ha.run()
    hb.run()
    for p in range(3):
        assert np.array_equal(ha.dst[p], hb.dst[p]), f"plane {p}"


def test_clamp_units_conversion(pkg):
    """workload.clamp_units (the unit batch on exact-size references): flags
    exactly the inter units whose footprint (with the aligned-load margins)
    leaves the plane, packs their position as x | y << 16, re-expresses the
    others' src_off in the exact stride, and moves the flagged units to the
    end of their class (class_warp); every other field is untouched."""
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.abi as abi
    fd = wl.make_frame(wl.FrameConfig(width=256, height=128, seed=3, mv_range=100))
    fdc, exact = wl.clamp_units(fd)
    assert [a.shape for a in exact[0]] == [(h, w) for (w, h) in fd.plane_wh]
    assert np.array_equal(fdc.class_start, fd.class_start)
    u, c = fdc.units, fdc.class_start
    flagged = ((u["mx0"] | u["mx1"]) & 0x80) != 0
    assert flagged.sum() == fdc.stats["clamped_units"] > 0
    for t in range(abi.N_TX):   # flagged units form the tail of each class range
        seg = flagged[c[t]:c[t + 1]]
        assert seg.sum() == fdc.class_warp[t] and not seg[:len(seg) - seg.sum()].any()
    for i in np.flatnonzero(flagged)[:200]:
        for k in range(2):
            if u[f"mx{k}"][i] & 0x80:
                so = int(u[f"src_off{k}"][i])
                x, y = (so & 0xffff) - ((so & 0x8000) << 1), so >> 16
                assert (x, y) == tuple(fdc.src_xy[i, k])
    # (the intra / CfL views alias the inter fields in the union)
    keep = ["dst_off", "coef_off", "tx", "txtp", "plane", "pred", "nzw", "nzh", "bw4", "bh4", "my0", "my1",
            "filter2d", "ref0", "ref1", "weight"]
    a = np.sort(fd.units[keep], order=keep)
    b = np.sort(u[keep], order=keep)
    assert np.array_equal(a, b)


def test_clamp_units_launch_ahead_kinds(pkg):
    """Round 6: clamp_units flags every launch-ahead unit
    (WARP / INTER_INTRA / INTER_WMASK / INTER_OBMC / INTER_SCALED), rewrites
    the OBMC lap and scaled-reference records to x | y << 16 with their clamp
    bits, and defers the clamped COMPOUND_SEG chroma units to a second batch."""
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.abi as abi
    for kind in ("ext", "ext2"):
        fd = wl.make_frame(wl.FrameConfig(width=256, height=128, seed=5, kind=kind, mv_range=200))
        fdc, _ = wl.clamp_units(fd)
        parts = [fdc] + ([fdc.deferred] if fdc.deferred is not None else [])
        assert sum(f.n_units for f in parts) == fd.n_units
        for f in parts:
            u = f.units
            la = np.isin(u["pred"], abi.SECOND_LAUNCH_KINDS)
            assert ((u["mx0"][la] & 0x80) != 0).all()
            assert (u["src_off0"][u["pred"] == abi.PRED_WARP] == 0).all()
            for t in range(abi.N_TX):   # flagged units form each class's tail
                c0, c1 = f.class_start[t], f.class_start[t + 1]
                assert not la[c0:c1 - f.class_warp[t]].any()
        ap = fdc.aux_pool.view(np.int32)
        pad, u = fd.cfg.ref_pad, fdc.units
        for i in np.nonzero(u["pred"] == abi.PRED_INTER_OBMC)[0][:50]:
            o = int(fdc.aux[i])
            for e in range(int(ap[o // 4])):
                b = o + 16 + 16 * e
                assert fdc.aux_pool[b + 4] & 0x80
                old = int(fd.aux_pool.view(np.int32)[b // 4])
                rs = fd.refs[0][u["plane"][i]].shape[1]
                x, y = wl._decode_off(old, rs, pad)
                v = int(ap[b // 4])
                assert ((v & 0xffff) - ((v & 0x8000) << 1), v >> 16) == (int(x), int(y))
        if kind == "ext2":
            assert fdc.deferred is not None
            assert (fdc.deferred.units["pred"] == abi.PRED_INTER_MASK).all()
