"""CDEF oracle checks on CPU.

The oracle (oracle/dsp_ref.c) restates bytefn(dav1d_cdef_brow)
(src/cdef_apply_tmpl.c:97-309) with the reference's own state: the picture
filtered in place, the pre-filter rows kept in cdef_line (backup2lines,
:41-63), the pre-filter columns in lr_bak (backup2x8, :65-89), driven per
superblock row with the two-row delay of dav1d_filter_sbrow_cdef
(src/recon_tmpl.c:2076-2102).  Below, a second restatement in numpy that
holds none of that state: every block reads a pristine copy of the deblocked
picture, unavailable pixels outside the frame's 8x8 grid.  The two agree on
every pixel, which pins the walker's backup bookkeeping to the frame-level
meaning the device kernel implements.  The reference ships no CDEF vectors
(its checkasm is differential, tests/checkasm/cdef.c), so parity against the
binary stays unpinned, as for the rest of the oracle; hand-derived known
answers pin cdef_find_dir and the filter on simple pictures.
"""
import ctypes

import numpy as np
import pytest

NONE = -32768
DIRS = [((-1, 1), (-2, 2)), ((0, 1), (-1, 2)), ((0, 1), (0, 2)), ((0, 1), (1, 2)),
        ((1, 1), (2, 2)), ((1, 0), (2, 1)), ((1, 0), (2, 0)), ((1, 0), (2, -1))]


def ulog2(v):
    return int(v).bit_length() - 1


def find_dir(blk, bdmax):
    """cdef_find_dir_c, src/cdef_tmpl.c:238-304."""
    bd8 = bdmax.bit_length() - 8
    hv = [[0] * 8 for _ in range(2)]
    diag = [[0] * 15 for _ in range(2)]
    alt = [[0] * 11 for _ in range(4)]
    for y in range(8):
        for x in range(8):
            px = (int(blk[y, x]) >> bd8) - 128
            diag[0][y + x] += px
            alt[0][y + (x >> 1)] += px
            hv[0][y] += px
            alt[1][3 + y - (x >> 1)] += px
            diag[1][7 + y - x] += px
            alt[2][3 - (y >> 1) + x] += px
            hv[1][x] += px
            alt[3][(y >> 1) + x] += px
    div = [840, 420, 280, 210, 168, 140, 120]
    cost = [0] * 8
    cost[2] = 105 * sum(v * v for v in hv[0])
    cost[6] = 105 * sum(v * v for v in hv[1])
    for i, d in ((0, 0), (4, 1)):
        cost[i] = sum((diag[d][n] ** 2 + diag[d][14 - n] ** 2) * div[n] for n in range(7)) + diag[d][7] ** 2 * 105
    for n in range(4):
        c = 105 * sum(alt[n][3 + m] ** 2 for m in range(5))
        c += sum((alt[n][m] ** 2 + alt[n][10 - m] ** 2) * div[2 * m + 1] for m in range(3))
        cost[2 * n + 1] = c
    cost = [c & 0xffffffff for c in cost]
    best = max(range(8), key=lambda n: (cost[n], -n))
    return best, ((cost[best] - cost[best ^ 4]) & 0xffffffff) >> 10


def constrain(diff, thr, shift):
    ad = np.abs(diff)
    v = np.minimum(ad, np.maximum(0, thr - (ad >> shift)))
    return np.where(diff < 0, -v, v)


def filt(t, h, w, pri, sec, d, damping, bdmax):
    """cdef_filter_block_c, src/cdef_tmpl.c:104-215, on the (h+4) x (w+4)
    neighbourhood t (NONE where absent)."""
    bd8 = bdmax.bit_length() - 8
    px = t[2:2 + h, 2:2 + w]
    tap = lambda dy, dx: t[2 + dy:2 + dy + h, 2 + dx:2 + dx + w]  # noqa: E731
    s = np.zeros((h, w), np.int64)
    mn, mx = px.copy(), px.copy()
    pri_tap = 4 - ((pri >> bd8) & 1)
    for k in range(2):
        taps = []
        if pri:
            (dy, dx) = DIRS[d][k]
            for q in (tap(dy, dx), tap(-dy, -dx)):
                s += (pri_tap if k == 0 else (pri_tap & 3) | 2) * constrain(q - px, pri, max(0, damping - ulog2(pri)))
                taps.append(q)
        if sec:
            for dd in ((d + 2) & 7, (d + 6) & 7):
                (dy, dx) = DIRS[dd][k]
                for q in (tap(dy, dx), tap(-dy, -dx)):
                    s += (2 - k) * constrain(q - px, sec, damping - ulog2(sec))
                    taps.append(q)
        for q in taps:
            mn = np.where(q.astype(np.uint32) < mn.astype(np.uint32), q, mn)
            mx = np.maximum(mx, q)
    v = px + ((s - (s < 0) + 8) >> 4)
    if pri and sec:
        v = np.clip(v, mn, mx)
    return v


def np_cdef_frame(case):
    """The frame-level meaning: each 8x8 block filtered from the pristine
    deblocked picture (dav1d_cdef_brow's strength / skip / direction logic,
    src/cdef_apply_tmpl.c:124-296)."""
    bdmax, lay = case.bitdepth_max, case.layout
    bd8 = bdmax.bit_length() - 8
    bw, bh = ((case.width + 7) >> 3) << 1, ((case.height + 7) >> 3) << 1
    sx, sy = int(lay != 3), int(lay == 1)
    pads, outs = [], []
    for a in case.planes:
        p = np.full((a.shape[0] + 4, a.shape[1] + 4), NONE, np.int64)
        p[2:-2, 2:-2] = a
        pads.append(p)
        outs.append(a.copy())
    uv_dir = [0, 1, 2, 3, 4, 5, 6, 7] if lay != 2 else [7, 0, 2, 4, 5, 6, 6, 6]
    strength = lambda lvl: ((lvl >> 2) << bd8, ((lvl & 3) + ((lvl & 3) == 3)) << bd8)  # noqa: E731
    for by in range(0, bh, 2):
        for bx in range(0, bw, 2):
            idx = int(case.cdef_idx[by >> 4, bx >> 4])
            if idx < 0 or not (case.y_strength[idx] or case.uv_strength[idx]):
                continue
            if not case.noskip[by >> 1, bx >> 1]:
                continue
            (ypri, ysec), (uvpri, uvsec) = strength(case.y_strength[idx]), strength(case.uv_strength[idx])
            damping = case.damping + bd8
            d, var = 0, 0
            if ypri or uvpri:
                d, var = find_dir(case.planes[0][by * 4:by * 4 + 8, bx * 4:bx * 4 + 8], bdmax)
            if ypri:
                adj = 0 if not var else (ypri * (4 + (min(ulog2(var >> 6), 12) if var >> 6 else 0)) + 8) >> 4
                job = (adj, ysec, d) if (adj or ysec) else None
            else:
                job = (0, ysec, 0) if ysec else None
            if job:
                y0, x0 = by * 4, bx * 4
                outs[0][y0:y0 + 8, x0:x0 + 8] = filt(pads[0][y0:y0 + 12, x0:x0 + 12], 8, 8, *job, damping, bdmax)
            if case.uv_strength[idx] and lay:
                h, w = 8 >> sy, 8 >> sx
                y0, x0 = (by * 4) >> sy, (bx * 4) >> sx
                for pl in (1, 2):
                    outs[pl][y0:y0 + h, x0:x0 + w] = filt(pads[pl][y0:y0 + h + 4, x0:x0 + w + 4], h, w, uvpri, uvsec,
                                                          uv_dir[d] if uvpri else 0, damping - 1, bdmax)
    return outs


CASES = [(8, 255, 1, 0), (8, 255, 2, 1), (8, 255, 3, 0), (8, 255, 0, 1),
         (16, 1023, 1, 1), (16, 1023, 3, 0), (16, 4095, 1, 0), (16, 4095, 2, 1)]


@pytest.mark.parametrize("bpc,bdmax,layout,sb128", CASES)
def test_walker_equals_frame_meaning(oracle, bpc, bdmax, layout, sb128):
    """Oracle walker (in place + backups) == pristine-copy restatement, odd grid sizes included."""
    import dav1d_mirror_amd.cdef as cdef
    for seed, (w, h) in enumerate([(200, 116), (132, 260)]):
        c = cdef.make_cdef_case(seed=10 * bpc + layout + seed, width=w, height=h, bpc=bpc, bitdepth_max=bdmax,
                                layout=layout)
        got = oracle.cdef_frame(c, sb128)
        want = np_cdef_frame(c)
        for p, (a, b) in enumerate(zip(got, want)):
            bad = np.argwhere(a != b)
            assert len(bad) == 0, f"plane {p}: {len(bad)} differ, first {bad[:5].tolist()}"
        assert any(not np.array_equal(a, b) for a, b in zip(got, c.planes)), "the case filtered nothing"


def test_sb_size_does_not_matter(oracle):
    import dav1d_mirror_amd.cdef as cdef
    c = cdef.make_cdef_case(seed=3, width=300, height=270)
    for a, b in zip(oracle.cdef_frame(c, 0), oracle.cdef_frame(c, 1)):
        assert np.array_equal(a, b)


def test_skipped_frame_is_a_copy(oracle):
    import dav1d_mirror_amd.cdef as cdef
    c = cdef.make_cdef_case(seed=4, width=120, height=72)
    c.cdef_idx[:] = -1
    for a, b in zip(oracle.cdef_frame(c), c.planes):
        assert np.array_equal(a, b)
    c = cdef.make_cdef_case(seed=5, width=120, height=72, p_noskip=0.0)
    for a, b in zip(oracle.cdef_frame(c), c.planes):
        assert np.array_equal(a, b)


def _dsp_block(bpc, img):
    pdt = np.uint8 if bpc == 8 else np.uint16
    return np.ascontiguousarray(img.astype(pdt))


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_find_dir_known_answers(oracle, bpc, bdmax):
    """Rows constant -> horizontal (2); columns constant -> vertical (6);
    constant along x + y -> 45 degrees up-right (0); along x - y -> (4);
    flat -> 0 with variance 0."""
    c = oracle.cdef_dsp(bpc)
    hbd = [] if bpc == 8 else [bdmax]
    rng = np.random.default_rng(1)
    v = rng.integers(0, bdmax + 1, 16)
    yy, xx = np.mgrid[0:8, 0:8]
    for img, want in [(v[yy], 2), (v[xx], 6), (v[xx + yy], 0), (v[7 - xx + yy], 4), (np.full((8, 8), v[0]), 0)]:
        b = _dsp_block(bpc, img)
        var = ctypes.c_uint()
        d = c.dir(b.ctypes.data, b.strides[0], ctypes.byref(var), *hbd)
        assert d == want, (d, want)
        assert (d, var.value) == find_dir(b, bdmax)
    # random blocks: the two restatements agree on direction and variance
    for _ in range(200):
        b = _dsp_block(bpc, rng.integers(0, bdmax + 1, (8, 8)))
        var = ctypes.c_uint()
        d = c.dir(b.ctypes.data, b.strides[0], ctypes.byref(var), *hbd)
        assert (d, var.value) == find_dir(b, bdmax)


def test_flat_picture_unchanged(oracle):
    import dav1d_mirror_amd.cdef as cdef
    c = cdef.make_cdef_case(seed=6, width=128, height=64, p_skip_sb=0.0, p_noskip=1.0)
    c.planes = [np.full_like(a, 77) for a in c.planes]
    for a, b in zip(oracle.cdef_frame(c), c.planes):
        assert np.array_equal(a, b)
