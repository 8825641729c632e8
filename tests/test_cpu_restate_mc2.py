"""A second, independent restatement of the rest of the mc / itx tables in
numpy, checked against the C oracle (oracle/dsp_ref.c) over checkasm's
iteration spaces at 8, 10 and 12 bit -- the entries tests/test_cpu_restate.py
does not cover:

* scaled mc: put / prep_8tap_scaled and the bilinear scaled pair
  (src/mc_tmpl.c:173-328, :452-585), tests/checkasm/mc.c:169-275 (steps
  1..2048 and the dy = 1.0 / 2.0 paths);
* warp8x8 / warp8x8t (src/mc_tmpl.c:758-825), checkasm :565-640;
* blend / blend_v / blend_h (:641-681), checkasm :447-563;
* emu_edge (:827-875) over all 15 edge cases of checkasm :646-721;
* the 64-point inverse DCT (src/itx_1d.c:436-781) through every itx entry
  with a 64-point side (src/itx_tmpl.c:102-160), eob 0 / partial / full.

This restatement computes positions in closed form where the reference
steps them (the scaled / warp filters' running sums), reads emu_edge as a
clamp of every coordinate, and writes the 64-point DCT's rotations as
direct products in int64 where the reference uses (c - 4096) forms; the
filters come from csrc/dsp_tables.h (generated from src/tables.c).  The
reference holds no known-answer vectors for these functions.
"""
import ctypes
import os

import numpy as np
import pytest

import test_cpu_restate as R

ROOT = R.ROOT
SUBPEL = R.SUBPEL
WARP = R._table("dspt_warp").reshape(193, 8)
OBMC = R._table("dspt_obmc")
_r, _s181 = R._r, R._s181


def _lib():
    return ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))


def _ib(bdmax):
    return 4 if bdmax == 255 else 14 - bdmax.bit_length()


def _pb(bdmax):
    return 0 if bdmax == 255 else 8192


# --------------------------------------------------------------- scaled mc
def _bank(ftype, frac, n, horiz):
    """GET_H_FILTER / GET_V_FILTER (src/mc_tmpl.c:99-108) for a 0..15 fraction per position."""
    t = ftype & 3 if horiz else ftype >> 2
    b = t if n > 4 else 3 + (t & 1)
    f = np.zeros((len(frac), 8), np.int64)
    nz = frac > 0
    f[nz] = SUBPEL[b, frac[nz] - 1]
    return f, nz


def scaled_8tap(src, w, h, mx, my, dx, dy, ftype, bdmax, prep):
    """put / prep_8tap_scaled for src (int64, origin at [3, 3] plus margins)."""
    ib, pb = _ib(bdmax), _pb(bdmax)
    px = mx + np.arange(w) * dx
    col, fx = px >> 10, (px & 1023) >> 6
    fh, hnz = _bank(ftype, fx, w, True)
    rows = (((h - 1) * dy + my) >> 10) + 8
    mid = np.zeros((rows, w), np.int64)
    for r in range(rows):
        line = src[r]   # source row r - 3 of the block
        taps = np.stack([line[3 + col - 3 + k] for k in range(8)], 1)
        mid[r] = np.where(hnz, _r((taps * fh).sum(1), 6 - ib), line[3 + col] << ib)
    py = my + np.arange(h) * dy
    base, fy = py >> 10, (py & 1023) >> 6
    fv, vnz = _bank(ftype, fy, h, False)
    out = np.zeros((h, w), np.int64)
    for y in range(h):
        if vnz[y]:
            acc = sum(fv[y, k] * mid[base[y] + k] for k in range(8))
            out[y] = _r(acc, 6) - pb if prep else np.clip(_r(acc, 6 + ib), 0, bdmax)
        else:
            m = mid[base[y] + 3]
            out[y] = m - pb if prep else np.clip(_r(m, ib) if ib else m, 0, bdmax)
    return out


def scaled_bilin(src, w, h, mx, my, dx, dy, bdmax, prep):
    """put / prep_bilin_scaled: no filter margin, rows from the block's own top."""
    ib, pb = _ib(bdmax), _pb(bdmax)
    px = mx + np.arange(w) * dx
    col, fx = px >> 10, (px & 1023) >> 6
    rows = (((h - 1) * dy + my) >> 10) + 2
    mid = np.zeros((rows, w), np.int64)
    for r in range(rows):
        line = src[3 + r]
        a, b = line[3 + col], line[3 + col + 1]
        mid[r] = _r(16 * a + fx * (b - a), 4 - ib) if ib < 4 else 16 * a + fx * (b - a)
    py = my + np.arange(h) * dy
    base, fy = py >> 10, (py & 1023) >> 6
    out = np.zeros((h, w), np.int64)
    for y in range(h):
        a, b = mid[base[y]], mid[base[y] + 1]
        v = 16 * a + fy[y] * (b - a)
        out[y] = _r(v, 4) - pb if prep else np.clip(_r(v, 4 + ib), 0, bdmax)
    return out


def _h_next(h):   # tests/checkasm/mc.c:43-56
    return {2: 4, 4: 6, 6: 8, 8: 12, 12: 16, 16: 24, 24: 32, 32: 64, 64: 128}.get(h, 256)


@pytest.mark.parametrize("bdmax", [255, 1023, 4095])
def test_scaled_mc_restatement_matches_oracle(bdmax):
    hbd = bdmax > 255
    L = _lib()
    tab = (ctypes.c_void_p * 53)()
    getattr(L, f"oracle_mc_dsp_init_{16 if hbd else 8}bpc")(ctypes.byref(tab))
    pdt, bpp = (np.uint16, 2) if hbd else (np.uint8, 1)
    VP, SZ, I = ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_int
    ex = [I] if hbd else []
    PUT = ctypes.CFUNCTYPE(None, VP, SZ, VP, SZ, I, I, I, I, I, I, *ex)
    PREP = ctypes.CFUNCTYPE(None, VP, VP, SZ, I, I, I, I, I, I, *ex)
    rng = np.random.default_rng(bdmax + 31)
    S = 263
    buf = rng.integers(0, bdmax + 1, (S, S)).astype(pdt)
    s64 = buf.astype(np.int64)
    n = 0
    for f in range(10):
        for w in (2, 4, 8, 16, 32, 64, 128):
            for p in range(3):
                hs, h = [], 2 if w <= 32 else w // 4
                while h <= max(min(w * 4, 128), 32):
                    hs.append(h)
                    h = _h_next(h)
                for h in rng.choice(hs, size=min(2, len(hs)), replace=False):
                    h = int(h)
                    mx, my = int(rng.integers(0, 1024)), int(rng.integers(0, 1024))
                    dx = int(rng.integers(1, 2049))
                    dy = int(rng.integers(1, 2049)) if not p else p << 10
                    if (((h - 1) * dy + my) >> 10) + 8 > S - 8 or (((w - 1) * dx + mx) >> 10) + 8 > S - 8:
                        continue
                    src_p = buf.ctypes.data + (3 * S + 3) * bpp
                    want = scaled_bilin(s64, w, h, mx, my, dx, dy, bdmax, False) if f == 9 else \
                        scaled_8tap(s64, w, h, mx, my, dx, dy, R.FT[f], bdmax, False)
                    dst = np.zeros((h, w), pdt)
                    PUT(tab[10 + f])(dst.ctypes.data, w * bpp, src_p, S * bpp, w, h, mx, my, dx, dy,
                                     *([bdmax] if hbd else []))
                    assert np.array_equal(dst, want.astype(pdt)), f"put_scaled f{f} {w}x{h} m{mx},{my} d{dx},{dy}"
                    if w >= 4 and h >= max(w // 4, 4):
                        want = scaled_bilin(s64, w, h, mx, my, dx, dy, bdmax, True) if f == 9 else \
                            scaled_8tap(s64, w, h, mx, my, dx, dy, R.FT[f], bdmax, True)
                        tmp = np.zeros((h, w), np.int16)
                        PREP(tab[30 + f])(tmp.ctypes.data, src_p, S * bpp, w, h, mx, my, dx, dy,
                                          *([bdmax] if hbd else []))
                        assert np.array_equal(tmp, want.astype(np.int16)), \
                            f"prep_scaled f{f} {w}x{h} m{mx},{my} d{dx},{dy}"
                    n += 1
    assert n > 300


# -------------------------------------------------------------------- warp
def warp(src, abcd, mx, my, bdmax, prep):
    """warp_affine_8x8(t): src int64 15 x 15 (the 8x8 at [3, 3])."""
    ib, pb = _ib(bdmax), _pb(bdmax)
    a, b, c, d = (int(v) for v in abcd)
    r = np.arange(15)[:, None]
    x = np.arange(8)[None, :]
    fx = WARP[64 + ((mx + r * b + x * a + 512) >> 10)]          # (15, 8, 8) taps per position
    win = np.stack([src[:, x0:x0 + 8] for x0 in range(8)], 1)   # (15, 8 positions, 8 taps)
    mid = _r((fx * win).sum(2), 7 - ib)
    y = np.arange(8)[:, None]
    fy = WARP[64 + ((my + y * d + x * c + 512) >> 10)]          # (8, 8, 8)
    colwin = np.stack([mid[y0:y0 + 8] for y0 in range(8)], 0)   # (8 rows, 8 taps, 8 cols)
    acc = (fy * colwin.transpose(0, 2, 1)).sum(2)
    return _r(acc, 7) - pb if prep else np.clip(_r(acc, 7 + ib), 0, bdmax)


@pytest.mark.parametrize("bdmax", [255, 1023, 4095])
def test_warp_restatement_matches_oracle(bdmax):
    hbd = bdmax > 255
    L = _lib()
    tab = (ctypes.c_void_p * 53)()
    getattr(L, f"oracle_mc_dsp_init_{16 if hbd else 8}bpc")(ctypes.byref(tab))
    pdt, bpp = (np.uint16, 2) if hbd else (np.uint8, 1)
    VP, SZ, I = ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_int
    ex = [I] if hbd else []
    W8 = ctypes.CFUNCTYPE(None, VP, SZ, VP, SZ, VP, I, I, *ex)
    rng = np.random.default_rng(bdmax + 77)
    for it in range(300):   # checkasm :565-640: mx, my, abcd = (rnd & 0x1fff) - 0xa00
        mx, my = (int(v) for v in (rng.integers(0, 0x2000, 2) - 0xa00))
        abcd = (rng.integers(0, 0x2000, 4) - 0xa00).astype(np.int16)
        src = rng.integers(0, bdmax + 1, (15, 15)).astype(pdt)
        sp = src.ctypes.data + (15 * 3 + 3) * bpp
        dst = np.zeros((8, 8), pdt)
        W8(tab[49])(dst.ctypes.data, 8 * bpp, sp, 15 * bpp, abcd.ctypes.data, mx, my, *([bdmax] if hbd else []))
        assert np.array_equal(dst, warp(src.astype(np.int64), abcd, mx, my, bdmax, False).astype(pdt)), it
        tmp = np.zeros((8, 8), np.int16)
        W8(tab[50])(tmp.ctypes.data, 8, sp, 15 * bpp, abcd.ctypes.data, mx, my, *([bdmax] if hbd else []))
        assert np.array_equal(tmp, warp(src.astype(np.int64), abcd, mx, my, bdmax, True).astype(np.int16)), it


# ------------------------------------------------------- blend / emu_edge
@pytest.mark.parametrize("bdmax", [255, 1023, 4095])
def test_blend_and_emu_edge_restatement_matches_oracle(bdmax):
    hbd = bdmax > 255
    L = _lib()
    tab = (ctypes.c_void_p * 53)()
    getattr(L, f"oracle_mc_dsp_init_{16 if hbd else 8}bpc")(ctypes.byref(tab))
    pdt, bpp = (np.uint16, 2) if hbd else (np.uint8, 1)
    VP, SZ, I, IP = ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_int, ctypes.c_ssize_t
    BLEND = ctypes.CFUNCTYPE(None, VP, SZ, VP, I, I, VP)
    BDIR = ctypes.CFUNCTYPE(None, VP, SZ, VP, I, I)
    EMU = ctypes.CFUNCTYPE(None, IP, IP, IP, IP, IP, IP, VP, SZ, VP, SZ)
    rng = np.random.default_rng(bdmax + 5)
    bl = lambda a, b, m: (a * (64 - m) + b * m + 32) >> 6  # noqa: E731
    n = 0
    for w in (4, 8, 16, 32):   # blend: checkasm :447-486
        for h in (4, 8, 16, 32):
            if not max(w // 2, 4) <= h <= min(w * 2, 32):
                continue
            dst = rng.integers(0, bdmax + 1, (h, w)).astype(pdt)
            tmp = rng.integers(0, bdmax + 1, (h, w)).astype(pdt)
            m = rng.integers(0, 65, (h, w)).astype(np.uint8)
            want = bl(dst.astype(np.int64), tmp.astype(np.int64), m.astype(np.int64))
            BLEND(tab[46])(dst.ctypes.data, w * bpp, tmp.ctypes.data, w, h, m.ctypes.data)
            assert np.array_equal(dst, want.astype(pdt)), f"blend {w}x{h}"
            n += 1
    for w in (2, 4, 8, 16, 32):   # blend_v: the left 3/4 of the columns, mask by column
        for h in [2 << k for k in range(7)]:
            if h > (64 if w == 2 else 128):
                continue
            dst = rng.integers(0, bdmax + 1, (h, w)).astype(pdt)
            tmp = rng.integers(0, bdmax + 1, (h, w)).astype(pdt)
            want = dst.astype(np.int64)
            c = (w * 3) >> 2
            want[:, :c] = bl(want[:, :c], tmp[:, :c].astype(np.int64), OBMC[w:w + c][None, :])
            BDIR(tab[47])(dst.ctypes.data, w * bpp, tmp.ctypes.data, w, h)
            assert np.array_equal(dst, want.astype(pdt)), f"blend_v {w}x{h}"
            n += 1
    for w in (2, 4, 8, 16, 32, 64, 128):   # blend_h: the top 3/4 of the rows, mask by row
        for h in (2, 4, 8, 16, 32):
            if w == 128 and h < 4:
                continue
            dst = rng.integers(0, bdmax + 1, (h, w)).astype(pdt)
            tmp = rng.integers(0, bdmax + 1, (h, w)).astype(pdt)
            want = dst.astype(np.int64)
            r = (h * 3) >> 2
            want[:r] = bl(want[:r], tmp[:r].astype(np.int64), OBMC[h:h + r][:, None])
            BDIR(tab[48])(dst.ctypes.data, w * bpp, tmp.ctypes.data, w, h)
            assert np.array_equal(dst, want.astype(pdt)), f"blend_h {w}x{h}"
            n += 1
    # emu_edge: every pixel of the bw x bh window at (x, y) reads the plane at
    # the clamped coordinate (checkasm :646-721, all 15 edge cases)
    src = rng.integers(0, bdmax + 1, (160, 160)).astype(pdt)
    for w in (4, 8, 16, 32, 64, 128):
        for h in [4 << k for k in range(6)]:
            if not max(w // 4, 4) <= h <= min(w * 4, 128):
                continue
            for edge in range(15):
                bw, bh = w + int(rng.integers(0, 8)), h + int(rng.integers(0, 8))
                x, iw = _edge_offset(rng, edge & 12, bw, 4, 8)
                y, ih = _edge_offset(rng, edge & 3, bh, 1, 2)
                dst = np.zeros((bh, 192), pdt)
                EMU(tab[51])(bw, bh, iw, ih, x, y, dst.ctypes.data, 192 * bpp, src.ctypes.data, 160 * bpp)
                yy = np.clip(y + np.arange(bh), 0, ih - 1)[:, None]
                xx = np.clip(x + np.arange(bw), 0, iw - 1)[None, :]
                assert np.array_equal(dst[:, :bw], src[yy, xx]), f"emu_edge {bw}x{bh} edge {edge}"
                n += 1
    assert n > 400


def _edge_offset(rng, have, b, first, second):
    """random_offset_for_edge (tests/checkasm/mc.c:652-677) for one axis:
    `first` is HAVE_TOP / HAVE_LEFT, `second` HAVE_BOTTOM / HAVE_RIGHT."""
    i = 160 if have else 1 + int(rng.integers(0, b - 2))
    if have == first | second:
        pos = int(rng.integers(0, i - b + 1))
    elif have == first:
        pos = (i - b) + 1 + int(rng.integers(0, b - 1))
    elif have == second:
        pos = -(1 + int(rng.integers(0, b - 1)))
    else:
        pos = -(1 + int(rng.integers(0, b - i - 1)))
    return pos, i


# ---------------------------------------------------------- 64-point DCT
def dct64(c, cl):
    """The 64-point inverse DCT (src/itx_1d.c:436-781) on (N, 64) rows
    whose entries 32..63 are zero: the 32-point DCT of the even inputs,
    then the odd half in direct int64 products."""
    e = R.dct32(c[:, 0:64:2].copy(), cl)
    i = {k: c[:, k] for k in range(1, 32, 2)}
    t = {}
    # stage 1: single rotations of the odd inputs (their partners are the zero upper half)
    s1 = [(32, 1, 101), (33, 31, -2824), (34, 17, 1660), (35, 15, -1474), (36, 9, 897), (37, 23, -2191),
          (38, 25, 2359), (39, 7, -700), (40, 5, 501), (41, 27, -2520), (42, 21, 2019), (43, 11, -1092),
          (44, 13, 1285), (45, 19, -1842), (46, 29, 2675), (47, 3, -301), (48, 3, 4085), (49, 29, 3102),
          (50, 19, 3659), (51, 13, 3889), (52, 11, 3948), (53, 21, 3564), (54, 27, 3229), (55, 5, 4065),
          (56, 7, 4036), (57, 25, 3349), (58, 23, 3461), (59, 9, 3996), (60, 15, 3822), (61, 17, 3745),
          (62, 31, 2967), (63, 1, 4095)]
    a = {k: _r(i[src] * m, 12) for k, src, m in s1}
    # stage 2: butterflies in groups of four (+, -, -, + with the pair order swapped in the second half)
    for g in range(32, 64, 4):
        t[g], t[g + 1] = cl(a[g] + a[g + 1]), cl(a[g] - a[g + 1])
        t[g + 2], t[g + 3] = cl(a[g + 3] - a[g + 2]), cl(a[g + 3] + a[g + 2])

    def rot(x, y, cx, cy, sh=12):
        return _r(x * cx + y * cy, sh)
    # stage 3
    u = dict(t)
    u[33], u[62] = rot(t[33], t[62], -4076, 401), rot(t[33], t[62], 401, 4076)
    u[34], u[61] = rot(t[34], t[61], -401, -4076), rot(t[34], t[61], -4076, 401)
    u[37], u[58] = rot(t[37], t[58], -1299, 1583, 11), rot(t[37], t[58], 1583, 1299, 11)
    u[38], u[57] = rot(t[38], t[57], -1583, -1299, 11), rot(t[38], t[57], -1299, 1583, 11)
    u[41], u[54] = rot(t[41], t[54], -3612, 1931), rot(t[41], t[54], 1931, 3612)
    u[42], u[53] = rot(t[42], t[53], -1931, -3612), rot(t[42], t[53], -3612, 1931)
    u[45], u[50] = rot(t[45], t[50], -1189, 3920), rot(t[45], t[50], 3920, 1189)
    u[46], u[49] = rot(t[46], t[49], -3920, -1189), rot(t[46], t[49], -1189, 3920)
    # stage 4: butterflies of spans of 4 (lo + hi, inner pairs crossed)
    v = {}
    for g in range(32, 64, 8):
        v[g], v[g + 3] = cl(u[g] + u[g + 3]), cl(u[g] - u[g + 3])
        v[g + 1], v[g + 2] = cl(u[g + 1] + u[g + 2]), cl(u[g + 1] - u[g + 2])
        v[g + 4], v[g + 7] = cl(u[g + 7] - u[g + 4]), cl(u[g + 7] + u[g + 4])
        v[g + 5], v[g + 6] = cl(u[g + 6] - u[g + 5]), cl(u[g + 6] + u[g + 5])
    # stage 5
    w_ = dict(v)
    w_[34], w_[61] = rot(v[34], v[61], -4017, 799), rot(v[34], v[61], 799, 4017)
    w_[35], w_[60] = rot(v[35], v[60], -4017, 799), rot(v[35], v[60], 799, 4017)
    w_[36], w_[59] = rot(v[36], v[59], -799, -4017), rot(v[36], v[59], -4017, 799)
    w_[37], w_[58] = rot(v[37], v[58], -799, -4017), rot(v[37], v[58], -4017, 799)
    w_[42], w_[53] = rot(v[42], v[53], -1138, 1703, 11), rot(v[42], v[53], 1703, 1138, 11)
    w_[43], w_[52] = rot(v[43], v[52], -1138, 1703, 11), rot(v[43], v[52], 1703, 1138, 11)
    w_[44], w_[51] = rot(v[44], v[51], -1703, -1138, 11), rot(v[44], v[51], -1138, 1703, 11)
    w_[45], w_[50] = rot(v[45], v[50], -1703, -1138, 11), rot(v[45], v[50], -1138, 1703, 11)
    # stage 6: butterflies of spans of 8
    x = {}
    for g in range(32, 64, 16):
        for k in range(4):
            x[g + k], x[g + 7 - k] = cl(w_[g + k] + w_[g + 7 - k]), cl(w_[g + k] - w_[g + 7 - k])
            x[g + 8 + k], x[g + 15 - k] = cl(w_[g + 15 - k] - w_[g + 8 + k]), cl(w_[g + 15 - k] + w_[g + 8 + k])
    # stage 7
    y = dict(x)
    for lo, hi in ((36, 59), (37, 58), (38, 57), (39, 56)):
        y[lo], y[hi] = rot(x[lo], x[hi], -3784, 1567), rot(x[lo], x[hi], 1567, 3784)
    for lo, hi in ((40, 55), (41, 54), (42, 53), (43, 52)):
        y[lo], y[hi] = rot(x[lo], x[hi], -1567, -3784), rot(x[lo], x[hi], -3784, 1567)
    # stage 8: butterflies of spans of 16
    z = {}
    for k in range(8):
        z[32 + k], z[47 - k] = cl(y[32 + k] + y[47 - k]), cl(y[32 + k] - y[47 - k])
        z[48 + k], z[63 - k] = cl(y[63 - k] - y[48 + k]), cl(y[63 - k] + y[48 + k])
    # stage 9: the 181/256 rotations of the middle
    f = dict(z)
    for k in range(8):
        f[40 + k], f[55 - k] = _s181(z[55 - k] - z[40 + k]), _s181(z[40 + k] + z[55 - k])
    o = [f[63 - k] for k in range(32)]
    return np.concatenate([np.stack([cl(e[:, k] + o[k]) for k in range(32)], 1),
                           np.stack([cl(e[:, 31 - k] - o[31 - k]) for k in range(32)], 1)], 1)


SHIFT64 = {(16, 64): 2, (32, 64): 1, (64, 16): 2, (64, 32): 1, (64, 64): 2}


def inv_txfm_add_64(dst, coeff, eob, w, h, bdmax):
    """inv_txfm_add_c (src/itx_tmpl.c:40-100), DCT_DCT, a 64-point side."""
    shift = SHIFT64[(w, h)]
    rect2 = w * 2 == h or h * 2 == w
    rnd = (1 << shift) >> 1
    if eob < 1:
        dc = int(coeff[0])
        coeff[0] = 0
        if rect2:
            dc = _s181(dc)
        dc = (_s181(dc) + rnd) >> shift
        return np.clip(dst + ((dc * 181 + 128 + 2048) >> 12), 0, bdmax)
    sw, sh = min(w, 32), min(h, 32)
    rmin = -32768 if bdmax == 255 else -((bdmax + 1) << 7)
    cmin = -32768 if bdmax == 255 else -((bdmax + 1) << 5)
    rcl = lambda v: np.clip(v, rmin, ~rmin)  # noqa: E731
    ccl = lambda v: np.clip(v, cmin, ~cmin)  # noqa: E731
    one = lambda c, cl: dct64(c, cl) if c.shape[1] == 64 else R.DCT[c.shape[1]](c, cl)  # noqa: E731
    rows = np.zeros((sh, w), np.int64)
    rows[:, :sw] = coeff[:sw * sh].astype(np.int64).reshape(sw, sh).T
    if rect2:
        rows = _s181(rows)
    rows = one(rows, rcl)
    coeff[:sw * sh] = 0
    tmp = np.zeros((h, w), np.int64)
    tmp[:sh] = ccl((rows + rnd) >> shift)
    cols = one(tmp.T.copy(), ccl).T
    return np.clip(dst + ((cols + 8) >> 4), 0, bdmax)


@pytest.mark.parametrize("bdmax", [255, 1023, 4095])
def test_dct64_restatement_matches_oracle(bdmax):
    hbd = bdmax > 255
    L = _lib()
    tab = R._itx_table(L, hbd)
    pdt, cdt = (np.uint16, np.int32) if hbd else (np.uint8, np.int16)
    args = [ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p, ctypes.c_int] + ([ctypes.c_int] if hbd else [])
    FN = ctypes.CFUNCTYPE(None, *args)
    rng = np.random.default_rng(bdmax + 64)
    cmax = 32767 if not hbd else (~(~127 << (bdmax.bit_length()))) & 0x7fffffff
    n = 0
    for tx, (w, h) in enumerate(R.TX_WH):
        if max(w, h) != 64:
            continue
        fn = FN(tab[tx * 17 + 0])   # DCT_DCT, the only type with a 64-point side
        sw, sh = min(w, 32), min(h, 32)
        for it in range(9):
            dst = rng.integers(0, bdmax + 1, (h, w)).astype(pdt)
            cf = np.zeros(sw * sh, cdt)
            reg = [(1, 1), (max(1, sw // 2), max(1, sh // 2)), (sw, sh)][it % 3]
            amp = [64, bdmax * 8, cmax][it // 3]
            blk = rng.integers(-amp, amp + 1, size=(reg[0], reg[1]))
            for x in range(reg[0]):
                cf[x * sh:x * sh + reg[1]] = blk[x]
            eob = 0 if it == 0 else 1 + int(rng.integers(0, sw * sh))
            want = inv_txfm_add_64(dst.astype(np.int64), cf.astype(np.int64).copy(), eob, w, h, bdmax)
            got, gcf = dst.copy(), cf.copy()
            fn(*([got.ctypes.data, w * got.itemsize, gcf.ctypes.data, eob] + ([bdmax] if hbd else [])))
            assert np.array_equal(got, want.astype(pdt)), f"dct64 {w}x{h} case {it}"
            assert not gcf.any()
            n += 1
    assert n == 45


def test_dct64_known_answers():
    """A DC-only input spreads evenly: dct64(e0) is e0 * 181 / 256 everywhere
    (the even half's DC path, odd half zero)."""
    c = np.zeros((1, 64), np.int64)
    c[0, 0] = 1024
    cl = lambda v: np.clip(v, -32768, 32767)  # noqa: E731
    assert (dct64(c, cl) == _s181(1024)).all()
