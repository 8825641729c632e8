"""Loop-restoration oracle checks on CPU: the restated
wiener_c / sgr_*_c (src/looprestoration_tmpl.c) against properties the
reference's arithmetic guarantees and a second restatement of the Wiener
path in numpy.  The reference ships no vectors for these functions (its
checkasm is differential, tests/checkasm/looprestoration.c): parity against
the binary stays unpinned, as for the rest of the oracle."""
import ctypes

import numpy as np
import pytest

ST = 448


def _buffers(rng, bpc, bdmax):
    pdt = np.uint8 if bpc == 8 else np.uint16
    pic = rng.integers(0, bdmax + 1, (64 + 1, ST)).astype(pdt)
    lpf = rng.integers(0, bdmax + 1, (8, ST)).astype(pdt)
    left = rng.integers(0, bdmax + 1, (64, 4)).astype(pdt)
    return pic, lpf, left


def _call(fn, bpc, bdmax, pic, lpf, left, w, h, prm, edges):
    out = pic.copy()
    b = out.itemsize
    args = [out[1:].ctypes.data + 8 * b, ST * b, left.ctypes.data, lpf.ctypes.data + 8 * b, w, h, ctypes.byref(prm),
            edges]
    if bpc != 8:
        args.append(bdmax)
    fn(*args)
    return out


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_identity_filters(oracle, pkg, bpc, bdmax):
    """Wiener with a unit impulse and SGR with zero weights leave the unit unchanged, for every edge set."""
    c = oracle.lr_dsp(bpc, bdmax.bit_length())
    rng = np.random.default_rng(bpc + bdmax)
    pic, lpf, left = _buffers(rng, bpc, bdmax)
    prm = pkg.abi.LrParams()
    for k in range(7):
        prm.filter[0][k] = prm.filter[1][k] = 0
    prm.filter[0][3] = 0 if bpc == 8 else 128   # 8 bpc adds the 128 centre tap itself (:160-162)
    prm.filter[1][3] = 128
    for edges in range(16):
        out = _call(c.wiener[0], bpc, bdmax, pic, lpf, left, 200, 40, prm, edges)
        assert np.array_equal(out, pic), edges
    sg = pkg.abi.LrParams()
    sg.sgr.s0, sg.sgr.s1, sg.sgr.w0, sg.sgr.w1 = 140, 3236, 0, 0
    for k in range(3):
        out = _call(c.sgr[k], bpc, bdmax, pic, lpf, left, 130, 33, sg, 15)
        assert np.array_equal(out, pic), k


def _wiener_np(pic, lpf, left, w, h, f, edges, bpc, bdmax):
    """wiener_c (:134-190) over padding() (:40-132), restated with numpy."""
    hl, hr = edges & 1, (edges >> 1) & 1
    P = pic[1:].astype(np.int64)[:, 8:]
    Lp = lpf.astype(np.int64)   # the unit's column 0 is lpf column 8
    t = np.zeros((h + 6, w + 6), np.int64)
    for r in range(h + 6):
        for cc in range(w + 6):
            c = min(cc, w + 2) if not hr else cc
            c = max(c, 3) if not hl else c
            x = c - 3
            if r < 3:
                v = Lp[1 if r == 2 else 0, 8 + x] if edges & 4 else (left[0, x + 4] if x < 0 else P[0, x])
            elif r < h + 3:
                v = left[r - 3, x + 4] if x < 0 else P[r - 3, x]
            else:
                v = Lp[6 if r == h + 3 else 7, 8 + x] if edges & 8 else (left[h - 1, x + 4] if x < 0 else P[h - 1, x])
            t[r, cc] = v
    bd = bdmax.bit_length()
    rbh = 3 + 2 * (bd == 12)
    hor = np.full((h + 6, w), 1 << (bd + 6), np.int64)
    if bpc == 8:
        hor += t[:, 3:3 + w] * 128
    for k in range(7):
        hor += t[:, k:k + w] * f[0][k]
    hor = np.clip((hor + (1 << (rbh - 1))) >> rbh, 0, (1 << (bd + 1 + 7 - rbh)) - 1)
    rbv = 11 - 2 * (bd == 12)
    s = np.full((h, w), -(1 << (bd + rbv - 1)), np.int64)
    for k in range(7):
        s += hor[k:k + h] * f[1][k]
    return np.clip((s + (1 << (rbv - 1))) >> rbv, 0, bdmax)


@pytest.mark.parametrize("bpc,bdmax", [(8, 255), (16, 1023), (16, 4095)])
def test_wiener_two_restatements(oracle, pkg, bpc, bdmax):
    c = oracle.lr_dsp(bpc, bdmax.bit_length())
    rng = np.random.default_rng(7 * bpc + bdmax)
    for edges in range(16):
        pic, lpf, left = _buffers(rng, bpc, bdmax)
        prm = pkg.abi.LrParams()
        f = [[0] * 7, [0] * 7]
        for d in range(2):
            f[d][0] = f[d][6] = int(rng.integers(0, 16)) - 5
            f[d][1] = f[d][5] = int(rng.integers(0, 32)) - 23
            f[d][2] = f[d][4] = int(rng.integers(0, 64)) - 17
            f[d][3] = (128 if d else 0) - 2 * (f[d][0] + f[d][1] + f[d][2]) + (128 if (bpc != 8 and not d) else 0)
            for k in range(7):
                prm.filter[d][k] = f[d][k]
        w, h = int(rng.integers(1, 40)), int(rng.integers(1, 12))
        out = _call(c.wiener[0], bpc, bdmax, pic, lpf, left, w, h, prm, edges)
        want = _wiener_np(pic, lpf, left, w, h, f, edges, bpc, bdmax)
        assert np.array_equal(out[1:1 + h, 8:8 + w].astype(np.int64), want), edges
        assert not np.array_equal(out, pic)
