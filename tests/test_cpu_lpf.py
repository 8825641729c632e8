"""Deblocking oracle checks on CPU.

The oracle (oracle/dsp_ref.c) restates dav1d_loopfilter_sbrow_cols / _rows
(src/lf_apply_tmpl.c:314-466) and the loop_filter_sb DSP entries
(src/loopfilter_tmpl.c:37-245), run superblock row by superblock row, column
edges then row edges per row, as dav1d_filter_sbrow_deblock_cols / _rows
(src/recon_tmpl.c:2037-2069) do.  The restatement below decodes the same
Av1Filter masks edge by edge and filters the whole frame in two passes (every
column edge, then every row edge), the order the device uses.  The two agree
on every pixel, which pins the mask decoding and the pass-order argument
(no two edges of one pass touch the same pixel) on frames whose masks follow
the transform partition.  The reference ships no deblocking vectors (its
checkasm is differential, tests/checkasm/loopfilter.c): parity against the
binary stays unpinned, as for the rest of the oracle.
"""
import numpy as np
import pytest

# 13-tap outputs p5..q5 over s = p6..p0 q0..q6 (loopfilter_tmpl.c:94-117)
W16 = np.array([[7, 2, 2, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0],
                [5, 2, 2, 2, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0],
                [4, 1, 2, 2, 2, 1, 1, 1, 1, 1, 0, 0, 0, 0],
                [3, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 0, 0, 0],
                [2, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 0, 0],
                [1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 0],
                [0, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1],
                [0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 2],
                [0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 3],
                [0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 1, 4],
                [0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 5],
                [0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 7]])
W8 = np.array([[3, 2, 1, 1, 1, 0, 0, 0], [2, 1, 2, 1, 1, 1, 0, 0], [1, 1, 1, 2, 1, 1, 1, 0],
               [0, 1, 1, 1, 2, 1, 1, 1], [0, 0, 1, 1, 1, 2, 1, 2], [0, 0, 0, 1, 1, 1, 2, 3]])   # p2..q2 over p3..q3
W6 = np.array([[3, 2, 2, 1, 0, 0], [1, 2, 2, 2, 1, 0], [0, 1, 2, 2, 2, 1], [0, 0, 1, 2, 2, 3]])   # p1..q1 over p2..q2


def edge(line, E, I, H, wd, bdmax):
    """loop_filter(), one line: line[k] for k in -7..6 at index k + 7."""
    bd8 = bdmax.bit_length() - 8
    F = 1 << bd8
    E, I, H = int(E) << bd8, int(I) << bd8, int(H) << bd8
    p = [int(line[6 - k]) for k in range(7)]
    q = [int(line[7 + k]) for k in range(7)]
    fm = abs(p[1] - p[0]) <= I and abs(q[1] - q[0]) <= I and abs(p[0] - q[0]) * 2 + (abs(p[1] - q[1]) >> 1) <= E
    if wd > 4:
        fm = fm and abs(p[2] - p[1]) <= I and abs(q[2] - q[1]) <= I
    if wd > 6:
        fm = fm and abs(p[3] - p[2]) <= I and abs(q[3] - q[2]) <= I
    if not fm:
        return line
    flat_out = wd >= 16 and all(abs(p[k] - p[0]) <= F and abs(q[k] - q[0]) <= F for k in (4, 5, 6))
    flat_in = wd >= 6 and all(abs(p[k] - p[0]) <= F and abs(q[k] - q[0]) <= F for k in (1, 2))
    if wd >= 8:
        flat_in = flat_in and abs(p[3] - p[0]) <= F and abs(q[3] - q[0]) <= F
    out = line.copy()
    if wd >= 16 and flat_out and flat_in:
        out[1:13] = (W16 @ line[0:14].astype(np.int64) + 8) >> 4
    elif wd >= 8 and flat_in:
        out[4:10] = (W8 @ line[3:11].astype(np.int64) + 4) >> 3
    elif wd == 6 and flat_in:
        out[5:9] = (W6 @ line[4:10].astype(np.int64) + 4) >> 3
    else:
        lo, hi = -128 << bd8, (128 << bd8) - 1
        clip = lambda v: max(lo, min(hi, v))  # noqa: E731
        px = lambda v: max(0, min(bdmax, v))  # noqa: E731
        if abs(p[1] - p[0]) > H or abs(q[1] - q[0]) > H:
            f = clip(3 * (q[0] - p[0]) + clip(p[1] - q[1]))
            out[6], out[7] = px(p[0] + (min(f + 3, hi) >> 3)), px(q[0] - (min(f + 4, hi) >> 3))
        else:
            f = clip(3 * (q[0] - p[0]))
            f1, f2 = min(f + 4, hi) >> 3, min(f + 3, hi) >> 3
            out[6], out[7] = px(p[0] + f2), px(q[0] - f1)
            out[5], out[8] = px(p[1] + ((f1 + 1) >> 1)), px(q[1] - ((f1 + 1) >> 1))
    return out


def two_pass(case):
    """Every column edge of the frame, then every row edge, from the masks."""
    lay, bdmax = case.layout, case.bitdepth_max
    sx, sy = int(lay != 3), int(lay == 1)
    w4, h4 = (case.width + 3) >> 2, (case.height + 3) >> 2
    e, i, _ = case.lut
    pics = [np.pad(a.astype(np.int64), 8, constant_values=-9999) for a in case.planes]   # 128-aligned planes
    planes = [(0, 0, 0, 16, w4, h4)]
    if lay and case.filter_uv:
        planes += [(p, sx, sy, 16 >> (sy), (w4 + sx) >> sx, (h4 + sy) >> sy) for p in (1, 2)]
    for d in (0, 1):
        for (pl, ssx, ssy, _, cw, ch) in planes:
            cpx, cpy = 32 >> ssx, 32 >> ssy
            n_sizes = 3 if pl == 0 else 2
            comp = d if pl == 0 else 1 + pl
            for cy in range(ch):
                for cx in range(cw):
                    if (d == 0 and cx == 0) or (d == 1 and cy == 0):
                        continue
                    m = case.masks[cy // cpy, cx // cpx]
                    arr = m["filter_y"] if pl == 0 else m["filter_uv"]
                    if d == 0:
                        line, pos, per = cx % cpx, cy % cpy, 16 >> ssy
                    else:
                        line, pos, per = cy % cpy, cx % cpx, 16 >> ssx
                    half, bit = divmod(pos, per)
                    idx = [k for k in range(n_sizes) if (arr[d, line, k, half] >> bit) & 1]
                    if not idx:
                        continue
                    k = max(idx)
                    wd = (4 << k) if pl == 0 else 4 + 2 * k
                    L = int(case.level[cy, cx, comp]) or int(case.level[cy - (d == 1), cx - (d == 0), comp])
                    if not L:
                        continue
                    P = pics[pl]
                    for j in range(4):
                        if d == 0:
                            y, x = 8 + 4 * cy + j, 8 + 4 * cx
                            P[y, x - 7:x + 7] = edge(P[y, x - 7:x + 7], e[L], i[L], L >> 4, wd, bdmax)
                        else:
                            y, x = 8 + 4 * cy, 8 + 4 * cx + j
                            P[y - 7:y + 7, x] = edge(P[y - 7:y + 7, x], e[L], i[L], L >> 4, wd, bdmax)
    return [p[8:-8, 8:-8] for p in pics]


@pytest.mark.parametrize("bpc,bdmax,layout,sb128", [(8, 255, 1, 0), (8, 255, 2, 1), (8, 255, 3, 0), (8, 255, 0, 0),
                                                     (16, 1023, 1, 1), (16, 4095, 3, 0), (16, 4095, 2, 0)])
def test_walker_equals_two_pass(oracle, bpc, bdmax, layout, sb128):
    import dav1d_mirror_amd.lpf as lpf
    for seed, (w, h) in enumerate([(200, 120), (136, 260)]):
        c = lpf.make_lpf_case(seed=7 * bpc + layout + seed, width=w, height=h, bpc=bpc, bitdepth_max=bdmax,
                              layout=layout, sb128=sb128)
        got = oracle.loopfilter_frame(c)
        want = two_pass(c)
        for p, (a, b) in enumerate(zip(got, want)):
            bad = np.argwhere(a != b)
            assert len(bad) == 0, f"plane {p}: {len(bad)} differ, first {bad[:5].tolist()}"
        changed = [int((a != b).sum()) for a, b in zip(got, c.planes)]
        assert changed[0] > 0 and (not layout or changed[1] > 0), changed


def test_masks_follow_partition():
    """Every generated edge fits the smaller transform on either side (the
    property the two-pass order needs)."""
    import dav1d_mirror_amd.lpf as lpf
    c = lpf.make_lpf_case(seed=3, width=256, height=192)
    fy = c.masks["filter_y"]
    assert fy.any() and c.masks["filter_uv"].any()


def test_zero_levels_change_nothing(oracle):
    import dav1d_mirror_amd.lpf as lpf
    c = lpf.make_lpf_case(seed=4, width=160, height=96, p_zero_level=1.0)
    for a, b in zip(oracle.loopfilter_frame(c), c.planes):
        assert np.array_equal(a, b)
