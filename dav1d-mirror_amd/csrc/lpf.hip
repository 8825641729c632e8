// lpf.hip -- the deblocking loop filter on the device (SURVEY 8(f) row 3;
// include/dav1d_gpu.h, Dav1dLoopFilterDSPContext and
// Dav1dGpuLoopFilterFrame).
//
// Frame tier: dav1d_loopfilter_sbrow_cols / _rows (src/lf_apply_tmpl.c:
// 314-466) for a whole frame in two launches, k_lpf<BPC, ROWS>: every column
// edge, then every row edge, in place.  One thread per 4x4 cell of a plane
// decodes the cell's bit from the Av1Filter masks the way
// filter_plane_{cols,rows}_{y,uv} (:176-312) assemble them (64-row halves,
// have_left / have_top, the column bound of column edges), picks the level
// (the cell's, else its left / upper neighbour's, loopfilter_tmpl.c:174,
// :194) and filters the edge's 4 lines with loop_filter() (:37-161).
// Within a pass no two edges touch the same pixel, because a filter of
// length n needs transforms of at least n on both sides (what
// dav1d_create_lf_mask_* encode), so the threads are independent; the
// reference's per-superblock-row interleaving of the two passes touches
// disjoint rows (a row's row edges never reach the next row's pixels that
// its column edges read), so the two launches give its pixels.
//
// Per-call tier: the four loop_filter_sb entries.  The host reads the masks
// and levels (host memory, as the reference does) and stages exactly the
// pixels each filtered segment reads (2, 3, 4 or 7 on each side for lengths
// 4, 6, 8, 16); one thread per segment line on the device.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "dav1d_gpu.h"
#include "dsp_common.hpp"
#include "runtime.hpp"

namespace dgpu {

// loop_filter(), src/loopfilter_tmpl.c:37-161, one line: d points at q0,
// sb steps across the edge (pixels)
template <int BPC>
__device__ __forceinline__ void lpf_line(typename Px<BPC>::pixel *d, ptrdiff_t sb, int E, int I, int H, int wd,
                                         int bdmax) {
    using P = typename Px<BPC>::pixel;
    const int bd8 = bits_of(bdmax) - 8, F = 1 << bd8;
    E <<= bd8;
    I <<= bd8;
    H <<= bd8;
    const int p1 = d[-2 * sb], p0 = d[-sb], q0 = d[0], q1 = d[sb];
    int p2 = 0, q2 = 0, p3 = 0, q3 = 0;
    bool fm = abs(p1 - p0) <= I && abs(q1 - q0) <= I && abs(p0 - q0) * 2 + (abs(p1 - q1) >> 1) <= E;
    if (wd > 4) {
        p2 = d[-3 * sb];
        q2 = d[2 * sb];
        fm = fm && abs(p2 - p1) <= I && abs(q2 - q1) <= I;
        if (wd > 6) {
            p3 = d[-4 * sb];
            q3 = d[3 * sb];
            fm = fm && abs(p3 - p2) <= I && abs(q3 - q2) <= I;
        }
    }
    if (!fm) return;
    bool flat8in = false;
    if (wd >= 6) flat8in = abs(p2 - p0) <= F && abs(p1 - p0) <= F && abs(q1 - q0) <= F && abs(q2 - q0) <= F;
    if (wd >= 8) flat8in = flat8in && abs(p3 - p0) <= F && abs(q3 - q0) <= F;
    if (wd >= 16 && flat8in) {
        const int p6 = d[-7 * sb], p5 = d[-6 * sb], p4 = d[-5 * sb], q4 = d[4 * sb], q5 = d[5 * sb], q6 = d[6 * sb];
        if (abs(p6 - p0) <= F && abs(p5 - p0) <= F && abs(p4 - p0) <= F && abs(q4 - q0) <= F && abs(q5 - q0) <= F &&
            abs(q6 - q0) <= F) {
            // 13-tap smoothing (:94-117) as a running window: each output
            // drops two taps and adds two
            int s = p6 * 7 + p5 * 2 + p4 * 2 + p3 + p2 + p1 + p0 + q0;
            d[-6 * sb] = (P)((s + 8) >> 4);
            s += -p6 * 2 + p3 + q1;
            d[-5 * sb] = (P)((s + 8) >> 4);
            s += -p6 - p5 + p2 + q2;
            d[-4 * sb] = (P)((s + 8) >> 4);
            s += -p6 - p4 + p1 + q3;
            d[-3 * sb] = (P)((s + 8) >> 4);
            s += -p6 - p3 + p0 + q4;
            d[-2 * sb] = (P)((s + 8) >> 4);
            s += -p6 - p2 + q0 + q5;
            d[-sb] = (P)((s + 8) >> 4);
            s += -p6 - p1 + q1 + q6;
            d[0] = (P)((s + 8) >> 4);
            s += -p5 - p0 + q2 + q6;
            d[sb] = (P)((s + 8) >> 4);
            s += -p4 - q0 + q3 + q6;
            d[2 * sb] = (P)((s + 8) >> 4);
            s += -p3 - q1 + q4 + q6;
            d[3 * sb] = (P)((s + 8) >> 4);
            s += -p2 - q2 + q5 + q6;
            d[4 * sb] = (P)((s + 8) >> 4);
            s += -p1 - q3 + q6 * 2;
            d[5 * sb] = (P)((s + 8) >> 4);
            return;
        }
    }
    if (wd >= 8 && flat8in) {   // :118-124
        d[-3 * sb] = (P)((p3 * 3 + 2 * p2 + p1 + p0 + q0 + 4) >> 3);
        d[-2 * sb] = (P)((p3 * 2 + p2 + 2 * p1 + p0 + q0 + q1 + 4) >> 3);
        d[-sb] = (P)((p3 + p2 + p1 + 2 * p0 + q0 + q1 + q2 + 4) >> 3);
        d[0] = (P)((p2 + p1 + p0 + 2 * q0 + q1 + q2 + q3 + 4) >> 3);
        d[sb] = (P)((p1 + p0 + q0 + 2 * q1 + q2 + q3 * 2 + 4) >> 3);
        d[2 * sb] = (P)((p0 + q0 + q1 + 2 * q2 + q3 * 3 + 4) >> 3);
    } else if (wd == 6 && flat8in) {   // :125-129
        d[-2 * sb] = (P)((p2 * 3 + 2 * p1 + 2 * p0 + q0 + 4) >> 3);
        d[-sb] = (P)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
        d[0] = (P)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
        d[sb] = (P)((p0 + 2 * q0 + 2 * q1 + q2 * 3 + 4) >> 3);
    } else {   // :130-158
        const int lo = -128 * (1 << bd8), hi = 128 * (1 << bd8) - 1;
        const bool hev = abs(p1 - p0) > H || abs(q1 - q0) > H;
        int f = hev ? clampi(p1 - q1, lo, hi) : 0;
        f = clampi(3 * (q0 - p0) + f, lo, hi);
        const int f1 = min(f + 4, hi) >> 3, f2 = min(f + 3, hi) >> 3;
        d[-sb] = (P)clampi(p0 + f2, 0, bdmax);
        d[0] = (P)clampi(q0 - f1, 0, bdmax);
        if (!hev) {
            const int f3 = (f1 + 1) >> 1;
            d[-2 * sb] = (P)clampi(p1 + f3, 0, bdmax);
            d[sb] = (P)clampi(q1 - f3, 0, bdmax);
        }
    }
}

// (Round 5: a cell's four lines filtered from registers loaded all at once
// measured 46.9 against 37.9 us -- most lines stop after the mask test on
// four pixels -- and was deleted in round 6.)

template <int BPC> struct LpfArgs {
    using P = typename Px<BPC>::pixel;
    P *pic[3];
    int ps[3];                      // strides in pixels
    const Dav1dGpuAv1Filter *masks;
    const uint8_t *level;
    int b4s, sb128w;
    int w4, h4;                     // luma 4x4 units
    int cw[3], ch[3];               // per plane: 4x4 cells walked
    int cy0[3];                     // per plane: the first cell row walked (row ranges)
    int cells0, cells1;             // cumulative cell counts (plane 0, 0+1)
    int ssx, ssy, bdmax;
    Dav1dGpuFilterLUT lut;
};

// One 4x4 cell's edge of one pass (ROWS = 0: its left edge, 1: its top edge).
template <int BPC, int ROWS>
__global__ __launch_bounds__(256) void k_lpf(LpfArgs<BPC> a) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    int pl, cell;
    if (t < a.cells0) { pl = 0; cell = t; }
    else if (t < a.cells1) { pl = 1; cell = t - a.cells0; }
    else if (t < a.cells1 + (a.cells1 - a.cells0)) { pl = 2; cell = t - a.cells1; }
    else return;
    const int cyr = cell / a.cw[pl], cx = cell - cyr * a.cw[pl], cy = a.cy0[pl] + cyr;
    if (ROWS ? cy == 0 : cx == 0) return;   // picture edges (have_top / have_left)
    const int sx = pl ? a.ssx : 0, sy = pl ? a.ssy : 0;
    const int cpx = 32 >> sx, cpy = 32 >> sy;   // cells per 128x128 area
    const Dav1dGpuAv1Filter &m = a.masks[(cy / cpy) * a.sb128w + cx / cpx];
    const int line = ROWS ? cy % cpy : cx % cpx;
    const int pos = ROWS ? cx % cpx : cy % cpy;
    const int per = ROWS ? 16 >> sx : 16 >> sy;
    const int half = pos / per, bit = pos - half * per;
    int idx;
    if (pl == 0) {
        const uint16_t *f = &m.filter_y[ROWS][line][0][half];
        const int b0 = (f[0] >> bit) & 1, b1 = (f[2] >> bit) & 1, b2 = (f[4] >> bit) & 1;
        if (!(b0 | b1 | b2)) return;
        idx = b2 ? 2 : b1;
    } else {
        const uint16_t *f = &m.filter_uv[ROWS][line][0][half];
        const int b0 = (f[0] >> bit) & 1, b1 = (f[2] >> bit) & 1;
        if (!(b0 | b1)) return;
        idx = b1;
    }
    const int comp = pl ? 1 + pl : ROWS;
    const uint8_t *lv = a.level + ((size_t)cy * a.b4s + cx) * 4 + comp;
    int L = lv[0];
    if (!L) L = ROWS ? lv[-a.b4s * 4] : lv[-4];
    if (!L) return;
    const int wd = pl ? 4 + 2 * idx : 4 << idx;
    using P = typename Px<BPC>::pixel;
    const int ps = a.ps[pl];
    P *d = a.pic[pl] + (size_t)(cy * 4) * ps + cx * 4;
    const int E = a.lut.e[L], I = a.lut.i[L], H = L >> 4;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (ROWS) lpf_line<BPC>(d + j, ps, E, I, H, wd, a.bdmax);
        else lpf_line<BPC>(d + (size_t)j * ps, 1, E, I, H, wd, a.bdmax);
    }
}

template <int BPC>
static int launch_lpf(const Dav1dGpuLoopFilterFrame *f, hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    constexpr int B = BPC / 8;
    if (!f || f->layout < 0 || f->layout > 3 || !f->masks || !f->level || f->b4_stride <= 0) return -1;
    const int np = f->layout && f->filter_uv ? 3 : 1;
    LpfArgs<BPC> a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < np; p++) {
        if (!f->pic[p].data) return -1;
        a.pic[p] = (P *)f->pic[p].data;
        a.ps[p] = (int)(f->pic[p].stride / B);
    }
    const int W = f->pic[0].w, H = f->pic[0].h;
    if (W <= 0 || H <= 0) return -1;
    a.masks = f->masks;
    a.level = f->level;
    a.b4s = (int)f->b4_stride;
    a.w4 = (W + 3) >> 2;
    a.h4 = (H + 3) >> 2;
    const int bw = ((W + 7) >> 3) << 1;
    a.sb128w = (bw + 31) >> 5;
    a.ssx = f->layout != 3;
    a.ssy = f->layout == 1;
    a.bdmax = BPC == 8 ? 255 : f->bitdepth_max;
    a.lut = f->lut;
    // cells walked per pass.  Column edges: columns below w4 (the `w` bound
    // of filter_plane_cols_*, :188, :255), every row of a 64-row half that
    // starts inside the picture (hmask takes a whole half, :191-204).  Row
    // edges: rows below h4 (the y loop, :226, :295), every column of the
    // 128-wide areas (the C loops over all mask bits).
    const int halves = (a.h4 + 15) >> 4;
    // a row range (luma rows, superblock multiples): the cell rows in it
    const int r0 = f->row_start, r1 = f->row_end;
    if (r0 < 0 || r1 < 0 || (r0 & 63) || (r1 & 63) || (r1 && r1 <= r0)) return -1;
    const int y40 = r0 >> 2, y41 = r1 ? r1 >> 2 : 1 << 30;
    int cw[2][3], ch[2][3], c0[3];
    for (int p = 0; p < 3; p++) {
        const int sx = p ? a.ssx : 0, sy = p ? a.ssy : 0;
        c0[p] = y40 >> sy;
        cw[0][p] = (a.w4 + sx) >> sx;
        ch[0][p] = max(0, min(halves * 16, y41) - y40) >> sy;
        cw[1][p] = (a.sb128w * 32) >> sx;
        ch[1][p] = max(0, min((a.h4 + sy) >> sy << sy, y41) - y40 + sy) >> sy;
    }
    for (int pass = 0; pass < 2; pass++) {
        for (int p = 0; p < 3; p++) {
            a.cw[p] = cw[pass][p];
            a.ch[p] = ch[pass][p];
            a.cy0[p] = c0[p];
        }
        a.cells0 = a.cw[0] * a.ch[0];
        a.cells1 = a.cells0 + (np == 3 ? a.cw[1] * a.ch[1] : 0);
        const int total = a.cells1 + (np == 3 ? a.cw[2] * a.ch[2] : 0);
        if (!total) continue;   // (a range past the picture)
        const dim3 grid((unsigned)((total + 255) / 256));
        if (pass == 0) k_lpf<BPC, 0><<<grid, 256, 0, stream>>>(a);
        else k_lpf<BPC, 1><<<grid, 256, 0, stream>>>(a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "dav1d-gpu: loop filter launch failed: %s\n", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

// ---- per-call tier -------------------------------------------------------
struct LpfSeg {
    void *d;          // device pixel q0 of line 0
    int pitch;        // row pitch of its staged rect (pixels)
    int E, I, H, wd;
};
struct LpfSegs {
    LpfSeg s[32];
    int n, vert, bdmax;
};

template <int BPC>
__global__ __launch_bounds__(128) void k_lpf_sb(LpfSegs segs) {
    using P = typename Px<BPC>::pixel;
    const int i = threadIdx.x >> 2, j = threadIdx.x & 3;
    if (i >= segs.n) return;
    const LpfSeg &g = segs.s[i];
    P *d = (P *)g.d;
    if (segs.vert) lpf_line<BPC>(d + j, g.pitch, g.E, g.I, g.H, g.wd, segs.bdmax);
    else lpf_line<BPC>(d + (size_t)j * g.pitch, 1, g.E, g.I, g.H, g.wd, segs.bdmax);
}

// loop_filter_{h,v}_sb128{y,uv}_c (src/loopfilter_tmpl.c:163-245)
template <int BPC, int VERT, int UV>
static bool lpf_sb_t(typename Px<BPC>::pixel *dst, ptrdiff_t stride, const uint32_t *vmask, const uint8_t (*l)[4],
                     ptrdiff_t b4_stride, const Dav1dGpuFilterLUT *lut, int bdmax) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    const unsigned vm = vmask[0] | vmask[1] | (UV ? 0 : vmask[2]);
    struct Pending { int rect, k, E, I, H, wd; } pend[32];
    int n = 0;
    Stager st;
    for (int k = 0; k < 32; k++) {
        const unsigned b = 1u << k;
        if (!(vm & ~(b - 1))) break;
        if (!(vm & b)) continue;
        const uint8_t(*lk)[4] = l + (VERT ? k : (ptrdiff_t)k * b4_stride);
        const int L = lk[0][0] ? lk[0][0] : lk[VERT ? -b4_stride : -1][0];
        if (!L) continue;
        const int idx = UV ? !!(vmask[1] & b) : (vmask[2] & b) ? 2 : !!(vmask[1] & b);
        const int wd = UV ? 4 + 2 * idx : 4 << idx;
        const int r = wd == 16 ? 7 : wd / 2;   // pixels read on each side
        // the segment's 4 lines along the edge, r pixels on each side
        const int rect = VERT ? st.inout(dst, stride, (4L * k) * B, (4L * k + 4) * B, -r, r)
                              : st.inout(dst, stride, -r * B, r * B, 4L * k, 4L * k + 4);
        pend[n++] = { rect, k, lut->e[L], lut->i[L], L >> 4, wd };
    }
    if (!n) return true;
    if (!st.upload()) return false;
    LpfSegs s;
    memset(&s, 0, sizeof(s));
    for (int i = 0; i < n; i++) {
        const Pending &p = pend[i];
        P *o = st.origin<P>(p.rect);   // dst's (0, 0) in the rect's device copy
        const int pitch = (int)(st.pitch(p.rect) / B);
        s.s[i] = { VERT ? (void *)(o + 4 * p.k) : (void *)(o + (ptrdiff_t)(4 * p.k) * pitch), pitch, p.E, p.I, p.H,
                   p.wd };
    }
    s.n = n;
    s.vert = VERT;
    s.bdmax = bdmax;
    k_lpf_sb<BPC><<<1, 128, 0, st.stream()>>>(s);
    return st.finish();
}

// The caller's entries before dav1d_loop_filter_dsp_init_gpu_* overwrote
// them (run when the GPU path fails: runtime.hpp's error contract).
static Dav1dLoopFilterDSPContext_8bpc g_fb8;
static Dav1dLoopFilterDSPContext_16bpc g_fb16;

#define LPF_ENTRIES(BPC, P, BDP, BDV)                                                                     \
template <int VERT, int UV>                                                                               \
static void lpf_##BPC(P *d, ptrdiff_t s, const uint32_t *m, const uint8_t (*l)[4], ptrdiff_t b4s,          \
                      const Dav1dGpuFilterLUT *lut, int w BDP)                                            \
{ DGPU_OR_FALLBACK((lpf_sb_t<BPC, VERT, UV>(d, s, m, l, b4s, lut, BDV)),                                 \
                   g_fb##BPC.loop_filter_sb[UV][VERT], d, s, m, l, b4s, lut, w BDV##_ARG); }

#define BD8_PARAM
#define BD8_VAL 255
#define BD8_VAL_ARG
#define BD16_PARAM , int bitdepth_max
#define BD16_VAL bitdepth_max
#define BD16_VAL_ARG , bitdepth_max
LPF_ENTRIES(8, uint8_t, BD8_PARAM, BD8_VAL)
LPF_ENTRIES(16, uint16_t, BD16_PARAM, BD16_VAL)

#define FILL_LPF(BPC, c)                                 \
    do {                                                 \
        c->loop_filter_sb[0][0] = lpf_##BPC<0, 0>;       \
        c->loop_filter_sb[0][1] = lpf_##BPC<1, 0>;       \
        c->loop_filter_sb[1][0] = lpf_##BPC<0, 1>;       \
        c->loop_filter_sb[1][1] = lpf_##BPC<1, 1>;       \
    } while (0)

}  // namespace dgpu

using namespace dgpu;

// bitfn(dav1d_loop_filter_dsp_init) replacement, src/loopfilter_tmpl.c:257-272
// The _gpu_ hooks keep the caller's previous entries as fallbacks.
extern "C" void dav1d_loop_filter_dsp_init_gpu_8bpc(Dav1dLoopFilterDSPContext_8bpc *c) {
    Dav1dLoopFilterDSPContext_8bpc g{}, *gp = &g;
    FILL_LPF(8, gp);
    save_fallback(&g_fb8, c, gp);
    FILL_LPF(8, c);
}
extern "C" void dav1d_loop_filter_dsp_init_gpu_16bpc(Dav1dLoopFilterDSPContext_16bpc *c) {
    Dav1dLoopFilterDSPContext_16bpc g{}, *gp = &g;
    FILL_LPF(16, gp);
    save_fallback(&g_fb16, c, gp);
    FILL_LPF(16, c);
}
extern "C" void dav1d_loop_filter_dsp_init_8bpc(Dav1dLoopFilterDSPContext_8bpc *c) { FILL_LPF(8, c); }
extern "C" void dav1d_loop_filter_dsp_init_16bpc(Dav1dLoopFilterDSPContext_16bpc *c) { FILL_LPF(16, c); }

extern "C" int dav1d_gpu_loopfilter_frame_8bpc(const Dav1dGpuLoopFilterFrame *f, void *stream) {
    return launch_lpf<8>(f, (hipStream_t)stream);
}
extern "C" int dav1d_gpu_loopfilter_frame_16bpc(const Dav1dGpuLoopFilterFrame *f, void *stream) {
    return launch_lpf<16>(f, (hipStream_t)stream);
}
