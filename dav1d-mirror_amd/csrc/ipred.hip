// ipred.hip -- Dav1dIntraPredDSPContext (src/ipred.h:81-90) on gfx950.
//
// Per-call kernels: one workgroup per call.  The edge array topleft[-2h..2w]
// is staged in LDS; the directional modes build their filtered / upsampled
// edge in LDS in parallel, then every lane predicts pixels independently.
// Filter-intra's 4x2 cells run as an anti-diagonal wavefront (a cell needs
// its left, top and top-left cells, src/ipred_tmpl.c:617-655).
#include "dav1d_gpu.h"
#include "dsp_common.hpp"
#include "runtime.hpp"

namespace dgpu {

constexpr int EOFF = 128;  // LDS index of topleft[0]

// get_filter_strength, src/ipred_tmpl.c:327-360
__device__ int edge_strength(int wh, int angle, int is_sm) {
    if (is_sm) {
        if (wh <= 8) return angle >= 64 ? 2 : angle >= 40 ? 1 : 0;
        if (wh <= 16) return angle >= 48 ? 2 : angle >= 20 ? 1 : 0;
        if (wh <= 24) return angle >= 4 ? 3 : 0;
        return 3;
    }
    if (wh <= 8) return angle >= 56 ? 1 : 0;
    if (wh <= 16) return angle >= 40 ? 1 : 0;
    if (wh <= 24) return angle >= 32 ? 3 : angle >= 16 ? 2 : angle >= 8 ? 1 : 0;
    if (wh <= 32) return angle >= 32 ? 3 : angle >= 4 ? 2 : 1;
    return 3;
}
__device__ __forceinline__ int use_upsample(int wh, int angle, int is_sm) {
    return angle < 40 && wh <= (16 >> is_sm);
}

// One output element of filter_edge (src/ipred_tmpl.c:362-385); `in` is an
// LDS array indexed relative to its element 0.
__device__ __forceinline__ int smooth_edge_px(const int *in, int i, int lim_from, int lim_to,
                                              int from, int to, int strength) {
    if (i < lim_from || i >= lim_to) return in[clampi(i, from, to - 1)];
    const int k0 = strength == 3 ? 2 : 0;
    const int k1 = strength == 1 ? 4 : strength == 2 ? 5 : 4;
    const int k2 = strength == 1 ? 8 : strength == 2 ? 6 : 4;
    const int s = k0 * in[clampi(i - 2, from, to - 1)] + k1 * in[clampi(i - 1, from, to - 1)] +
                  k2 * in[clampi(i, from, to - 1)] + k1 * in[clampi(i + 1, from, to - 1)] +
                  k0 * in[clampi(i + 2, from, to - 1)];
    return (s + 8) >> 4;
}

// One output element of upsample_edge (src/ipred_tmpl.c:391-406)
__device__ __forceinline__ int upsample_px(const int *in, int o, int hsz, int from, int to, int bdmax) {
    const int i = o >> 1;
    if (!(o & 1) || i >= hsz - 1) return in[clampi(i, from, to - 1)];
    const int s = -in[clampi(i - 1, from, to - 1)] + 9 * in[clampi(i, from, to - 1)] +
                  9 * in[clampi(i + 1, from, to - 1)] - in[clampi(i + 2, from, to - 1)];
    return clampi((s + 8) >> 4, 0, bdmax);
}

template <int BPC> struct IpredArgs {
    typename Px<BPC>::pixel *dst;
    ptrdiff_t ds;
    const typename Px<BPC>::pixel *tl;  // topleft[0]
    int w, h, mode, angle, max_w, max_h, bdmax;
    // cfl
    const int16_t *ac;
    int alpha, cfl;  // cfl: 1 -> cfl_pred with mode's DC flavour
};

__device__ __forceinline__ int dc_mul(int w, int h, unsigned s, bool hbd) {
    if (w == h) return (int)s;
    const int r4 = w > 2 * h || h > 2 * w;
    if (!hbd) return (int)((s * (r4 ? 0x3334u : 0x5556u)) >> 16);
    return (int)((s * (r4 ? 0x6667u : 0xAAABu)) >> 17);
}

template <int BPC>
__global__ __launch_bounds__(256) void k_ipred(IpredArgs<BPC> a) {
    __shared__ int e[EOFF * 2 + 1];      // topleft[-128..128]
    __shared__ int f[EOFF * 2 + 1];      // filtered / upsampled edge
    __shared__ int cell[64 * 64];        // filter-intra reconstruction
    __shared__ int dcv;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int w = a.w, h = a.h;
    for (int i = -2 * h + tid; i <= 2 * w; i += nt) e[EOFF + i] = a.tl[i];
    __syncthreads();
    const int *tl = &e[EOFF];
    const int mode = a.mode;
    const bool hbd = BPC == 16;

    if (mode == DGPU_DC_PRED || mode == DGPU_TOP_DC_PRED || mode == DGPU_LEFT_DC_PRED ||
        mode == DGPU_DC_128_PRED) {
        // dc_gen / dc_gen_top / dc_gen_left, src/ipred_tmpl.c:86-166
        if (tid == 0) {
            unsigned s;
            if (mode == DGPU_DC_128_PRED) {
                s = (a.bdmax + 1) >> 1;
            } else if (mode == DGPU_TOP_DC_PRED) {
                s = w >> 1;
                for (int i = 1; i <= w; i++) s += tl[i];
                s >>= __builtin_ctz(w);
            } else if (mode == DGPU_LEFT_DC_PRED) {
                s = h >> 1;
                for (int i = 1; i <= h; i++) s += tl[-i];
                s >>= __builtin_ctz(h);
            } else {
                s = (w + h) >> 1;
                for (int i = 1; i <= w; i++) s += tl[i];
                for (int i = 1; i <= h; i++) s += tl[-i];
                s >>= __builtin_ctz(w + h);
                s = dc_mul(w, h, s, hbd);
            }
            dcv = (int)s;
        }
        __syncthreads();
        const int dc = dcv;
        for (int i = tid; i < w * h; i += nt) {
            const int x = i % w, y = i / w;
            int v = dc;
            if (a.cfl) {  // cfl_pred, src/ipred_tmpl.c:71-84
                const int d = a.alpha * a.ac[i];
                const int mag = (abs(d) + 32) >> 6;
                v = clampi(dc + (d < 0 ? -mag : mag), 0, a.bdmax);
            }
            a.dst[y * a.ds + x] = (typename Px<BPC>::pixel)v;
        }
        return;
    }

    if (mode == DGPU_FILTER_PRED) {
        const int fidx = a.angle & 511;
        const signed char *taps = &dspt_filter_intra[fidx * 56];
        const int cw = w >> 2, ch = h >> 1;
        for (int step = 0; step < cw + ch - 1; step++) {
            for (int c = tid; c < cw * ch; c += nt) {
                const int cx = c % cw, cy = c / cw;
                if (cx + cy != step) continue;
                const int x = cx * 4, y = cy * 2;
                int p[7];
                if (y == 0) {
                    p[0] = x == 0 ? tl[0] : tl[x];
                    for (int i = 0; i < 4; i++) p[1 + i] = tl[1 + x + i];
                } else {
                    p[0] = x == 0 ? tl[-y] : cell[(y - 1) * 64 + x - 1];
                    for (int i = 0; i < 4; i++) p[1 + i] = cell[(y - 1) * 64 + x + i];
                }
                for (int i = 0; i < 2; i++) p[5 + i] = x == 0 ? tl[-(y + 1 + i)] : cell[(y + i) * 64 + x - 1];
                for (int k = 0; k < 8; k++) {
                    int acc = 0;
                    for (int i = 0; i < 7; i++) acc += taps[k * 7 + i] * p[i];
                    cell[(y + (k >> 2)) * 64 + x + (k & 3)] = clampi((acc + 8) >> 4, 0, a.bdmax);
                }
            }
            __syncthreads();
        }
        for (int i = tid; i < w * h; i += nt) {
            const int x = i % w, y = i / w;
            a.dst[y * a.ds + x] = (typename Px<BPC>::pixel)cell[y * 64 + x];
        }
        return;
    }

    const int is_sm = (a.angle >> 9) & 1, filt = a.angle >> 10, ang = a.angle & 511;

    if (mode == DGPU_Z1_PRED) {  // src/ipred_tmpl.c:408-460
        int dx = dspt_dr_deriv[ang >> 1];
        const int up = filt ? use_upsample(w + h, 90 - ang, is_sm) : 0;
        const int st = (!up && filt) ? edge_strength(w + h, 90 - ang, is_sm) : 0;
        const int *top;
        int maxb;
        if (up) {
            for (int o = tid; o < 2 * (w + h) - 1; o += nt)
                f[o] = upsample_px(&tl[1], o, w + h, -1, w + min(w, h), a.bdmax);
            top = f; maxb = 2 * (w + h) - 2; dx <<= 1;
        } else if (st) {
            for (int i = tid; i < w + h; i += nt)
                f[i] = smooth_edge_px(&tl[1], i, 0, w + h, -1, w + min(w, h), st);
            top = f; maxb = w + h - 1;
        } else {
            top = &tl[1]; maxb = w + min(w, h) - 1;
        }
        __syncthreads();
        for (int i = tid; i < w * h; i += nt) {
            const int x = i % w, y = i / w;
            const int xpos = (y + 1) * dx, frac = xpos & 0x3e;
            const int base = (xpos >> 6) + x * (1 + up);
            const int v = base < maxb ? (top[base] * (64 - frac) + top[base + 1] * frac + 32) >> 6 : top[maxb];
            a.dst[y * a.ds + x] = (typename Px<BPC>::pixel)v;
        }
        return;
    }

    if (mode == DGPU_Z3_PRED) {  // src/ipred_tmpl.c:542-599
        int dy = dspt_dr_deriv[(270 - ang) >> 1];
        const int up = filt ? use_upsample(w + h, ang - 180, is_sm) : 0;
        const int st = (!up && filt) ? edge_strength(w + h, ang - 180, is_sm) : 0;
        const int *left;
        int maxb;
        if (up) {
            for (int o = tid; o < 2 * (w + h) - 1; o += nt)
                f[o] = upsample_px(&tl[-(w + h)], o, w + h, max(w - h, 0), w + h + 1, a.bdmax);
            left = &f[2 * (w + h) - 2]; maxb = 2 * (w + h) - 2; dy <<= 1;
        } else if (st) {
            for (int i = tid; i < w + h; i += nt)
                f[i] = smooth_edge_px(&tl[-(w + h)], i, 0, w + h, max(w - h, 0), w + h + 1, st);
            left = &f[w + h - 1]; maxb = w + h - 1;
        } else {
            left = &tl[-1]; maxb = h + min(w, h) - 1;
        }
        __syncthreads();
        for (int i = tid; i < w * h; i += nt) {
            const int x = i % w, y = i / w;
            const int ypos = (x + 1) * dy, frac = ypos & 0x3e;
            const int base = (ypos >> 6) + y * (1 + up);
            const int v = base < maxb ? (left[-base] * (64 - frac) + left[-(base + 1)] * frac + 32) >> 6
                                      : left[-maxb];
            a.dst[y * a.ds + x] = (typename Px<BPC>::pixel)v;
        }
        return;
    }

    if (mode == DGPU_Z2_PRED) {  // src/ipred_tmpl.c:462-540
        int dy = dspt_dr_deriv[(ang - 90) >> 1];
        int dx = dspt_dr_deriv[(180 - ang) >> 1];
        const int upl = filt ? use_upsample(w + h, 180 - ang, is_sm) : 0;
        const int upa = filt ? use_upsample(w + h, ang - 90, is_sm) : 0;
        int *c = &f[EOFF];  // edge[64+64+1] with topleft at index 0
        if (upa) {
            for (int o = tid; o < 2 * w + 1; o += nt) c[o] = upsample_px(&tl[0], o, w + 1, 0, w + 1, a.bdmax);
        } else {
            const int st = filt ? edge_strength(w + h, ang - 90, is_sm) : 0;
            for (int i = tid; i < w; i += nt)
                c[1 + i] = st ? smooth_edge_px(&tl[1], i, 0, a.max_w, -1, w, st) : tl[1 + i];
        }
        if (upl) {
            for (int o = tid; o < 2 * h + 1; o += nt)
                c[-2 * h + o] = upsample_px(&tl[-h], o, h + 1, 0, h + 1, a.bdmax);
        } else {
            const int st = filt ? edge_strength(w + h, 180 - ang, is_sm) : 0;
            for (int i = tid; i < h; i += nt)
                c[-h + i] = st ? smooth_edge_px(&tl[-h], i, h - a.max_h, h, 0, h + 1, st) : tl[-h + i];
        }
        __syncthreads();
        if (tid == 0) c[0] = tl[0];
        if (upa) dx <<= 1;
        if (upl) dy <<= 1;
        __syncthreads();
        const int *left = &c[-(1 + upl)];
        for (int i = tid; i < w * h; i += nt) {
            const int x = i % w, y = i / w;
            const int xpos = ((1 + upa) << 6) - (y + 1) * dx;
            const int bx = (xpos >> 6) + x * (1 + upa);
            int v;
            if (bx >= 0) {
                const int fx = xpos & 0x3e;
                v = c[bx] * (64 - fx) + c[bx + 1] * fx;
            } else {
                const int ypos = (y << (6 + upl)) - (x + 1) * dy;
                const int by = ypos >> 6, fy = ypos & 0x3e;
                v = left[-by] * (64 - fy) + left[-(by + 1)] * fy;
            }
            a.dst[y * a.ds + x] = (typename Px<BPC>::pixel)((v + 32) >> 6);
        }
        return;
    }

    // V, H, Paeth, Smooth*: independent per pixel (src/ipred_tmpl.c:220-325)
    for (int i = tid; i < w * h; i += nt) {
        const int x = i % w, y = i / w;
        const int top = tl[1 + x], left = tl[-(1 + y)];
        int v;
        switch (mode) {
        case DGPU_VERT_PRED: v = top; break;
        case DGPU_HOR_PRED: v = left; break;
        case DGPU_PAETH_PRED: {
            const int c = tl[0], base = left + top - c;
            const int dl = abs(left - base), dt = abs(top - base), dc = abs(c - base);
            v = (dl <= dt && dl <= dc) ? left : dt <= dc ? top : c;
            break;
        }
        case DGPU_SMOOTH_PRED: {
            const int wv = dspt_sm_weights[h + y], wh = dspt_sm_weights[w + x];
            v = (wv * top + (256 - wv) * tl[-h] + wh * left + (256 - wh) * tl[w] + 256) >> 9;
            break;
        }
        case DGPU_SMOOTH_V_PRED: {
            const int wv = dspt_sm_weights[h + y];
            v = (wv * top + (256 - wv) * tl[-h] + 128) >> 8;
            break;
        }
        default: {  // SMOOTH_H
            const int wh = dspt_sm_weights[w + x];
            v = (wh * left + (256 - wh) * tl[w] + 128) >> 8;
            break;
        }
        }
        a.dst[y * a.ds + x] = (typename Px<BPC>::pixel)v;
    }
}

// cfl_ac_c, src/ipred_tmpl.c:657-703
template <int BPC> struct CflAcArgs {
    int16_t *ac;
    const typename Px<BPC>::pixel *y;
    ptrdiff_t ys;
    int w_pad, h_pad, cw, ch, ssh, ssv;
};

template <int BPC>
__global__ __launch_bounds__(256) void k_cfl_ac(CflAcArgs<BPC> a) {
    __shared__ int v[32 * 32];
    __shared__ int sumv;
    const int tid = threadIdx.x, n = a.cw * a.ch;
    const int vw = a.cw - 4 * a.w_pad, vh = a.ch - 4 * a.h_pad;
    for (int i = tid; i < n; i += blockDim.x) {
        const int x = i % a.cw, y = i / a.cw;
        const int sx = min(x, vw - 1), sy = min(y, vh - 1);
        const auto *p = a.y + (sy << a.ssv) * a.ys + (sx << a.ssh);
        int s = p[0];
        if (a.ssh) s += p[1];
        if (a.ssv) {
            s += p[a.ys];
            if (a.ssh) s += p[a.ys + 1];
        }
        v[i] = s << (1 + !a.ssv + !a.ssh);
    }
    __syncthreads();
    if (tid == 0) {
        const int lg = __builtin_ctz(a.cw) + __builtin_ctz(a.ch);
        int s = (1 << lg) >> 1;
        for (int i = 0; i < n; i++) s += v[i];
        sumv = s >> lg;
    }
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) a.ac[i] = (int16_t)(v[i] - sumv);
}

// pal_pred_c, src/ipred_tmpl.c:717-730
template <int BPC>
__global__ __launch_bounds__(256) void k_pal(typename Px<BPC>::pixel *dst, ptrdiff_t ds,
                                             const typename Px<BPC>::pixel *pal, const uint8_t *idx,
                                             int w, int h) {
    for (int i = threadIdx.x; i < w * h; i += blockDim.x) {
        const int x = i % w, y = i / w;
        const int b = idx[(y * w + x) >> 1];
        dst[y * ds + x] = pal[(x & 1) ? (b >> 4) : (b & 7)];
    }
}

// ---------------------------------------------------------------------------
template <int BPC>
static bool run_ipred(typename Px<BPC>::pixel *dst, ptrdiff_t stride,
                      const typename Px<BPC>::pixel *tl, int w, int h, int mode, int angle,
                      int max_w, int max_h, const int16_t *ac, int alpha, int cfl, int bdmax) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    Stager st;
    const int ie = st.in1(tl - 2 * h, (long)(2 * h + 2 * w + 1) * B);
    const int ia = cfl ? st.in1(ac, (long)w * h * 2) : -1;
    const int od = st.out(dst, stride, 0, w * B, 0, h);
    if (!st.upload()) return false;
    IpredArgs<BPC> a;
    a.dst = st.origin<P>(od);
    a.ds = st.pitch(od) / B;
    a.tl = st.origin<const P>(ie) + 2 * h;
    a.w = w; a.h = h; a.mode = mode; a.angle = angle; a.max_w = max_w; a.max_h = max_h;
    a.bdmax = bdmax;
    a.ac = cfl ? st.origin<const int16_t>(ia) : nullptr;
    a.alpha = alpha;
    a.cfl = cfl;
    k_ipred<BPC><<<1, 256, 0, st.stream()>>>(a);
    return st.finish();
}

template <int BPC, int SSH, int SSV>
static bool cfl_ac_run(int16_t *ac, const typename Px<BPC>::pixel *y, ptrdiff_t stride, int w_pad,
                     int h_pad, int cw, int ch) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    const long vw = (cw - 4 * w_pad) << SSH, vh = (ch - 4 * h_pad) << SSV;
    Stager st;
    const int iy = st.in(y, stride, 0, vw * B, 0, vh);
    const int oa = st.out1(ac, (long)cw * ch * 2);
    if (!st.upload()) return false;
    CflAcArgs<BPC> a;
    a.ac = st.origin<int16_t>(oa);
    a.y = st.origin<const P>(iy);
    a.ys = st.pitch(iy) / B;
    a.w_pad = w_pad; a.h_pad = h_pad; a.cw = cw; a.ch = ch; a.ssh = SSH; a.ssv = SSV;
    k_cfl_ac<BPC><<<1, 256, 0, st.stream()>>>(a);
    return st.finish();
}

template <int BPC>
static bool pal_pred_run(typename Px<BPC>::pixel *dst, ptrdiff_t stride,
                       const typename Px<BPC>::pixel *pal, const uint8_t *idx, int w, int h) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    Stager st;
    const int ip = st.in1(pal, 8 * B);
    const int ii = st.in1(idx, (long)w * h / 2);
    const int od = st.out(dst, stride, 0, w * B, 0, h);
    if (!st.upload()) return false;
    k_pal<BPC><<<1, 256, 0, st.stream()>>>(st.origin<P>(od), st.pitch(od) / B,
                                           st.origin<const P>(ip), st.origin<const uint8_t>(ii), w, h);
    return st.finish();
}

// The caller's entries before dav1d_intra_pred_dsp_init_gpu_* overwrote
// them (run when the GPU path fails: runtime.hpp's error contract).
static Dav1dIntraPredDSPContext_8bpc g_fb8;
static Dav1dIntraPredDSPContext_16bpc g_fb16;

#define IPRED_ENTRIES(BPC, P, BDP, BDV)                                                        \
template <int MODE>                                                                            \
static void ipred_##BPC(P *d, ptrdiff_t s, const P *tl, int w, int h, int a, int mw, int mh BDP)\
{ DGPU_OR_FALLBACK((run_ipred<BPC>(d, s, tl, w, h, MODE, a, mw, mh, nullptr, 0, 0, BDV)),      \
                   g_fb##BPC.intra_pred[MODE], d, s, tl, w, h, a, mw, mh BDV##_ARG); }         \
template <int MODE>                                                                            \
static void cfl_##BPC(P *d, ptrdiff_t s, const P *tl, int w, int h, const int16_t *ac,         \
                      int alpha BDP)                                                           \
{ DGPU_OR_FALLBACK((run_ipred<BPC>(d, s, tl, w, h, MODE, 0, 0, 0, ac, alpha, 1, BDV)),         \
                   g_fb##BPC.cfl_pred[MODE], d, s, tl, w, h, ac, alpha BDV##_ARG); }           \
template <int SSH, int SSV>                                                                    \
static void cfl_ac_##BPC(int16_t *ac, const P *y, ptrdiff_t s, int wp, int hp, int cw, int ch) \
{ DGPU_OR_FALLBACK((cfl_ac_run<BPC, SSH, SSV>(ac, y, s, wp, hp, cw, ch)),                      \
                   g_fb##BPC.cfl_ac[SSH + SSV == 2 ? 0 : SSH ? 1 : 2], ac, y, s, wp, hp, cw, ch); } \
static void pal_pred_##BPC(P *d, ptrdiff_t s, const P *pal, const uint8_t *idx, int w, int h)  \
{ DGPU_OR_FALLBACK((pal_pred_run<BPC>(d, s, pal, idx, w, h)), g_fb##BPC.pal_pred, d, s, pal, idx, w, h); }

#define BD8_PARAM
#define BD8_VAL 255
#define BD8_VAL_ARG
#define BD16_PARAM , int bitdepth_max
#define BD16_VAL bitdepth_max
#define BD16_VAL_ARG , bitdepth_max
IPRED_ENTRIES(8, uint8_t, BD8_PARAM, BD8_VAL)
IPRED_ENTRIES(16, uint16_t, BD16_PARAM, BD16_VAL)

#define FILL_IPRED(BPC, c)                                                                     \
    do {                                                                                       \
        c->intra_pred[DGPU_DC_PRED] = ipred_##BPC<DGPU_DC_PRED>;                               \
        c->intra_pred[DGPU_VERT_PRED] = ipred_##BPC<DGPU_VERT_PRED>;                           \
        c->intra_pred[DGPU_HOR_PRED] = ipred_##BPC<DGPU_HOR_PRED>;                             \
        c->intra_pred[DGPU_LEFT_DC_PRED] = ipred_##BPC<DGPU_LEFT_DC_PRED>;                     \
        c->intra_pred[DGPU_TOP_DC_PRED] = ipred_##BPC<DGPU_TOP_DC_PRED>;                       \
        c->intra_pred[DGPU_DC_128_PRED] = ipred_##BPC<DGPU_DC_128_PRED>;                       \
        c->intra_pred[DGPU_Z1_PRED] = ipred_##BPC<DGPU_Z1_PRED>;                               \
        c->intra_pred[DGPU_Z2_PRED] = ipred_##BPC<DGPU_Z2_PRED>;                               \
        c->intra_pred[DGPU_Z3_PRED] = ipred_##BPC<DGPU_Z3_PRED>;                               \
        c->intra_pred[DGPU_SMOOTH_PRED] = ipred_##BPC<DGPU_SMOOTH_PRED>;                       \
        c->intra_pred[DGPU_SMOOTH_V_PRED] = ipred_##BPC<DGPU_SMOOTH_V_PRED>;                   \
        c->intra_pred[DGPU_SMOOTH_H_PRED] = ipred_##BPC<DGPU_SMOOTH_H_PRED>;                   \
        c->intra_pred[DGPU_PAETH_PRED] = ipred_##BPC<DGPU_PAETH_PRED>;                         \
        c->intra_pred[DGPU_FILTER_PRED] = ipred_##BPC<DGPU_FILTER_PRED>;                       \
        c->cfl_ac[0] = cfl_ac_##BPC<1, 1>;                                                     \
        c->cfl_ac[1] = cfl_ac_##BPC<1, 0>;                                                     \
        c->cfl_ac[2] = cfl_ac_##BPC<0, 0>;                                                     \
        c->cfl_pred[DGPU_DC_PRED] = cfl_##BPC<DGPU_DC_PRED>;                                   \
        c->cfl_pred[DGPU_DC_128_PRED] = cfl_##BPC<DGPU_DC_128_PRED>;                           \
        c->cfl_pred[DGPU_TOP_DC_PRED] = cfl_##BPC<DGPU_TOP_DC_PRED>;                           \
        c->cfl_pred[DGPU_LEFT_DC_PRED] = cfl_##BPC<DGPU_LEFT_DC_PRED>;                         \
        c->pal_pred = pal_pred_##BPC;                                                          \
    } while (0)

}  // namespace dgpu

using namespace dgpu;

// bitfn(dav1d_intra_pred_dsp_init) replacement, src/ipred_tmpl.c:740-774
// The _gpu_ hooks keep the caller's previous entries as fallbacks.
extern "C" void dav1d_intra_pred_dsp_init_gpu_8bpc(Dav1dIntraPredDSPContext_8bpc *c) {
    Dav1dIntraPredDSPContext_8bpc g{}, *gp = &g;
    FILL_IPRED(8, gp);
    save_fallback(&g_fb8, c, gp);
    FILL_IPRED(8, c);
}
extern "C" void dav1d_intra_pred_dsp_init_gpu_16bpc(Dav1dIntraPredDSPContext_16bpc *c) {
    Dav1dIntraPredDSPContext_16bpc g{}, *gp = &g;
    FILL_IPRED(16, gp);
    save_fallback(&g_fb16, c, gp);
    FILL_IPRED(16, c);
}
extern "C" void dav1d_intra_pred_dsp_init_8bpc(Dav1dIntraPredDSPContext_8bpc *c) { FILL_IPRED(8, c); }
extern "C" void dav1d_intra_pred_dsp_init_16bpc(Dav1dIntraPredDSPContext_16bpc *c) { FILL_IPRED(16, c); }
