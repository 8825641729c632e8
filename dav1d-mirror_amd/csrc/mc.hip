// mc.hip -- Dav1dMCDSPContext (src/mc.h:116-132) on gfx950.
//
// Per-call kernels: one thread per output pixel, each evaluating the
// reference formula for that pixel directly (the 8 intermediate rows of an
// hv filter are recomputed per pixel; the per-call tier is latency-bound by
// its PCIe round trip, the batch tier in recon.hip is the throughput path).
// Semantics: src/mc_tmpl.c (line citations on each device function).
#include "dav1d_gpu.h"
#include "dsp_common.hpp"
#include "runtime.hpp"

namespace dgpu {

// filter_type = type_h | type_v << 2 per Filter2d (src/mc_tmpl.c:376-384)
static constexpr int kFtype[9] = { 0, 4, 8, 2, 6, 10, 1, 5, 9 };

template <int BPC> struct McArgs {
    using P = typename Px<BPC>::pixel;
    P *dst;
    ptrdiff_t ds;
    int16_t *tmp;
    const P *src;
    ptrdiff_t ss;
    int w, h, mx, my, dx, dy;
    int ftype;   // 0..10, or -1 for bilinear
    int scaled;
    int bdmax;
};

template <int BPC, typename T>
__device__ __forceinline__ int tap8(const T *p, ptrdiff_t step, const signed char *k) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += k[i] * (int)p[(i - 3) * step];
    return s;
}

// put_8tap_c / prep_8tap_c, src/mc_tmpl.c:113-171, :223-282
template <int BPC>
__device__ int mc_8tap_px(const McArgs<BPC> &a, int x, int y, bool put) {
    const int ib = Px<BPC>::ibits(a.bdmax);
    const int PB = Px<BPC>::PBIAS;
    const signed char *fh = subpel_kernel(a.ftype & 3, a.mx, a.w);
    const signed char *fv = subpel_kernel(a.ftype >> 2, a.my, a.h);
    const auto *s = a.src + y * a.ss + x;
    if (fh && fv) {
        int acc = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int mid = (int16_t)rnd_sh(tap8<BPC>(s + (k - 3) * a.ss, 1, fh), 6 - ib);
            acc += fv[k] * mid;
        }
        return put ? clampi(rnd_sh(acc, 6 + ib), 0, a.bdmax) : rnd_sh(acc, 6) - PB;
    }
    if (fh) {
        const int acc = tap8<BPC>(s, 1, fh);
        return put ? clampi((acc + 32 + ((1 << (6 - ib)) >> 1)) >> 6, 0, a.bdmax)
                   : rnd_sh(acc, 6 - ib) - PB;
    }
    if (fv) {
        const int acc = tap8<BPC>(s, a.ss, fv);
        return put ? clampi(rnd_sh(acc, 6), 0, a.bdmax) : rnd_sh(acc, 6 - ib) - PB;
    }
    return put ? (int)s[0] : ((int)s[0] << ib) - PB;
}

__device__ __forceinline__ int blin(int a, int b, int m) { return 16 * a + m * (b - a); }

// put_bilin_c / prep_bilin_c, src/mc_tmpl.c:395-450, :493-546
template <int BPC>
__device__ int mc_bilin_px(const McArgs<BPC> &a, int x, int y, bool put) {
    const int ib = Px<BPC>::ibits(a.bdmax);
    const int PB = Px<BPC>::PBIAS;
    const auto *s = a.src + y * a.ss + x;
    const ptrdiff_t ss = a.ss;
    if (a.mx && a.my) {
        const int m0 = (int16_t)rnd_sh(blin(s[0], s[1], a.mx), 4 - ib);
        const int m1 = (int16_t)rnd_sh(blin(s[ss], s[ss + 1], a.mx), 4 - ib);
        return put ? clampi(rnd_sh(blin(m0, m1, a.my), 4 + ib), 0, a.bdmax)
                   : rnd_sh(blin(m0, m1, a.my), 4) - PB;
    }
    if (a.mx) {
        const int px = rnd_sh(blin(s[0], s[1], a.mx), 4 - ib);
        return put ? clampi(rnd_sh(px, ib), 0, a.bdmax) : px - PB;
    }
    if (a.my)
        return put ? clampi(rnd_sh(blin(s[0], s[ss], a.my), 4), 0, a.bdmax)
                   : rnd_sh(blin(s[0], s[ss], a.my), 4 - ib) - PB;
    return put ? (int)s[0] : ((int)s[0] << ib) - PB;
}

// put/prep_8tap_scaled_c, src/mc_tmpl.c:173-221, :284-328.  Column x samples
// source column (mx + x*dx) >> 10, sub-pel ((mx + x*dx) & 1023) >> 6; the
// intermediate row for output row y is (my + y*dy) >> 10 (+3 for the taps).
template <int BPC>
__device__ int mc_8tap_scaled_px(const McArgs<BPC> &a, int x, int y, bool put) {
    const int ib = Px<BPC>::ibits(a.bdmax);
    const int PB = Px<BPC>::PBIAS;
    const int px = a.mx + x * a.dx, py = a.my + y * a.dy;
    const int col = px >> 10, row = py >> 10;
    const signed char *fh = subpel_kernel(a.ftype & 3, (px & 1023) >> 6, a.w);
    const signed char *fv = subpel_kernel(a.ftype >> 2, (py & 1023) >> 6, a.h);
    auto mid = [&](int r) -> int {  // intermediate row r, source row r - 3
        const auto *s = a.src + (r - 3) * a.ss + col;
        return fh ? (int16_t)rnd_sh(tap8<BPC>(s, 1, fh), 6 - ib) : (int16_t)((int)s[0] << ib);
    };
    if (fv) {
        int acc = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) acc += fv[k] * mid(row + k);
        return put ? clampi(rnd_sh(acc, 6 + ib), 0, a.bdmax) : rnd_sh(acc, 6) - PB;
    }
    const int m = mid(row + 3);
    return put ? clampi(rnd_sh(m, ib), 0, a.bdmax) : m - PB;
}

// put/prep_bilin_scaled_c, src/mc_tmpl.c:452-491, :548-585
template <int BPC>
__device__ int mc_bilin_scaled_px(const McArgs<BPC> &a, int x, int y, bool put) {
    const int ib = Px<BPC>::ibits(a.bdmax);
    const int PB = Px<BPC>::PBIAS;
    const int px = a.mx + x * a.dx, py = a.my + y * a.dy;
    const int col = px >> 10, row = py >> 10, fx = (px & 1023) >> 6, fy = (py & 1023) >> 6;
    const auto *s = a.src + row * a.ss + col;
    const int m0 = (int16_t)rnd_sh(blin(s[0], s[1], fx), 4 - ib);
    const int m1 = (int16_t)rnd_sh(blin(s[a.ss], s[a.ss + 1], fx), 4 - ib);
    return put ? clampi(rnd_sh(blin(m0, m1, fy), 4 + ib), 0, a.bdmax) : rnd_sh(blin(m0, m1, fy), 4) - PB;
}

template <int BPC>
__global__ __launch_bounds__(256) void k_mc(McArgs<BPC> a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.w || y >= a.h) return;
    const bool put = a.dst != nullptr;
    int v;
    if (a.ftype < 0)
        v = a.scaled ? mc_bilin_scaled_px(a, x, y, put) : mc_bilin_px(a, x, y, put);
    else
        v = a.scaled ? mc_8tap_scaled_px(a, x, y, put) : mc_8tap_px(a, x, y, put);
    if (put) a.dst[y * a.ds + x] = (typename Px<BPC>::pixel)v;
    else a.tmp[y * a.w + x] = (int16_t)v;
}

// avg_c / w_avg_c / mask_c / w_mask_c, src/mc_tmpl.c:587-639, :683-726.
// kind 0 avg, 1 w_avg, 2 mask, 3 w_mask (ssh/ssv = sub-sampling of the
// written mask).  The w_mask mask pixel is produced by the thread owning
// its top-left luma position from the 1/2/4 derived weights.
template <int BPC> struct AvgArgs {
    typename Px<BPC>::pixel *dst;
    ptrdiff_t ds;
    const int16_t *t1, *t2;
    const uint8_t *mask_in;
    uint8_t *mask_out;
    int w, h, kind, weight, sign, ssh, ssv, bdmax;
};

template <int BPC>
__device__ __forceinline__ int wmask_m(const AvgArgs<BPC> &a, int i, int msh, int mrnd) {
    return min(38 + ((abs(a.t1[i] - a.t2[i]) + mrnd) >> msh), 64);
}

template <int BPC>
__global__ __launch_bounds__(256) void k_avg(AvgArgs<BPC> a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.w || y >= a.h) return;
    const int ib = Px<BPC>::ibits(a.bdmax);
    const int PB = Px<BPC>::PBIAS;
    const int i = y * a.w + x;
    const int p = a.t1[i], q = a.t2[i];
    int v;
    if (a.kind == 0) {
        v = (p + q + (1 << ib) + 2 * PB) >> (ib + 1);
    } else if (a.kind == 1) {
        v = (p * a.weight + q * (16 - a.weight) + (8 << ib) + 16 * PB) >> (ib + 4);
    } else {
        int m;
        const int msh = bits_of(a.bdmax) + ib - 4, mrnd = 1 << (msh - 5);
        if (a.kind == 2) m = a.mask_in[i];
        else m = wmask_m(a, i, msh, mrnd);
        v = (p * m + q * (64 - m) + (32 << ib) + 64 * PB) >> (ib + 6);
        if (a.kind == 3 && !(x & a.ssh) && !(y & a.ssv)) {
            const int mw = a.w >> a.ssh;
            int out;
            if (!a.ssh) {
                out = m;
            } else if (!a.ssv) {
                out = (m + wmask_m(a, i + 1, msh, mrnd) + 1 - a.sign) >> 1;
            } else {
                const int s = m + wmask_m(a, i + 1, msh, mrnd) + wmask_m(a, i + a.w, msh, mrnd) +
                              wmask_m(a, i + a.w + 1, msh, mrnd);
                out = (s + 2 - a.sign) >> 2;
            }
            a.mask_out[(y >> a.ssv) * mw + (x >> a.ssh)] = (uint8_t)out;
        }
    }
    a.dst[y * a.ds + x] = (typename Px<BPC>::pixel)clampi(v, 0, a.bdmax);
}

// blend_c / blend_v_c / blend_h_c, src/mc_tmpl.c:641-681.  kind 0 blend
// (per-pixel mask), 1 blend_v (OBMC columns), 2 blend_h (OBMC rows).
template <int BPC> struct BlendArgs {
    typename Px<BPC>::pixel *dst;
    ptrdiff_t ds;
    const typename Px<BPC>::pixel *tmp;
    const uint8_t *mask;
    int w, h, kind;
};

template <int BPC>
__global__ __launch_bounds__(256) void k_blend(BlendArgs<BPC> a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.w || y >= a.h) return;
    int m;
    if (a.kind == 0) m = a.mask[y * a.w + x];
    else if (a.kind == 1) {
        if (x >= (a.w * 3) >> 2) return;
        m = dspt_obmc[a.w + x];
    } else {
        if (y >= (a.h * 3) >> 2) return;
        m = dspt_obmc[a.h + y];
    }
    auto &d = a.dst[y * a.ds + x];
    d = (typename Px<BPC>::pixel)((d * (64 - m) + a.tmp[y * a.w + x] * m + 32) >> 6);
}

// warp_affine_8x8(t)_c, src/mc_tmpl.c:758-825
template <int BPC> struct WarpArgs {
    typename Px<BPC>::pixel *dst;
    ptrdiff_t ds;
    int16_t *tmp;
    ptrdiff_t ts;
    const typename Px<BPC>::pixel *src;
    ptrdiff_t ss;
    int a0, a1, a2, a3, mx, my, bdmax;
};

template <int BPC>
__global__ __launch_bounds__(64) void k_warp(WarpArgs<BPC> a) {
    const int x = threadIdx.x & 7, y = threadIdx.x >> 3;
    const int ib = Px<BPC>::ibits(a.bdmax);
    const int coly = a.my + y * a.a3 + x * a.a2;
    const signed char *kv = &dspt_warp[(64 + ((coly + 512) >> 10)) * 8];
    int acc = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int r = y + k;  // intermediate row r <-> source row r - 3
        const int rowx = a.mx + r * a.a1 + x * a.a0;
        const signed char *kh = &dspt_warp[(64 + ((rowx + 512) >> 10)) * 8];
        const auto *s = a.src + (r - 3) * a.ss + x;
        const int mid = (int16_t)rnd_sh(tap8<BPC>(s, 1, kh), 7 - ib);
        acc += kv[k] * mid;
    }
    if (a.dst) a.dst[y * a.ds + x] = (typename Px<BPC>::pixel)clampi(rnd_sh(acc, 7 + ib), 0, a.bdmax);
    else a.tmp[y * a.ts + x] = (int16_t)(rnd_sh(acc, 7) - Px<BPC>::PBIAS);
}

// emu_edge_c, src/mc_tmpl.c:827-875: replicate padding == clamped fetch
template <int BPC> struct EmuArgs {
    typename Px<BPC>::pixel *dst;
    ptrdiff_t ds;
    const typename Px<BPC>::pixel *ref;
    ptrdiff_t rs;
    int bw, bh, iw, ih, x, y;
};

template <int BPC>
__global__ __launch_bounds__(256) void k_emu_edge(EmuArgs<BPC> a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.bw || y >= a.bh) return;
    const int sy = clampi(a.y + y, 0, a.ih - 1), sx = clampi(a.x + x, 0, a.iw - 1);
    a.dst[y * a.ds + x] = a.ref[sy * a.rs + sx];
}

// resize_c, src/mc_tmpl.c:877-903 (14-bit source position)
template <int BPC> struct ResizeArgs {
    typename Px<BPC>::pixel *dst;
    ptrdiff_t ds;
    const typename Px<BPC>::pixel *src;
    ptrdiff_t ss;
    int dst_w, h, src_w, dx, mx0, bdmax;
};

template <int BPC>
__global__ __launch_bounds__(256) void k_resize(ResizeArgs<BPC> a) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= a.dst_w || y >= a.h) return;
    const int pos = a.mx0 + x * a.dx;
    const int sx = (pos >> 14) - 1;
    const signed char *k = &dspt_resize[((pos & 0x3fff) >> 8) * 8];
    const auto *s = a.src + y * a.ss;
    int sum = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) sum += k[i] * (int)s[clampi(sx + i - 3, 0, a.src_w - 1)];
    a.dst[y * a.ds + x] = (typename Px<BPC>::pixel)clampi((-sum + 64) >> 7, 0, a.bdmax);
}

// Super-res frame tier (dav1d_filter_sbrow_resize for the whole frame): one
// launch, blockIdx.z = plane.  A wave upscales 256 consecutive output pixels
// of kRzRows rows: the source spans they read (at most 256 * dx / 2^14 + 8
// pixels per row, dx <= 2^14 since super-res only upscales) are loaded once
// into LDS with the reference's column clamp applied at load time (every
// row's loads in flight together), then each lane filters four outputs
// (x0 + lane + 64 k) per row from LDS with the 8 taps of resize_c.
constexpr int kRzOut = 256, kRzSpan = kRzOut + 16;
// Rows per wave: 2 measured 27.6 against 26.8 us; 4 neighbouring outputs
// per lane stored as one 4-pixel word 27.3 against 27.2 (both deleted in
// round 6).
constexpr int kRzRows = 1;
template <int BPC> struct ResizeFrameArgs {
    typename Px<BPC>::pixel *dst[3];
    const typename Px<BPC>::pixel *src[3];
    int ds[3], ss[3];   // pixels
    int dst_w[3], src_w[3], h[3], dx[3], mx0[3];
    int bdmax;
};
template <int BPC>
__global__ __launch_bounds__(256) void k_resize_frame(ResizeFrameArgs<BPC> a) {
    using P = typename Px<BPC>::pixel;
    __shared__ P span[4][kRzRows][kRzSpan];
    const int p = blockIdx.z, w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int y0 = (blockIdx.y * 4 + w) * kRzRows, x0 = blockIdx.x * kRzOut;
    const int dw = a.dst_w[p], sw = a.src_w[p], dx = a.dx[p], mx0 = a.mx0[p], hh = a.h[p];
    if (y0 >= hh || x0 >= dw) return;   // wave-uniform
    const int s0 = ((mx0 + x0 * dx) >> 14) - 4;   // first source column a tap of this run reads
    constexpr int NK = kRzSpan / 64 + 1;
    P v[kRzRows][NK];
#pragma unroll
    for (int r = 0; r < kRzRows; r++) {   // every row's loads first
        const P *s = a.src[p] + (size_t)min(y0 + r, hh - 1) * a.ss[p];
#pragma unroll
        for (int k = 0; k < NK; k++) {
            const int i = l + 64 * k;
            if (i < kRzSpan) v[r][k] = s[clampi(s0 + i, 0, sw - 1)];
        }
    }
#pragma unroll
    for (int r = 0; r < kRzRows; r++)
#pragma unroll
        for (int k = 0; k < NK; k++) {
            const int i = l + 64 * k;
            if (i < kRzSpan) span[w][r][i] = v[r][k];
        }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int r = 0; r < kRzRows; r++) {
        if (y0 + r >= hh) break;
        const P *t = span[w][r];
        P *d = a.dst[p] + (size_t)(y0 + r) * a.ds[p];
#pragma unroll
        for (int k = 0; k < kRzOut / 64; k++) {
            const int x = x0 + l + 64 * k;
            if (x < dw) {
                const int pos = mx0 + x * dx;
                const P *c = t + ((pos >> 14) - 4 - s0);   // taps c[0..7] = source (pos >> 14) - 4 .. + 3
                const signed char *f = &dspt_resize[((pos & 0x3fff) >> 8) * 8];
                int sum = 0;
#pragma unroll
                for (int i = 0; i < 8; i++) sum += f[i] * (int)c[i];
                d[x] = (P)clampi((-sum + 64) >> 7, 0, a.bdmax);
            }
        }
    }
}

template <int BPC>
static int launch_resize_frame(const Dav1dGpuResizeFrame *f, hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    constexpr int B = BPC / 8;
    if (!f || f->layout < 0 || f->layout > 3) return -1;
    const int np = f->layout ? 3 : 1;
    ResizeFrameArgs<BPC> a{};
    int gw = 0, gh = 0;
    for (int p = 0; p < np; p++) {
        const Dav1dGpuPlane &i = f->in[p], &o = f->out[p];
        if (!i.data || !o.data || i.w <= 0 || o.w <= 0 || i.h <= 0 || o.h < i.h || i.stride < (int64_t)i.w * B ||
            o.stride < (int64_t)o.w * B || (i.stride % B) || (o.stride % B))
            return -1;
        a.src[p] = (const P *)i.data;
        a.dst[p] = (P *)o.data;
        a.ss[p] = (int)(i.stride / B);
        a.ds[p] = (int)(o.stride / B);
        a.src_w[p] = i.w;
        a.dst_w[p] = o.w;
        a.h[p] = i.h;
        a.dx[p] = f->step[p ? 1 : 0];
        a.mx0[p] = f->start[p ? 1 : 0];
        if (f->step[p ? 1 : 0] <= 0 || f->step[p ? 1 : 0] > 1 << 14) return -1;   // super-res upscales
        gw = max(gw, (o.w + kRzOut - 1) / kRzOut);
        gh = max(gh, (i.h + 4 * kRzRows - 1) / (4 * kRzRows));
    }
    a.bdmax = BPC == 8 ? 255 : f->bitdepth_max;
    k_resize_frame<BPC><<<dim3(gw, gh, np), 256, 0, stream>>>(a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ---------------------------------------------------------------------------
// Host entries with the reference signatures.
// ---------------------------------------------------------------------------
static inline dim3 grid16(int w, int h) { return dim3((w + 15) / 16, (h + 15) / 16); }

template <int BPC> struct HostPx;
template <> struct HostPx<8> { static constexpr int bdmax(int) { return 255; } };
template <> struct HostPx<16> { static int bdmax(int v) { return v; } };

template <int BPC, int F, bool SCALED>
static bool run_mc(typename Px<BPC>::pixel *dst, ptrdiff_t dst_stride, int16_t *tmp,
                   const typename Px<BPC>::pixel *src, ptrdiff_t src_stride, int w, int h,
                   int mx, int my, int dx, int dy, int bdmax) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    const bool bil = F == DGPU_FILTER_2D_BILINEAR;
    long c0, c1, r0, r1;
    if (!SCALED) {
        if (bil) {
            c0 = 0; c1 = w + (mx ? 1 : 0);
            r0 = 0; r1 = h + (my ? 1 : 0);
        } else {
            c0 = mx ? -3 : 0; c1 = w + (mx ? 4 : 0);
            r0 = my ? -3 : 0; r1 = h + (my ? 4 : 0);
        }
    } else {
        // exact footprint of the reference loops (src/mc_tmpl.c:182-199)
        c0 = 1L << 30; c1 = -(1L << 30);
        for (int x = 0; x < w; x++) {
            const int pos = mx + x * dx, off = pos >> 10;
            const bool f = bil || ((pos & 1023) >> 6) != 0;
            const long lo = bil ? off : f ? off - 3 : off;
            const long hi = bil ? off + 2 : f ? off + 5 : off + 1;
            if (lo < c0) c0 = lo;
            if (hi > c1) c1 = hi;
        }
        const int rows = (((h - 1) * dy + my) >> 10) + (bil ? 2 : 8);
        r0 = bil ? 0 : -3;
        r1 = r0 + rows;
    }
    Stager st;
    const int is = st.in(src, src_stride, c0 * B, c1 * B, r0, r1);
    const int od = dst ? st.out(dst, dst_stride, 0, w * B, 0, h) : st.out1(tmp, (long)w * h * 2);
    if (!st.upload()) return false;
    McArgs<BPC> a;
    a.dst = dst ? st.origin<P>(od) : nullptr;
    a.ds = dst ? st.pitch(od) / B : 0;
    a.tmp = dst ? nullptr : st.origin<int16_t>(od);
    a.src = st.origin<const P>(is);
    a.ss = st.pitch(is) / B;
    a.w = w; a.h = h; a.mx = mx; a.my = my; a.dx = dx; a.dy = dy;
    a.ftype = bil ? -1 : kFtype[F];
    a.scaled = SCALED;
    a.bdmax = bdmax;
    k_mc<BPC><<<grid16(w, h), 256, 0, st.stream()>>>(a);
    return st.finish();
}

// The caller's entries before dav1d_mc_dsp_init_gpu_* overwrote them (C
// defaults, run when the GPU path fails: runtime.hpp's error contract).
static Dav1dMCDSPContext_8bpc g_fb8;
static Dav1dMCDSPContext_16bpc g_fb16;

// --- 8bpc / 16bpc signature adapters --------------------------------------
#define BD8_PARAM
#define BD8_VAL 255
#define BD8_VAL_ARG
#define BD16_PARAM , int bitdepth_max
#define BD16_VAL bitdepth_max
#define BD16_VAL_ARG , bitdepth_max

#define MC_ENTRIES(BPC, P, BDP, BDV)                                                           \
template <int F> static void put_##BPC(P *d, ptrdiff_t ds, const P *s, ptrdiff_t ss, int w,    \
                                       int h, int mx, int my BDP)                              \
{ DGPU_OR_FALLBACK((run_mc<BPC, F, false>(d, ds, nullptr, s, ss, w, h, mx, my, 0, 0, BDV)),    \
                   g_fb##BPC.mc[F], d, ds, s, ss, w, h, mx, my BDV##_ARG); }                   \
template <int F> static void prep_##BPC(int16_t *t, const P *s, ptrdiff_t ss, int w, int h,    \
                                        int mx, int my BDP)                                    \
{ DGPU_OR_FALLBACK((run_mc<BPC, F, false>(nullptr, 0, t, s, ss, w, h, mx, my, 0, 0, BDV)),     \
                   g_fb##BPC.mct[F], t, s, ss, w, h, mx, my BDV##_ARG); }                      \
template <int F> static void put_scaled_##BPC(P *d, ptrdiff_t ds, const P *s, ptrdiff_t ss,    \
                                              int w, int h, int mx, int my, int dx, int dy BDP)\
{ DGPU_OR_FALLBACK((run_mc<BPC, F, true>(d, ds, nullptr, s, ss, w, h, mx, my, dx, dy, BDV)),   \
                   g_fb##BPC.mc_scaled[F], d, ds, s, ss, w, h, mx, my, dx, dy BDV##_ARG); }    \
template <int F> static void prep_scaled_##BPC(int16_t *t, const P *s, ptrdiff_t ss, int w,    \
                                               int h, int mx, int my, int dx, int dy BDP)      \
{ DGPU_OR_FALLBACK((run_mc<BPC, F, true>(nullptr, 0, t, s, ss, w, h, mx, my, dx, dy, BDV)),    \
                   g_fb##BPC.mct_scaled[F], t, s, ss, w, h, mx, my, dx, dy BDV##_ARG); }

MC_ENTRIES(8, uint8_t, BD8_PARAM, BD8_VAL)
MC_ENTRIES(16, uint16_t, BD16_PARAM, BD16_VAL)

template <int BPC>
static bool run_avg(typename Px<BPC>::pixel *dst, ptrdiff_t dst_stride, const int16_t *t1,
                    const int16_t *t2, int w, int h, int kind, int weight, const uint8_t *mask_in,
                    uint8_t *mask_out, int sign, int ssh, int ssv, int bdmax) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    Stager st;
    const long n = (long)w * h;
    const int i1 = st.in1(t1, n * 2), i2 = st.in1(t2, n * 2);
    const int im = kind == 2 ? st.in1(mask_in, n) : -1;
    const int om = kind == 3 ? st.out1(mask_out, (long)(w >> ssh) * (h >> ssv)) : -1;
    const int od = st.out(dst, dst_stride, 0, w * B, 0, h);
    if (!st.upload()) return false;
    AvgArgs<BPC> a;
    a.dst = st.origin<P>(od);
    a.ds = st.pitch(od) / B;
    a.t1 = st.origin<const int16_t>(i1);
    a.t2 = st.origin<const int16_t>(i2);
    a.mask_in = im >= 0 ? st.origin<const uint8_t>(im) : nullptr;
    a.mask_out = om >= 0 ? st.origin<uint8_t>(om) : nullptr;
    a.w = w; a.h = h; a.kind = kind; a.weight = weight; a.sign = sign; a.ssh = ssh; a.ssv = ssv;
    a.bdmax = bdmax;
    k_avg<BPC><<<grid16(w, h), 256, 0, st.stream()>>>(a);
    return st.finish();
}

#define AVG_ENTRIES(BPC, P, BDP, BDV)                                                          \
static void avg_##BPC(P *d, ptrdiff_t ds, const int16_t *a, const int16_t *b, int w, int h BDP)\
{ DGPU_OR_FALLBACK((run_avg<BPC>(d, ds, a, b, w, h, 0, 0, nullptr, nullptr, 0, 0, 0, BDV)),    \
                   g_fb##BPC.avg, d, ds, a, b, w, h BDV##_ARG); }                              \
static void w_avg_##BPC(P *d, ptrdiff_t ds, const int16_t *a, const int16_t *b, int w, int h,  \
                        int wt BDP)                                                            \
{ DGPU_OR_FALLBACK((run_avg<BPC>(d, ds, a, b, w, h, 1, wt, nullptr, nullptr, 0, 0, 0, BDV)),   \
                   g_fb##BPC.w_avg, d, ds, a, b, w, h, wt BDV##_ARG); }                        \
static void mask_##BPC(P *d, ptrdiff_t ds, const int16_t *a, const int16_t *b, int w, int h,   \
                       const uint8_t *m BDP)                                                   \
{ DGPU_OR_FALLBACK((run_avg<BPC>(d, ds, a, b, w, h, 2, 0, m, nullptr, 0, 0, 0, BDV)),          \
                   g_fb##BPC.mask, d, ds, a, b, w, h, m BDV##_ARG); }                          \
template <int SSH, int SSV>                                                                    \
static void w_mask_##BPC(P *d, ptrdiff_t ds, const int16_t *a, const int16_t *b, int w, int h, \
                         uint8_t *m, int sign BDP)                                             \
{ DGPU_OR_FALLBACK((run_avg<BPC>(d, ds, a, b, w, h, 3, 0, nullptr, m, sign, SSH, SSV, BDV)),   \
                   g_fb##BPC.w_mask[SSH + SSV], d, ds, a, b, w, h, m, sign BDV##_ARG); }

AVG_ENTRIES(8, uint8_t, BD8_PARAM, BD8_VAL)
AVG_ENTRIES(16, uint16_t, BD16_PARAM, BD16_VAL)

template <int BPC>
static bool run_blend(typename Px<BPC>::pixel *dst, ptrdiff_t dst_stride,
                      const typename Px<BPC>::pixel *tmp, int w, int h, const uint8_t *mask,
                      int kind) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    Stager st;
    const int it = st.in1(tmp, (long)w * h * B);
    const int im = kind == 0 ? st.in1(mask, (long)w * h) : -1;
    const long cw = kind == 1 ? (w * 3) >> 2 : w;
    const long ch = kind == 2 ? (h * 3) >> 2 : h;
    const int od = st.inout(dst, dst_stride, 0, cw * B, 0, ch);
    if (!st.upload()) return false;
    BlendArgs<BPC> a;
    a.dst = st.origin<P>(od);
    a.ds = st.pitch(od) / B;
    a.tmp = st.origin<const P>(it);
    a.mask = im >= 0 ? st.origin<const uint8_t>(im) : nullptr;
    a.w = w; a.h = h; a.kind = kind;
    k_blend<BPC><<<grid16(w, h), 256, 0, st.stream()>>>(a);
    return st.finish();
}

template <int BPC>
static bool run_warp(typename Px<BPC>::pixel *dst, ptrdiff_t dst_stride, int16_t *tmp,
                     ptrdiff_t tmp_stride, const typename Px<BPC>::pixel *src,
                     ptrdiff_t src_stride, const int16_t *abcd, int mx, int my, int bdmax) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    Stager st;
    const int is = st.in(src, src_stride, -3 * B, 12 * B, -3, 12);
    const int od = dst ? st.out(dst, dst_stride, 0, 8 * B, 0, 8)
                       : st.out(tmp, tmp_stride * 2, 0, 16, 0, 8);
    if (!st.upload()) return false;
    WarpArgs<BPC> a;
    a.dst = dst ? st.origin<P>(od) : nullptr;
    a.ds = dst ? st.pitch(od) / B : 0;
    a.tmp = dst ? nullptr : st.origin<int16_t>(od);
    a.ts = dst ? 0 : st.pitch(od) / 2;
    a.src = st.origin<const P>(is);
    a.ss = st.pitch(is) / B;
    a.a0 = abcd[0]; a.a1 = abcd[1]; a.a2 = abcd[2]; a.a3 = abcd[3];
    a.mx = mx; a.my = my; a.bdmax = bdmax;
    k_warp<BPC><<<1, 64, 0, st.stream()>>>(a);
    return st.finish();
}

template <int BPC>
static bool emu_edge_t(intptr_t bw, intptr_t bh, intptr_t iw, intptr_t ih, intptr_t x, intptr_t y,
                       typename Px<BPC>::pixel *dst, ptrdiff_t dst_stride,
                       const typename Px<BPC>::pixel *ref, ptrdiff_t ref_stride) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    auto cl = [](long v, long lo, long hi) { return v < lo ? lo : v > hi ? hi : v; };
    const long sx0 = cl(x, 0, iw - 1), sx1 = cl(x + bw - 1, 0, iw - 1);
    const long sy0 = cl(y, 0, ih - 1), sy1 = cl(y + bh - 1, 0, ih - 1);
    Stager st;
    const int ir = st.in(ref, ref_stride, sx0 * B, (sx1 + 1) * B, sy0, sy1 + 1);
    const int od = st.out(dst, dst_stride, 0, bw * B, 0, bh);
    if (!st.upload()) return false;
    EmuArgs<BPC> a;
    a.dst = st.origin<P>(od);
    a.ds = st.pitch(od) / B;
    a.ref = st.origin<const P>(ir);
    a.rs = st.pitch(ir) / B;
    a.bw = (int)bw; a.bh = (int)bh; a.iw = (int)iw; a.ih = (int)ih; a.x = (int)x; a.y = (int)y;
    k_emu_edge<BPC><<<grid16((int)bw, (int)bh), 256, 0, st.stream()>>>(a);
    return st.finish();
}

template <int BPC>
static bool run_resize(typename Px<BPC>::pixel *dst, ptrdiff_t dst_stride,
                       const typename Px<BPC>::pixel *src, ptrdiff_t src_stride, int dst_w, int h,
                       int src_w, int dx, int mx0, int bdmax) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    Stager st;
    const int is = st.in(src, src_stride, 0, src_w * B, 0, h);
    const int od = st.out(dst, dst_stride, 0, dst_w * B, 0, h);
    if (!st.upload()) return false;
    ResizeArgs<BPC> a;
    a.dst = st.origin<P>(od);
    a.ds = st.pitch(od) / B;
    a.src = st.origin<const P>(is);
    a.ss = st.pitch(is) / B;
    a.dst_w = dst_w; a.h = h; a.src_w = src_w; a.dx = dx; a.mx0 = mx0; a.bdmax = bdmax;
    k_resize<BPC><<<dim3((dst_w + 63) / 64, (h + 3) / 4), 256, 0, st.stream()>>>(a);
    return st.finish();
}

#define MISC_ENTRIES(BPC, P, BDP, BDV)                                                         \
static void blend_##BPC(P *d, ptrdiff_t ds, const P *t, int w, int h, const uint8_t *m)        \
{ DGPU_OR_FALLBACK((run_blend<BPC>(d, ds, t, w, h, m, 0)), g_fb##BPC.blend, d, ds, t, w, h, m); }\
static void blend_v_##BPC(P *d, ptrdiff_t ds, const P *t, int w, int h)                        \
{ DGPU_OR_FALLBACK((run_blend<BPC>(d, ds, t, w, h, nullptr, 1)), g_fb##BPC.blend_v, d, ds, t, w, h); }\
static void blend_h_##BPC(P *d, ptrdiff_t ds, const P *t, int w, int h)                        \
{ DGPU_OR_FALLBACK((run_blend<BPC>(d, ds, t, w, h, nullptr, 2)), g_fb##BPC.blend_h, d, ds, t, w, h); }\
static void warp_##BPC(P *d, ptrdiff_t ds, const P *s, ptrdiff_t ss, const int16_t *abcd,      \
                       int mx, int my BDP)                                                     \
{ DGPU_OR_FALLBACK((run_warp<BPC>(d, ds, nullptr, 0, s, ss, abcd, mx, my, BDV)),               \
                   g_fb##BPC.warp8x8, d, ds, s, ss, abcd, mx, my BDV##_ARG); }                 \
static void warpt_##BPC(int16_t *t, ptrdiff_t ts, const P *s, ptrdiff_t ss,                    \
                        const int16_t *abcd, int mx, int my BDP)                               \
{ DGPU_OR_FALLBACK((run_warp<BPC>(nullptr, 0, t, ts, s, ss, abcd, mx, my, BDV)),               \
                   g_fb##BPC.warp8x8t, t, ts, s, ss, abcd, mx, my BDV##_ARG); }                \
static void emu_edge_##BPC(intptr_t bw, intptr_t bh, intptr_t iw, intptr_t ih, intptr_t x,     \
                           intptr_t y, P *d, ptrdiff_t ds, const P *r, ptrdiff_t rs)           \
{ DGPU_OR_FALLBACK((emu_edge_t<BPC>(bw, bh, iw, ih, x, y, d, ds, r, rs)),                      \
                   g_fb##BPC.emu_edge, bw, bh, iw, ih, x, y, d, ds, r, rs); }                  \
static void resize_##BPC(P *d, ptrdiff_t ds, const P *s, ptrdiff_t ss, int dw, int h, int sw,  \
                         int dx, int mx BDP)                                                   \
{ DGPU_OR_FALLBACK((run_resize<BPC>(d, ds, s, ss, dw, h, sw, dx, mx, BDV)),                    \
                   g_fb##BPC.resize, d, ds, s, ss, dw, h, sw, dx, mx BDV##_ARG); }

MISC_ENTRIES(8, uint8_t, BD8_PARAM, BD8_VAL)
MISC_ENTRIES(16, uint16_t, BD16_PARAM, BD16_VAL)

#define FILL_MC(BPC, c)                                                                        \
    do {                                                                                       \
        c->mc[0] = put_##BPC<0>; c->mc[1] = put_##BPC<1>; c->mc[2] = put_##BPC<2>;             \
        c->mc[3] = put_##BPC<3>; c->mc[4] = put_##BPC<4>; c->mc[5] = put_##BPC<5>;             \
        c->mc[6] = put_##BPC<6>; c->mc[7] = put_##BPC<7>; c->mc[8] = put_##BPC<8>;             \
        c->mc[9] = put_##BPC<9>;                                                               \
        c->mct[0] = prep_##BPC<0>; c->mct[1] = prep_##BPC<1>; c->mct[2] = prep_##BPC<2>;       \
        c->mct[3] = prep_##BPC<3>; c->mct[4] = prep_##BPC<4>; c->mct[5] = prep_##BPC<5>;       \
        c->mct[6] = prep_##BPC<6>; c->mct[7] = prep_##BPC<7>; c->mct[8] = prep_##BPC<8>;       \
        c->mct[9] = prep_##BPC<9>;                                                             \
        c->mc_scaled[0] = put_scaled_##BPC<0>; c->mc_scaled[1] = put_scaled_##BPC<1>;          \
        c->mc_scaled[2] = put_scaled_##BPC<2>; c->mc_scaled[3] = put_scaled_##BPC<3>;          \
        c->mc_scaled[4] = put_scaled_##BPC<4>; c->mc_scaled[5] = put_scaled_##BPC<5>;          \
        c->mc_scaled[6] = put_scaled_##BPC<6>; c->mc_scaled[7] = put_scaled_##BPC<7>;          \
        c->mc_scaled[8] = put_scaled_##BPC<8>; c->mc_scaled[9] = put_scaled_##BPC<9>;          \
        c->mct_scaled[0] = prep_scaled_##BPC<0>; c->mct_scaled[1] = prep_scaled_##BPC<1>;      \
        c->mct_scaled[2] = prep_scaled_##BPC<2>; c->mct_scaled[3] = prep_scaled_##BPC<3>;      \
        c->mct_scaled[4] = prep_scaled_##BPC<4>; c->mct_scaled[5] = prep_scaled_##BPC<5>;      \
        c->mct_scaled[6] = prep_scaled_##BPC<6>; c->mct_scaled[7] = prep_scaled_##BPC<7>;      \
        c->mct_scaled[8] = prep_scaled_##BPC<8>; c->mct_scaled[9] = prep_scaled_##BPC<9>;      \
        c->avg = avg_##BPC; c->w_avg = w_avg_##BPC; c->mask = mask_##BPC;                      \
        c->w_mask[0] = w_mask_##BPC<0, 0>; c->w_mask[1] = w_mask_##BPC<1, 0>;                  \
        c->w_mask[2] = w_mask_##BPC<1, 1>;                                                     \
        c->blend = blend_##BPC; c->blend_v = blend_v_##BPC; c->blend_h = blend_h_##BPC;        \
        c->warp8x8 = warp_##BPC; c->warp8x8t = warpt_##BPC;                                    \
        c->emu_edge = emu_edge_##BPC; c->resize = resize_##BPC;                               \
    } while (0)

}  // namespace dgpu

using namespace dgpu;

// bitfn(dav1d_mc_dsp_init) replacement, src/mc_tmpl.c:915-957
// The _gpu_ hooks keep the caller's previous entries as fallbacks.
extern "C" void dav1d_mc_dsp_init_gpu_8bpc(Dav1dMCDSPContext_8bpc *c) {
    Dav1dMCDSPContext_8bpc g{}, *gp = &g;
    FILL_MC(8, gp);
    save_fallback(&g_fb8, c, gp);
    FILL_MC(8, c);
}
extern "C" void dav1d_mc_dsp_init_gpu_16bpc(Dav1dMCDSPContext_16bpc *c) {
    Dav1dMCDSPContext_16bpc g{}, *gp = &g;
    FILL_MC(16, gp);
    save_fallback(&g_fb16, c, gp);
    FILL_MC(16, c);
}
extern "C" void dav1d_mc_dsp_init_8bpc(Dav1dMCDSPContext_8bpc *c) { FILL_MC(8, c); }
extern "C" void dav1d_mc_dsp_init_16bpc(Dav1dMCDSPContext_16bpc *c) { FILL_MC(16, c); }

extern "C" int dav1d_gpu_resize_frame_8bpc(const Dav1dGpuResizeFrame *f, void *stream) {
    return launch_resize_frame<8>(f, (hipStream_t)stream);
}
extern "C" int dav1d_gpu_resize_frame_16bpc(const Dav1dGpuResizeFrame *f, void *stream) {
    return launch_resize_frame<16>(f, (hipStream_t)stream);
}
