// lr.hip -- loop restoration on the device (include/
// dav1d_gpu.h, Dav1dLoopRestorationDSPContext): the per-call entries of
// src/looprestoration_tmpl.c (wiener_c :134-190, sgr_5x5_c / sgr_3x3_c /
// sgr_mix_c :449-525) for one restoration-unit stripe per call.
//
// One 256-thread workgroup per 32-column strip of the unit.  The strip's
// (h + 6) x (32 + 6) context is built in LDS with padding()'s rules
// (:40-132) in closed form: rows above / below from the loop-filtered `lpf`
// rows (0, 0, 1 above; 6, 7, 7 below) or the first / last row, columns left
// of the unit from `left` or replicated, right of it from the picture or
// replicated.  Wiener: the horizontal 7-tap pass into LDS (uint16 range
// clip), then the vertical one.  Self-guided (round 5: both radii in one
// pass): A / B of the 5x5 and 3x3 boxes from horizontal sums slid down each
// column in registers (the reference's boxsum5 / boxsum3, the
// dav1d_sgr_x_by_x lookup and the inversion, with its unsigned arithmetic),
// one barrier, then both weightings and the w0 / w1 blend per pixel.
// Latency-bound per call like the
// other per-call entries.
//
// Frame tier, k_lr_frame: bytefn(dav1d_lr_sbrow) (lr_apply_tmpl.c:169-202)
// for a whole frame in one launch, one workgroup per (plane, stripe,
// 32-column strip), the same strip code with the stripe's context rows from
// the deblocked picture (what dav1d_copy_lpf saves) and the unit's left and
// right columns from the pre-LR picture (what lr_sbrow backs up).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "dav1d_gpu.h"
#include "dsp_common.hpp"
#include "runtime.hpp"

namespace dgpu {

constexpr int kLrSW = 32;              // strip width
constexpr int kLrTW = kLrSW + 6;       // tile width
constexpr int kLrTH = 64 + 6;          // tile height
constexpr int kLrGroup = 8;            // frame tier: consecutive strips per XCD run

template <int BPC> struct LrArgs {
    using P = typename Px<BPC>::pixel;
    const P *src;     // the unit's pixels (rows 0..h-1), pitch ss
    P *dst;           // output rect, pitch ds
    const P *top;     // lpf rows 0-1 (HAVE_TOP), pitch ts
    const P *bot;     // lpf rows 6-7 (HAVE_BOTTOM), pitch bs
    const P *left;    // [h][4]; null: the columns left of the unit are src's
    int ss, ds, ts, bs;
    int w, h, edges, kind, bdmax;   // kind: 0 wiener, 1 sgr 5x5, 2 sgr 3x3, 3 mix
    int vec;                        // every pointer and pitch 16-byte aligned
    Dav1dGpuLrParams prm;
};

constexpr int kLrVH = 66;   // A / B rows: unit rows -1..64

// Full 32-column strips on 16-byte-aligned planes (`vec`) move their pixels
// in 16-byte pieces instead of one pixel per lane: the copied (unrestored)
// strips and the tile's 32 interior columns (the 3 + 3 padding columns keep
// the per-pixel padding() code).  Measured and deleted in round 6: outputs
// staged in LDS and stored as whole rows (two more barriers, slower), the
// next tile row's LDS reads issued one A / B iteration ahead (slower); the
// A / B loop stays unrolled by two (47.8-48.0 against 48.8-49.3 us,
// profiles/r5/r5z_lr_unroll_ab.json).

// A / B of selfguided_filter (:373-392) from one position's box sum and sum
// of squares (n = 25 or 9), with the reference's unsigned arithmetic
template <int n>
__device__ __forceinline__ void lr_ab_sums(int sum, int sumsq, unsigned s, int bd8, const uint8_t *x_by_x, int &A,
                                           int &B) {
    constexpr unsigned one_by_x = n == 25 ? 164 : 455;
    const int a = (sumsq + ((1 << (2 * bd8)) >> 1)) >> (2 * bd8);
    const int b = (sum + ((1 << bd8) >> 1)) >> bd8;
    const unsigned p = (unsigned)max(a * n - b * b, 0);
    const unsigned z = (p * s + (1u << 19)) >> 20;
    const unsigned x = x_by_x[min(z, 255u)];   // the block's LDS copy
    A = (int)((x * (unsigned)sum * one_by_x + (1u << 11)) >> 12);
    B = (int)x;
}

// One 32-column strip (columns x0.. of the unit) of one stripe.
template <int BPC>
__device__ __forceinline__ void lr_strip(const LrArgs<BPC> &a, const int x0) {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    // 16-bit tiles and scratch where the values fit (pixels, Wiener's clipped
    // horizontal sums, 5-row box sums, B = x_by_x <= 255): 31.8 KB, five
    // workgroups per CU
    __shared__ __attribute__((aligned(16))) int16_t T[kLrTH][kLrTW];
    // 3x3 A / B at unit rows -1..h (every row), strip columns -1..sw; the
    // Wiener units' horizontal pass reuses the A array
    // (32-bit A: 16-bit A arrays at 8 bit -- A <= 65089 fits -- gave 15.7 KB
    // per workgroup and 8 waves per SIMD but measured 60.9 against 50.9 us:
    // the 2-byte LDS accesses of neighbouring lanes share dwords)
    using AT = int;
    __shared__ AT AA[kLrVH][kLrSW + 2];
    __shared__ uint8_t BB[kLrVH][kLrSW + 2];
    // 5x5 A / B at unit rows -1, 1, .. (row jj at jj / 2)
    __shared__ AT AA5[kLrVH / 2][kLrSW + 2];
    __shared__ uint8_t BB5[kLrVH / 2][kLrSW + 2];
    // sgr_x_by_x in LDS: a global-memory lookup per A / B position put one
    // memory round trip per loop iteration on the block's critical path
    __shared__ uint8_t XBX[256];
    if (a.kind) XBX[threadIdx.x] = dspt_sgr_x_by_x[threadIdx.x];
    int16_t(*HOR)[kLrSW] = reinterpret_cast<int16_t(*)[kLrSW]>(&AA[0][0]);
    static_assert(kLrTH * kLrSW * 2 <= (int)sizeof(AA), "HOR fits the A array");
    const int sw = min(kLrSW, a.w - x0), h = a.h;
    // 8 bpc: compile-time bitdepth (the shifts and roundings of the A / B
    // sums and both filters fold away)
    const int bdmax = BPC == 8 ? 255 : a.bdmax, bd8 = BPC == 8 ? 0 : bits_of(a.bdmax) - 8;
    // a full strip on aligned planes (workgroup-uniform)
    const bool vec = a.vec && sw == kLrSW;
    if (vec) {   // the 32 interior columns read no padding: 16-byte row pieces
        constexpr int PR = kLrSW * (int)sizeof(P) / 16, NV = (kLrTH * PR + 255) / 256;   // pieces per row
        const bool ht = a.edges & DGPU_LR_HAVE_TOP, hb = a.edges & DGPU_LR_HAVE_BOTTOM;
        uint4 pv[NV];
#pragma unroll
        for (int i = 0; i < NV; i++) {
            const int t = threadIdx.x + 256 * i, r = t / PR, k = t % PR;
            if (r < h + 6) {
                const int j = min(max(r - 3, 0), h - 1);
                const P *p = a.src + (ptrdiff_t)j * a.ss + x0;
                if (r < 3 && ht) p = a.top + (r == 2) * a.ts + x0;
                if (r >= h + 3 && hb) p = a.bot + (r > h + 3) * a.bs + x0;
                pv[i] = *reinterpret_cast<const uint4 *>(p + k * (16 / (int)sizeof(P)));
            }
        }
        // the padding columns 0-2 and 35-37, a thread per (row, column)
        constexpr int NH = (kLrTH * 6 + 255) / 256;
        const bool hl = a.edges & DGPU_LR_HAVE_LEFT, hr = a.edges & DGPU_LR_HAVE_RIGHT;
        int hv[NH];
#pragma unroll
        for (int i = 0; i < NH; i++) {
            const int t = threadIdx.x + 256 * i, r = t / 6, e = t % 6, c = e < 3 ? e : kLrSW + e;
            int cc = x0 + c;
            if (!hr && cc >= a.w + 3) cc = a.w + 2;
            if (!hl && cc < 3) cc = 3;
            const int x = cc - 3;
            hv[i] = 0;
            if (r < h + 6) {
                const int j = min(max(r - 3, 0), h - 1);
                const P *p = x < 0 && a.left ? a.left + j * 4 + x + 4 : a.src + (ptrdiff_t)j * a.ss + x;
                if (r < 3 && ht) p = a.top + (r == 2) * a.ts + x;
                if (r >= h + 3 && hb) p = a.bot + (r > h + 3) * a.bs + x;
                hv[i] = *p;
            }
        }
#pragma unroll
        for (int i = 0; i < NV; i++) {
            const int t = threadIdx.x + 256 * i, r = t / PR, k = t % PR;
            if (r < h + 6) {
                constexpr int N = 16 / (int)sizeof(P);
                const P *q = reinterpret_cast<const P *>(&pv[i]);
#pragma unroll
                for (int m = 0; m < N; m++) T[r][3 + k * N + m] = (int16_t)q[m];
            }
        }
#pragma unroll
        for (int i = 0; i < NH; i++) {
            const int t = threadIdx.x + 256 * i, r = t / 6, e = t % 6, c = e < 3 ? e : kLrSW + e;
            if (r < h + 6) T[r][c] = (int16_t)hv[i];
        }
    } else {   // a thread per tile column and sixth of the rows: the column's
        // padding() case once, then per row only the row's source; every
        // load first, then the LDS writes
        constexpr int RG = 256 / kLrTW, NR = (kLrTH + RG - 1) / RG;   // 6 row groups, 12 rows each
        const int c = threadIdx.x % kLrTW, rg = threadIdx.x / kLrTW;
        const bool hl = a.edges & DGPU_LR_HAVE_LEFT, hr = a.edges & DGPU_LR_HAVE_RIGHT;
        int cc = x0 + c;
        if (!hr && cc >= a.w + 3) cc = a.w + 2;   // :110-118
        if (!hl && cc < 3) cc = 3;                // :120-126
        const int x = cc - 3;
        const bool lft = x < 0 && a.left;
        const bool col_ok = rg < RG && c < sw + 6;
        const bool ht = a.edges & DGPU_LR_HAVE_TOP, hb = a.edges & DGPU_LR_HAVE_BOTTOM;
        int tv[NR];
#pragma unroll
        for (int i = 0; i < NR; i++) {
            const int r = rg + RG * i;
            const int j = min(max(r - 3, 0), h - 1);
            const P *p = lft ? a.left + j * 4 + x + 4 : a.src + (ptrdiff_t)j * a.ss + x;
            if (r < 3 && ht) p = a.top + (r == 2) * a.ts + x;
            if (r >= h + 3 && hb) p = a.bot + (r > h + 3) * a.bs + x;
            tv[i] = col_ok && r < h + 6 ? (int)*p : 0;
        }
#pragma unroll
        for (int i = 0; i < NR; i++) {
            const int r = rg + RG * i;
            if (col_ok && r < h + 6) T[r][c] = (int16_t)tv[i];
        }
    }
    __syncthreads();
    constexpr int NP = (64 * kLrSW + 255) / 256;
    // the weighting's / Wiener vertical pass's thread layout: column wi,
    // rows wj0 .. wj0 + wrpt - 1
    const int wi = threadIdx.x & (kLrSW - 1), wrpt = (h + 7) >> 3, wj0 = (threadIdx.x >> 5) * wrpt;
    static_assert(kLrSW == 32, "8 row groups of 32 columns");
    if (a.kind == 0) {   // wiener_c, :157-189
        const int bd = bd8 + 8;
        const int rbh = 3 + (bd == 12) * 2, clip_limit = 1 << (bd + 1 + 7 - rbh);
        // horizontal: a thread per (row, 8 columns), its 14 tile values read once
        for (int k = threadIdx.x; k < (h + 6) * 4; k += 256) {
            const int r = k >> 2, i0 = (k & 3) * 8;
            if (i0 >= sw) continue;
            int tv[14];
#pragma unroll
            for (int t = 0; t < 14; t++) tv[t] = T[r][i0 + t];
#pragma unroll
            for (int t = 0; t < 8; t++) {
                int sum = 1 << (bd + 6);
                if (BPC == 8) sum += tv[t + 3] * 128;
#pragma unroll
                for (int q = 0; q < 7; q++) sum += tv[t + q] * a.prm.filter[0][q];
                if (i0 + t < sw) HOR[r][i0 + t] = (int16_t)clampi((sum + (1 << (rbh - 1))) >> rbh, 0, clip_limit - 1);   // < 2^15
            }
        }
        __syncthreads();
        // vertical: a thread slides down its column, each row read once
        const int rbv = 11 - (bd == 12) * 2, round_offset = 1 << (bd + (rbv - 1));
        if (wj0 < h && wi < sw) {
            int hv[7];
#pragma unroll
            for (int t = 0; t < 6; t++) hv[t] = HOR[wj0 + t][wi];
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const int j = wj0 + r;
                if (r >= wrpt || j >= h) break;
                hv[6] = HOR[j + 6][wi];
                int sum = -round_offset;
#pragma unroll
                for (int t = 0; t < 7; t++) sum += hv[t] * a.prm.filter[1][t];
                const P o = (P)clampi((sum + (1 << (rbv - 1))) >> rbv, 0, bdmax);
                a.dst[(size_t)j * a.ds + x0 + wi] = o;
#pragma unroll
                for (int t = 0; t < 6; t++) hv[t] = hv[t + 1];
            }
        }
        return;
    }
    // ---- self-guided (selfguided_filter, :349-440), both radii in one pass ----
    // A / B: a thread per A / B column ii (unit column ii - 1) and run of
    // rows, sliding down the tile: per new tile row the 5- and 3-wide
    // horizontal sums and sums of squares (the 3-wide ones are the middle of
    // the 5-wide window), kept for the last five rows in registers, give the
    // 5x5 box (rows jj .. jj + 4) and the 3x3 box (jj + 1 .. jj + 3) around
    // unit row jj - 1 -- the reference's boxsum5 / boxsum3 (:211-347) at
    // every position its A / B loop reads, with no vertical-sum array and no
    // barrier between the radii.  5x5 A / B exist on every other row from -1
    // (:375), stored at jj / 2.
    const bool do5 = a.kind != 2, do3 = a.kind != 1;
    {
        constexpr int NCOL = kLrSW + 2, NCH = 256 / NCOL, CH = (kLrVH + NCH - 1) / NCH;   // 34 columns, 7 runs of 10 rows
        const int t = threadIdx.x, ii = t % NCOL, ck = t / NCOL;
        const int nrow = h + 2, jj0 = ck * CH, jj1 = min(jj0 + CH, nrow);
        if (ck < NCH && ii < sw + 2 && jj0 < jj1) {
            const int c = ii + 2;   // tile column of unit column ii - 1
            int h5[5], q5[5], h3[5], q3[5];
            auto hrow = [&](int r, int &s5, int &sq5, int &s3, int &sq3) {
                const int p0 = T[r][c - 2], p1 = T[r][c - 1], p2 = T[r][c], p3 = T[r][c + 1], p4 = T[r][c + 2];
                s3 = p1 + p2 + p3;
                sq3 = p1 * p1 + p2 * p2 + p3 * p3;
                s5 = s3 + p0 + p4;
                sq5 = sq3 + p0 * p0 + p4 * p4;
            };
            // the window of unit row jj0 - 1: tile rows jj0 .. jj0 + 3 now, jj0 + 4 in the loop
#pragma unroll
            for (int k = 0; k < 4; k++) hrow(jj0 + k, h5[k + 1], q5[k + 1], h3[k + 1], q3[k + 1]);
            const unsigned s0 = a.prm.sgr.s0, s1 = a.prm.sgr.s1;
#pragma unroll 2
            for (int jj = jj0; jj < jj1; jj++) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    h5[k] = h5[k + 1], q5[k] = q5[k + 1], h3[k] = h3[k + 1], q3[k] = q3[k + 1];
                }
                hrow(jj + 4, h5[4], q5[4], h3[4], q3[4]);
                if (do3) {   // n = 9: rows jj + 1 .. jj + 3 of the window
                    const int sum = h3[1] + h3[2] + h3[3], sumsq = q3[1] + q3[2] + q3[3];
                    int A, B;
                    lr_ab_sums<9>(sum, sumsq, s1, bd8, XBX, A, B);
                    AA[jj][ii] = (AT)A;
                    BB[jj][ii] = (uint8_t)B;
                }
                if (do5 && !(jj & 1)) {   // n = 25: rows jj .. jj + 4
                    const int sum = h5[0] + h5[1] + h5[2] + h5[3] + h5[4];
                    const int sumsq = q5[0] + q5[1] + q5[2] + q5[3] + q5[4];
                    int A, B;
                    lr_ab_sums<25>(sum, sumsq, s0, bd8, XBX, A, B);
                    AA5[jj >> 1][ii] = (AT)A;
                    BB5[jj >> 1][ii] = (uint8_t)B;
                }
            }
        }
    }
    __syncthreads();
    // the weighting (:397-439), both radii, a thread per column and run of
    // rows sliding down it: each A / B row is read once per thread as a
    // (sum over columns ii-1..ii+1, centre) pair, from which the 6/5 and 4/3
    // neighbour weights follow:
    //   EIGHT: 4 s1 + 3 (s0 + s2) + c0 + c2;  SIX (even j): 5 (s0 + s2) +
    //   c0 + c2;  odd j: 5 s1 + c1  (rows 0/1/2 = unit rows j-1, j, j+1)
    int v[8];
#pragma unroll
    for (int m = 0; m < 8; m++) v[m] = 0;
    if (wj0 < h && wi < sw) {
        const int ii = wi + 1;
        auto row = [&](const AT *ar, const uint8_t *br, int &sa, int &ca, int &sb, int &cb) {
            const int a0 = ar[ii - 1], a1 = ar[ii], a2 = ar[ii + 1];
            const int b0 = br[ii - 1], b1 = br[ii], b2 = br[ii + 1];
            sa = a0 + a1 + a2;
            ca = a1;
            sb = b0 + b1 + b2;
            cb = b1;
        };
        if (do5) {   // 5x5: A / B rows at unit rows -1, 1, 3, .. (jj even, stored at jj / 2)
            const int w0 = a.prm.sgr.w0;
            // unit row j reads jj = j (even j: rows j - 1 and j + 1 are jj = j, j + 2) or jj = j + 1 (odd j)
            // held: A / B row jj = wj0 (wj0 even: its row j - 1) or wj0 + 1 (odd: its only row)
            int sA = 0, cA = 0, sB = 0, cB = 0;
            row(AA5[(wj0 + 1) >> 1], BB5[(wj0 + 1) >> 1], sA, cA, sB, cB);
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const int j = wj0 + r;
                if (r >= wrpt || j >= h) break;
                int aa, bb, sh;
                if (!(j & 1)) {   // rows jj = j (held) and j + 2
                    int s2a, c2a, s2b, c2b;
                    row(AA5[(j >> 1) + 1], BB5[(j >> 1) + 1], s2a, c2a, s2b, c2b);
                    aa = 5 * (sB + s2b) + cB + c2b;
                    bb = 5 * (sA + s2a) + cA + c2a;
                    sh = 9;
                    sA = s2a, cA = c2a, sB = s2b, cB = c2b;   // row j + 2 == jj of j + 1
                } else {          // row jj = j + 1 (held)
                    aa = 5 * sB + cB;
                    bb = 5 * sA + cA;
                    sh = 8;
                }
                const int px = T[j + 3][wi + 3];
                v[r] += w0 * (int)(C)((bb - aa * px + (1 << (sh - 1))) >> sh);   // stored as coef
            }
        }
        if (do3) {   // 3x3: A / B on every row, jj = j .. j + 2
            const int w1 = a.prm.sgr.w1;
            int s0a, c0a, s0b, c0b, s1a, c1a, s1b, c1b;
            row(AA[wj0], BB[wj0], s0a, c0a, s0b, c0b);
            row(AA[wj0 + 1], BB[wj0 + 1], s1a, c1a, s1b, c1b);
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const int j = wj0 + r;
                if (r >= wrpt || j >= h) break;
                int s2a, c2a, s2b, c2b;
                row(AA[j + 2], BB[j + 2], s2a, c2a, s2b, c2b);
                const int aa = 4 * s1b + 3 * (s0b + s2b) + c0b + c2b;
                const int bb = 4 * s1a + 3 * (s0a + s2a) + c0a + c2a;
                const int px = T[j + 3][wi + 3];
                v[r] += w1 * (int)(C)((bb - aa * px + (1 << 8)) >> 9);
                s0a = s1a, c0a = c1a, s0b = s1b, c0b = c1b;
                s1a = s2a, c1a = c2a, s1b = s2b, c1b = c2b;
            }
        }
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const int j = wj0 + r;
            if (r >= wrpt || j >= h) break;
            v[r] = clampi(T[j + 3][wi + 3] + ((v[r] + (1 << 10)) >> 11), 0, bdmax);
            a.dst[(size_t)j * a.ds + x0 + wi] = (P)v[r];
        }
    }
}

template <int BPC>
__global__ __launch_bounds__(256) void k_lr(LrArgs<BPC> a) {
    lr_strip<BPC>(a, blockIdx.x * kLrSW);
}

// ---- frame tier ------------------------------------------------------------
template <int BPC> struct LrFrameArgs {
    using P = typename Px<BPC>::pixel;
    const P *in[3];
    const P *lpf[3];
    P *out[3];
    const Dav1dGpuLrUnit *units[3];
    int is[3], ls[3], os[3], w[3], h[3], rows[3], cols[3], log2[3], restore[3], ss_ver[3];
    int xb0, xb01;   // strip blocks of plane 0, of planes 0 + 1 (the grid has no empty chroma columns)
    int sb128, bdmax;
    int vec;         // every plane pointer and pitch 16-byte aligned
    int k0;          // the first stripe run (row ranges): stripe = k0 + the grid row
    int nx, nwg;     // strips per stripe (all planes), workgroups (nx x stripes)
};

// lr_stripe's filter parameters (src/lr_apply_tmpl.c:51-80); kind 0 wiener,
// 1 sgr 5x5, 2 3x3, 3 mix
__device__ __forceinline__ int lr_params(const Dav1dGpuLrUnit &u, bool hbd, Dav1dGpuLrParams &prm) {
    if (u.type == 2) {
        for (int d = 0; d < 2; d++) {
            const int8_t *f = d ? u.filter_v : u.filter_h;
            prm.filter[d][0] = prm.filter[d][6] = f[0];
            prm.filter[d][1] = prm.filter[d][5] = f[1];
            prm.filter[d][2] = prm.filter[d][4] = f[2];
            prm.filter[d][3] = (int16_t)((d ? 128 : 0) - (f[0] + f[1] + f[2]) * 2 + (!d && hbd ? 128 : 0));
            prm.filter[d][7] = 0;
        }
        return 0;
    }
    const int s0 = dspt_sgr_params[(u.type - 3) * 2], s1 = dspt_sgr_params[(u.type - 3) * 2 + 1];
    prm.sgr.s0 = (uint32_t)s0;
    prm.sgr.s1 = (uint32_t)s1;
    prm.sgr.w0 = u.sgr_weights[0];
    prm.sgr.w1 = (int16_t)(128 - (u.sgr_weights[0] + u.sgr_weights[1]));
    return !!s0 + !!s1 * 2;
}

// One (plane, stripe, 32-column strip): stripes are 64 rows (the first 8
// luma rows shorter, :45-46), units unit_size columns (the last takes the
// rest, :135-166) and a superblock row's unit row is chosen as lr_sbrow does
// (:124-127).
template <int BPC>
__global__ __launch_bounds__(256, 5) void k_lr_frame(LrFrameArgs<BPC> f) {
    using P = typename Px<BPC>::pixel;
    // Workgroup order (the frame read 3.0x its picture): the
    // hardware deals workgroups round-robin over the 8 XCDs, which put the
    // 4-5 strips sharing a 128-B line of 8-bit pixels (32 px, plus the 3 + 3
    // halo columns) on different XCDs, each fetching the line.  Runs of
    // kLrGroup consecutive strips go to one XCD instead: FETCH 36.9 -> 12.0
    // MB per 4K frame.  The time hardly moves with the order (every order
    // within 45.6-48.9 us on one box; an XCD-contiguous run of whole stripes
    // 6.8 MB but slower on another; profiles/r6/r6c_lr_order_ab.json)
    const int b = (int)blockIdx.x, i8 = b >> 3, x8 = b & 7;
    const int lb = ((i8 / kLrGroup) * 8 + x8) * kLrGroup + i8 % kLrGroup;
    if (lb >= f.nwg) return;
    const int by = lb / f.nx, bx = lb - by * f.nx, pl = bx < f.xb0 ? 0 : bx < f.xb01 ? 1 : 2;
    const int w = f.w[pl], h = f.h[pl], sv = f.ss_ver[pl];
    const int xs = (bx - (pl == 0 ? 0 : pl == 1 ? f.xb0 : f.xb01)) * kLrSW;
    if (xs >= w) return;
    const int S64 = 64 >> sv, S8 = 8 >> sv, k = f.k0 + by;
    const int y0 = k ? k * S64 - S8 : 0, y1 = min((k + 1) * S64 - S8, h);
    if (y0 >= h) return;
    const int us = 1 << f.log2[pl];
    const int ucol = min(xs >> f.log2[pl], f.cols[pl] - 1);
    const int ux0 = ucol * us, ux1 = ucol == f.cols[pl] - 1 ? w : ux0 + us;
    const int sby = k >> f.sb128;   // the superblock row of this stripe
    const int row_y = sby * (S64 << f.sb128);
    int aligned = row_y & ~(us - 1);
    if (aligned && aligned + (us >> 1) > h) aligned -= us;
    const int urow = min(aligned >> f.log2[pl], f.rows[pl] - 1);
    const Dav1dGpuLrUnit &u = f.units[pl][(size_t)urow * f.cols[pl] + ucol];
    const P *src = f.in[pl] + (size_t)y0 * f.is[pl];
    P *dst = f.out[pl] + (size_t)y0 * f.os[pl];
    if (!f.restore[pl] || u.type == 0) {   // copied
        const int sw = min(kLrSW, w - xs), n = (y1 - y0) * kLrSW;   // <= 64 rows x 32
        if (f.vec && sw == kLrSW) {   // 16-byte pieces, loads first
            constexpr int N = 16 / (int)sizeof(P), PR = kLrSW / N, NV = (64 * PR + 255) / 256;
            const int nv = (y1 - y0) * PR;
            uint4 cv[NV];
#pragma unroll
            for (int m = 0; m < NV; m++) {
                const int t = threadIdx.x + 256 * m;
                if (t < nv) cv[m] = *reinterpret_cast<const uint4 *>(src + (size_t)(t / PR) * f.is[pl] + xs + (t % PR) * N);
            }
#pragma unroll
            for (int m = 0; m < NV; m++) {
                const int t = threadIdx.x + 256 * m;
                if (t < nv) *reinterpret_cast<uint4 *>(dst + (size_t)(t / PR) * f.os[pl] + xs + (t % PR) * N) = cv[m];
            }
            return;
        }
        constexpr int NC = (64 * kLrSW + 255) / 256;
        P cv[NC];
#pragma unroll
        for (int m = 0; m < NC; m++) {   // loads first, then the stores
            const int t = threadIdx.x + 256 * m, j = t / kLrSW, i = t % kLrSW;
            if (t < n && i < sw) cv[m] = src[(size_t)j * f.is[pl] + xs + i];
        }
#pragma unroll
        for (int m = 0; m < NC; m++) {
            const int t = threadIdx.x + 256 * m, j = t / kLrSW, i = t % kLrSW;
            if (t < n && i < sw) dst[(size_t)j * f.os[pl] + xs + i] = cv[m];
        }
        return;
    }
    LrArgs<BPC> a;
    a.src = src + ux0;
    a.ss = f.is[pl];
    a.dst = dst + ux0;
    a.ds = f.os[pl];
    a.left = nullptr;
    const bool bottom = y1 < h;
    a.edges = (y0 > 0 ? DGPU_LR_HAVE_TOP : 0) | (bottom ? DGPU_LR_HAVE_BOTTOM : 0) |
              (ux0 > 0 ? DGPU_LR_HAVE_LEFT : 0) | (ux1 < w ? DGPU_LR_HAVE_RIGHT : 0);
    // lr_lpf_line (dav1d_copy_lpf's backup_lpf, lf_apply_tmpl.c:40-100):
    // rows y0 - 2, y0 - 1 above and y1, y1 + 1 below (y1 again past the plane)
    a.top = y0 > 0 ? f.lpf[pl] + (size_t)(y0 - 2) * f.ls[pl] + ux0 : nullptr;
    a.ts = f.ls[pl];
    a.bot = bottom ? f.lpf[pl] + (size_t)y1 * f.ls[pl] + ux0 : nullptr;
    a.bs = y1 + 1 < h ? f.ls[pl] : 0;
    a.w = ux1 - ux0;
    a.h = y1 - y0;
    a.bdmax = f.bdmax;
    a.vec = f.vec;
    a.kind = lr_params(u, BPC != 8, a.prm);
    lr_strip<BPC>(a, xs - ux0);
}

template <int BPC>
static int launch_lr_frame(const Dav1dGpuLrFrame *F, hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    constexpr int B = BPC / 8;
    if (!F || F->layout < 0 || F->layout > 3) return -1;
    const int np = F->layout ? 3 : 1;
    LrFrameArgs<BPC> f;
    memset(&f, 0, sizeof(f));
    int maxh = 0;
    for (int p = 0; p < np; p++) {
        if (!F->in[p].data || !F->out[p].data || F->in[p].data == F->out[p].data) return -1;
        f.restore[p] = (F->restore_planes >> p) & 1;
        if (f.restore[p] && (!F->lpf[p].data || !F->units[p] || F->unit_rows[p] <= 0 || F->unit_cols[p] <= 0))
            return -1;
        const int l2 = F->unit_size_log2[!!p];
        if (f.restore[p] && (l2 < 5 || l2 > 8)) return -1;
        f.in[p] = (const P *)F->in[p].data;
        f.lpf[p] = (const P *)F->lpf[p].data;
        f.out[p] = (P *)F->out[p].data;
        f.units[p] = F->units[p];
        f.is[p] = (int)(F->in[p].stride / B);
        f.ls[p] = (int)(F->lpf[p].stride / B);
        f.os[p] = (int)(F->out[p].stride / B);
        f.w[p] = F->in[p].w;
        f.h[p] = F->in[p].h;
        f.rows[p] = F->unit_rows[p];
        f.cols[p] = F->unit_cols[p];
        f.log2[p] = l2;
        f.ss_ver[p] = p && F->layout == 1;
        maxh = max(maxh, f.h[p]);
    }
    f.sb128 = F->sb128;
    f.bdmax = BPC == 8 ? 255 : F->bitdepth_max;
    f.vec = 1;
    for (int p = 0; p < np; p++) {
        auto al = [](const void *q, int64_t pitch) { return q && !((uintptr_t)q & 15) && !(pitch & 15); };
        f.vec &= al(F->in[p].data, F->in[p].stride) && al(F->out[p].data, F->out[p].stride) &&
                 (!f.restore[p] || al(F->lpf[p].data, F->lpf[p].stride));
    }
    int stripes = (maxh + 8 + 63) / 64 + 1;
    // a row range (luma rows, multiples of 64): stripes start / 64 .. end / 64 - 1
    const int r0 = F->row_start, r1 = F->row_end;
    if (r0 < 0 || r1 < 0 || (r0 & 63) || (r1 & 63) || (r1 && r1 <= r0)) return -1;
    f.k0 = r0 >> 6;
    // the range holding the last superblock row filters down to the picture's
    // bottom (dav1d_lr_sbrow: not_last = 0, row_h = h, src/lr_apply_tmpl.c:
    // 174-191), i.e. every stripe from k0 on, also the one starting 8 rows
    // above a 64-row multiple (h % 64 in {0, 57..63})
    const bool last = r1 && r1 >= ((f.h[0] + 63) & ~63);
    stripes = min(stripes, r1 && !last ? r1 >> 6 : stripes) - f.k0;
    if (stripes <= 0) return 0;   // (a range past the picture)
    int xb[3] = {0, 0, 0};
    for (int p = 0; p < np; p++) xb[p] = (f.w[p] + kLrSW - 1) / kLrSW;
    f.xb0 = xb[0];
    f.xb01 = xb[0] + xb[1];
    f.nx = xb[0] + xb[1] + xb[2];
    f.nwg = f.nx * stripes;
    // (a grid of whole groups per XCD, so every logical workgroup has a block)
    constexpr int per = 8 * kLrGroup;
    k_lr_frame<BPC><<<(unsigned)((f.nwg + per - 1) / per * per), 256, 0, stream>>>(f);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "dav1d-gpu: loop restoration launch failed: %s\n", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

template <int BPC>
static bool lr_t(typename Px<BPC>::pixel *p, ptrdiff_t stride, const typename Px<BPC>::pixel (*left)[4],
                 const typename Px<BPC>::pixel *lpf, int w, int h, const Dav1dGpuLrParams *params, int edges,
                 int kind, int bdmax) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    if (w <= 0 || h <= 0) return true;
    const long hl = (edges & DGPU_LR_HAVE_LEFT) ? 3 : 0, hr = (edges & DGPU_LR_HAVE_RIGHT) ? 3 : 0;
    Stager st;
    const int ip = st.in(p, stride, -hl * B, (w + hr) * B, 0, h);
    const int op = st.out(p, stride, 0, w * B, 0, h);
    const int il = hl ? st.in1(left, (long)h * 4 * B) : -1;
    const int it = (edges & DGPU_LR_HAVE_TOP) ? st.in(lpf, stride, -hl * B, (w + hr) * B, 0, 2) : -1;
    const int ib = (edges & DGPU_LR_HAVE_BOTTOM) ? st.in(lpf, stride, -hl * B, (w + hr) * B, 6, 8) : -1;
    if (!st.upload()) return false;
    LrArgs<BPC> a;
    memset(&a, 0, sizeof(a));
    a.src = st.origin<const P>(ip);
    a.ss = (int)(st.pitch(ip) / B);
    a.dst = st.origin<P>(op);
    a.ds = (int)(st.pitch(op) / B);
    a.left = il >= 0 ? st.origin<const P>(il) : nullptr;
    a.top = it >= 0 ? st.origin<const P>(it) : nullptr;
    a.ts = it >= 0 ? (int)(st.pitch(it) / B) : 0;
    a.bot = ib >= 0 ? st.origin<const P>(ib) + 6 * (st.pitch(ib) / B) : nullptr;   // row 6
    a.bs = ib >= 0 ? (int)(st.pitch(ib) / B) : 0;
    a.w = w;
    a.h = h;
    a.edges = edges;
    a.kind = kind;
    a.bdmax = bdmax;
    a.prm = *params;
    k_lr<BPC><<<(w + kLrSW - 1) / kLrSW, 256, 0, st.stream()>>>(a);
    return st.finish();
}

// The caller's entries before dav1d_loop_restoration_dsp_init_gpu_*
// overwrote them (run when the GPU path fails: runtime.hpp's error
// contract).  KIND 0 serves both Wiener slots: the 7-tap entry wiener[0]
// handles any Wiener filter, so it is the fallback for both.
static Dav1dLoopRestorationDSPContext_8bpc g_fb8;
static Dav1dLoopRestorationDSPContext_16bpc g_fb16[2];   // 10 bit, 12 bit (fb16_slot)
#define LR_FB8 g_fb8
#define LR_FB16 g_fb16[fb16_slot_bdmax(bitdepth_max)]

#define LR_ENTRIES(BPC, P, BDP, BDV)                                                                      \
template <int KIND>                                                                                       \
static void lr_##BPC(P *d, ptrdiff_t s, const P (*l)[4], const P *lpf, int w, int h,                      \
                     const Dav1dGpuLrParams *prm, int edges BDP)                                          \
{ DGPU_OR_FALLBACK((lr_t<BPC>(d, s, l, lpf, w, h, prm, edges, KIND, BDV)),                               \
                   KIND == 0 ? LR_FB##BPC.wiener[0] : LR_FB##BPC.sgr[KIND ? KIND - 1 : 0], d, s, l, lpf,  \
                   w, h, prm, edges BDV##_ARG); }

#define BD8_PARAM
#define BD8_VAL 255
#define BD8_VAL_ARG
#define BD16_PARAM , int bitdepth_max
#define BD16_VAL bitdepth_max
#define BD16_VAL_ARG , bitdepth_max
LR_ENTRIES(8, uint8_t, BD8_PARAM, BD8_VAL)
LR_ENTRIES(16, uint16_t, BD16_PARAM, BD16_VAL)

#define FILL_LR(BPC, c)                                      \
    do {                                                     \
        c->wiener[0] = c->wiener[1] = lr_##BPC<0>;           \
        c->sgr[0] = lr_##BPC<1>;                             \
        c->sgr[1] = lr_##BPC<2>;                             \
        c->sgr[2] = lr_##BPC<3>;                             \
    } while (0)

}  // namespace dgpu

using namespace dgpu;

// bitfn(dav1d_loop_restoration_dsp_init) replacement, src/looprestoration_tmpl.c:539-558
// The _gpu_ hooks keep the caller's previous entries as fallbacks.
extern "C" void dav1d_loop_restoration_dsp_init_gpu_8bpc(Dav1dLoopRestorationDSPContext_8bpc *c, int bpc) {
    (void)bpc;
    Dav1dLoopRestorationDSPContext_8bpc g{}, *gp = &g;
    FILL_LR(8, gp);
    save_fallback(&g_fb8, c, gp);
    FILL_LR(8, c);
}
extern "C" void dav1d_loop_restoration_dsp_init_gpu_16bpc(Dav1dLoopRestorationDSPContext_16bpc *c, int bpc) {
    Dav1dLoopRestorationDSPContext_16bpc g{}, *gp = &g;
    FILL_LR(16, gp);
    save_fallback(&g_fb16[fb16_slot(bpc)], c, gp);
    FILL_LR(16, c);
}
extern "C" int dav1d_gpu_lr_frame_8bpc(const Dav1dGpuLrFrame *f, void *stream) {
    return launch_lr_frame<8>(f, (hipStream_t)stream);
}
extern "C" int dav1d_gpu_lr_frame_16bpc(const Dav1dGpuLrFrame *f, void *stream) {
    return launch_lr_frame<16>(f, (hipStream_t)stream);
}
extern "C" void dav1d_loop_restoration_dsp_init_8bpc(Dav1dLoopRestorationDSPContext_8bpc *c, int bpc) {
    (void)bpc;
    FILL_LR(8, c);
}
extern "C" void dav1d_loop_restoration_dsp_init_16bpc(Dav1dLoopRestorationDSPContext_16bpc *c, int bpc) {
    (void)bpc;
    FILL_LR(16, c);
}
