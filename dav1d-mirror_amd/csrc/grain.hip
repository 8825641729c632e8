// grain.hip -- film grain synthesis on the device (SURVEY 8(f) row 4;
// include/dav1d_gpu.h, Dav1dGpuFilmGrainBatch): bitfn(dav1d_apply_grain)
// (src/fg_apply_tmpl.c:222-241) for a whole picture in two launches.
//
// k_grain_prep (one 256-thread workgroup): the grain LUTs of
// generate_grain_y / generate_grain_uv (src/filmgrain_tmpl.c:51-144) and the
// scaling LUTs of generate_scaling (fg_apply_tmpl.c:41-97).
//   * The LFSR (get_random_number, :38-44) is linear over GF(2): lane l of a
//     plane's wave starts from the seed advanced l*96 steps (the constexpr
//     matrix kJump96 = M^96, applied l times) and draws its own 96 values.
//   * The auto-regressive filter reads only earlier pixels within lag 3, so
//     every pixel with the same x + 4y is independent: a wave sweeps these
//     anti-diagonals (about 350 for luma), one pixel per lane.
//   * Scaling entries are closed-form per index (the reference's running
//     sums d = 0x8000 + x * delta, and the 16 bpc in-between fill).
// k_grain_apply (one workgroup per 32x32 luma block): fgy_32x32xn /
// fguv_32x32xn (:166-420) for the block and its chroma, the block's random
// offsets recomputed from the row seeds, planes without grain copied.
// HBM-bound: each picture pixel is read once and written once (chroma
// re-reads the block's luma from L2).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <array>
#include <utility>

#include "dav1d_gpu.h"
#include "dsp_common.hpp"

namespace dgpu {

constexpr int kGW = DGPU_GRAIN_W, kGH = DGPU_GRAIN_H;
constexpr int kChunk = 96;   // LFSR values per lane (64 * 96 >= 82 * 73)

// GF(2) linear maps on the 16-bit LFSR state as 16 column images
struct Lin16 { uint16_t c[16]; };
constexpr uint16_t lin_apply(const Lin16 &m, uint16_t v) {
    uint16_t r = 0;
    for (int i = 0; i < 16; i++)
        if ((v >> i) & 1) r ^= m.c[i];
    return r;
}
constexpr Lin16 lin_step() {   // one get_random_number step
    Lin16 m{};
    for (int i = 0; i < 16; i++) {
        const unsigned r = 1u << i;
        const unsigned bit = (r ^ (r >> 1) ^ (r >> 3) ^ (r >> 12)) & 1;
        m.c[i] = (uint16_t)((r >> 1) | (bit << 15));
    }
    return m;
}
constexpr Lin16 lin_compose(const Lin16 &a, const Lin16 &b) {   // a after b
    Lin16 m{};
    for (int i = 0; i < 16; i++) m.c[i] = lin_apply(a, b.c[i]);
    return m;
}
constexpr Lin16 lin_pow(Lin16 b, int e) {
    Lin16 r{};
    for (int i = 0; i < 16; i++) r.c[i] = (uint16_t)(1u << i);
    while (e) {
        if (e & 1) r = lin_compose(b, r);
        b = lin_compose(b, b);
        e >>= 1;
    }
    return r;
}
constexpr Lin16 kJump96 = lin_pow(lin_step(), kChunk);
__constant__ uint16_t c_jump96[16] = {
    kJump96.c[0], kJump96.c[1], kJump96.c[2],  kJump96.c[3],  kJump96.c[4],  kJump96.c[5],
    kJump96.c[6], kJump96.c[7], kJump96.c[8],  kJump96.c[9],  kJump96.c[10], kJump96.c[11],
    kJump96.c[12], kJump96.c[13], kJump96.c[14], kJump96.c[15]};

// M^k for k = 0..255 and M^256: a block column's offset is the draw after
// c + 1 steps of its row seed, computed without stepping
struct JumpTab { Lin16 m[257]; };
constexpr JumpTab make_jumps() {
    JumpTab t{};
    Lin16 p{};
    for (int i = 0; i < 16; i++) p.c[i] = (uint16_t)(1u << i);
    const Lin16 st = lin_step();
    for (int k = 0; k <= 256; k++) {
        t.m[k] = p;
        p = lin_compose(st, p);
    }
    return t;
}
constexpr JumpTab kJumps = make_jumps();
template <size_t... I> constexpr auto flat_jumps(std::index_sequence<I...>) {
    return std::array<uint16_t, sizeof...(I)>{kJumps.m[I / 16].c[I % 16]...};
}
__constant__ std::array<uint16_t, 257 * 16> c_jumps = flat_jumps(std::make_index_sequence<257 * 16>());

__device__ __forceinline__ unsigned jump_apply(int k, unsigned s) {
    unsigned r = 0;
#pragma unroll
    for (int b = 0; b < 16; b++) r ^= ((s >> b) & 1) ? c_jumps[k * 16 + b] : 0u;
    return r;
}

__device__ __forceinline__ int fg_rand(int bits, unsigned &s) {
    const unsigned bit = (s ^ (s >> 1) ^ (s >> 3) ^ (s >> 12)) & 1;
    s = (s >> 1) | (bit << 15);
    return (int)((s >> (16 - bits)) & ((1u << bits) - 1));
}
__device__ __forceinline__ int rnd2(int x, int sh) { return sh ? (x + (1 << (sh - 1))) >> sh : x; }
__device__ __forceinline__ int bd8_of(int bdmax) { return bdmax == 255 ? 0 : bdmax == 1023 ? 2 : 4; }

struct GrainArgs {
    Dav1dGpuFilmGrainData d;
    int layout, bdmax;
    int16_t *grain;     // [3][73][82]
    uint8_t *scaling;   // [3][4096]
};

// generate_scaling entry `idx` of a point list (fg_apply_tmpl.c:41-97)
__device__ int scaling_entry(const uint8_t (*pts)[2], int num, int shx, int idx) {
    if (!num) return 0;
    const int first = pts[0][0] << shx, last = pts[num - 1][0] << shx;
    if (idx < first) return pts[0][1];
    if (idx >= last) return pts[num - 1][1];
    auto base = [&](int xb) -> int {   // an entry at a multiple of 1 << shx
        if (xb >= last) return pts[num - 1][1];
        const int xp = xb >> shx;
        int i = 0;
        while (i < num - 2 && pts[i + 1][0] <= xp) i++;
        const int bx = pts[i][0], by = pts[i][1], dx = pts[i + 1][0] - bx, dy = pts[i + 1][1] - by;
        const int delta = dy * ((0x10000 + (dx >> 1)) / dx);
        return by + ((0x8000 + (xp - bx) * delta) >> 16);
    };
    const int pad = 1 << shx;
    const int k = idx & (pad - 1), xb = idx - k;
    const int b0 = base(xb);
    if (!k) return b0;
    const int range = base(xb + pad) - b0;
    return (b0 + (((pad >> 1) + k * range) >> shx)) & 0xff;
}

// One plane's auto-regressive filter (filmgrain_tmpl.c:70-88 / 110-142) by
// one wave: pixels with equal x + 4y are independent (lag <= 3), so the
// wave sweeps those anti-diagonals, a pixel per lane, coefficients in
// registers and the taps unrolled.
// luma_done: the last luma anti-diagonal finished (written by the luma
// wave, read by the chroma waves, which start as soon as the luma grain
// they read is final instead of after the whole luma sweep)
template <int LAG>
__device__ void ar_sweep(int16_t (*g)[kGW], const int16_t (*gy)[kGW], const int8_t *cf_, int p, int cw, int ch,
                         int sx, int sy, int num_y, int shift, int gmin, int gmax, int lane, int *luma_done) {
    constexpr int NT = LAG * (2 * LAG + 1) + LAG;   // taps before the current pixel
    int cf[NT + 1];
#pragma unroll
    for (int k = 0; k <= NT; k++) cf[k] = cf_[k];
    const bool luma_term = p && num_y;
    const int tmax = (cw - 4) + 4 * (ch - 1);
    const int tmax_l = (kGW - 4) + 4 * (kGH - 1);
    for (int t = 15; t <= tmax; t++) {
        const int ylo = max(3, (t - (cw - 4) + 3) >> 2), yhi = min(ch - 1, (t - 3) >> 2);
        if (luma_term) {   // wait for the luma grain this step reads
            auto need = [&](int yy) {   // the highest luma diagonal pixel (yy, t - 4yy) reads
                const int xx = t - 4 * yy, lx = ((xx - 3) << sx) + 3 + sx, ly = ((yy - 3) << sy) + 3 + sy;
                return lx + 4 * ly;
            };
            const int req = min(max(need(ylo), need(yhi)), tmax_l);
            if (lane == 0)
                for (int it = 0; it < (1 << 22); it++) {
                    if (__hip_atomic_load(luma_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= req) break;
                    __builtin_amdgcn_s_sleep(1);
                }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            __builtin_amdgcn_wave_barrier();
        }
        const int y = ylo + lane, x = t - 4 * y;
        if (y <= yhi && x >= 3 && x < cw - 3) {
            int sum = 0, k = 0;
#pragma unroll
            for (int dy = -LAG; dy <= 0; dy++)
#pragma unroll
                for (int dx = -LAG; dx <= LAG; dx++) {
                    if (dy == 0 && dx >= 0) continue;
                    sum += cf[k++] * g[y + dy][x + dx];
                }
            if (luma_term) {   // the co-located luma grain (:115-128)
                const int lx = ((x - 3) << sx) + 3, ly = ((y - 3) << sy) + 3;
                int l = gy[ly][lx];
                if (sx) l += gy[ly][lx + 1];
                if (sy) l += gy[ly + 1][lx] + (sx ? gy[ly + 1][lx + 1] : 0);
                sum += rnd2(l, sx + sy) * cf[NT];
            }
            const int v = g[y][x] + rnd2(sum, shift);
            g[y][x] = (int16_t)min(max(v, gmin), gmax);
        }
        if (p == 0) {   // publish the finished diagonal to the chroma waves
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) __hip_atomic_store(luma_done, t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (p == 0 && lane == 0) __hip_atomic_store(luma_done, 1 << 30, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ __launch_bounds__(256) void k_grain_prep(GrainArgs a) {
    __shared__ int16_t g[3][kGH][kGW];
    __shared__ int luma_done;
    if (threadIdx.x == 0) luma_done = 0;
    const Dav1dGpuFilmGrainData &d = a.d;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bd8 = bd8_of(a.bdmax);
    const int sx = a.layout != 3, sy = a.layout == 1;
    const int gmin = -(128 << bd8), gmax = (128 << bd8) - 1;
    const bool need[3] = {true, d.num_uv_points[0] || d.chroma_scaling_from_luma,
                          d.num_uv_points[1] || d.chroma_scaling_from_luma};
    // 1. random fill: wave p draws plane p's values, 96 per lane
    if (wave < 3) {
        const int p = wave;
        const int cw = p && sx ? 44 : kGW, ch = p && sy ? 38 : kGH;
        for (int i = lane; i < kGH * kGW; i += 64) (&g[p][0][0])[i] = 0;
        if (need[p]) {
            unsigned s = d.seed ^ (p == 0 ? 0u : p == 1 ? 0xb524u : 0x49d8u);
            for (int j = 0; j < lane; j++) {   // seed advanced lane * 96 steps
                unsigned t = 0;
                for (int b = 0; b < 16; b++)
                    if ((s >> b) & 1) t ^= c_jump96[b];
                s = t;
            }
            const int shift = 4 - bd8 + d.grain_scale_shift;
            const int n = cw * ch;
            for (int k = 0; k < kChunk; k++) {
                const int i = lane * kChunk + k;
                const int v = fg_rand(11, s);
                if (i < n) g[p][i / cw][i % cw] = (int16_t)rnd2(dspt_gaussian[v], shift);
            }
        }
    }
    __syncthreads();
    // 2. the auto-regressive filter, anti-diagonal sweeps (x + 4y)
    const int lag = d.ar_coeff_lag;
    auto ar = [&](int p) {
        const int cw = p && sx ? 44 : kGW, ch = p && sy ? 38 : kGH;
        const int8_t *cf = p == 0 ? d.ar_coeffs_y : d.ar_coeffs_uv[p - 1];
        switch (lag) {
            case 0: ar_sweep<0>(g[p], g[0], cf, p, cw, ch, sx, sy, d.num_y_points, (int)d.ar_coeff_shift, gmin, gmax, lane, &luma_done); break;
            case 1: ar_sweep<1>(g[p], g[0], cf, p, cw, ch, sx, sy, d.num_y_points, (int)d.ar_coeff_shift, gmin, gmax, lane, &luma_done); break;
            case 2: ar_sweep<2>(g[p], g[0], cf, p, cw, ch, sx, sy, d.num_y_points, (int)d.ar_coeff_shift, gmin, gmax, lane, &luma_done); break;
            default: ar_sweep<3>(g[p], g[0], cf, p, cw, ch, sx, sy, d.num_y_points, (int)d.ar_coeff_shift, gmin, gmax, lane, &luma_done); break;
        }
    };
    if (wave == 0) ar(0);   // the chroma waves follow the luma sweep's front
    else if ((wave == 1 || wave == 2) && need[wave]) ar(wave);
    __syncthreads();
    // 3. out: grain LUTs and scaling LUTs
    for (int i = threadIdx.x; i < 3 * kGH * kGW; i += 256) a.grain[i] = (&g[0][0][0])[i];
    const int bitdepth = a.bdmax == 255 ? 8 : a.bdmax == 1023 ? 10 : 12, shx = bitdepth - 8, size = 1 << bitdepth;
    for (int i = threadIdx.x; i < 3 * 4096; i += 256) {
        const int p = i >> 12, idx = i & 4095;
        int v = 0;
        if (idx < size) {
            if (p == 0 && (d.num_y_points || d.chroma_scaling_from_luma))
                v = scaling_entry(d.y_points, d.num_y_points, shx, idx);
            else if (p > 0 && d.num_uv_points[p - 1])
                v = scaling_entry(d.uv_points[p - 1], d.num_uv_points[p - 1], shx, idx);
        }
        a.scaling[i] = (uint8_t)v;
    }
}

template <int BPC> struct ApplyArgs {
    using P = typename Px<BPC>::pixel;
    const P *in[3];
    P *out[3];
    int is[3], os[3];   // strides, pixels
    int w, h, layout, bdmax, is_id;
    Dav1dGpuFilmGrainData d;
    const int16_t *grain;
    const uint8_t *scaling;
};

// the row seed's offset for block column c: the (c+1)-th 8-bit draw
// (fgy_32x32xn, filmgrain_tmpl.c:187-205), by jump-ahead
__device__ __forceinline__ int fg_offset(unsigned seed, int row, int c) {
    unsigned s = seed;
    s ^= (unsigned)((((row) * 37 + 178) & 0xFF) << 8);
    s ^= (unsigned)(((row) * 173 + 105) & 0xFF);
    int k = c + 1;
    while (k > 256) {
        s = jump_apply(256, s);
        k -= 256;
    }
    s = jump_apply(k, s);
    return (int)((s >> 8) & 0xff);
}

// One plane of one 32x32-luma block, NP pixels per thread, in two phases so
// a workgroup issues the picture loads of all three planes before its first
// barrier and the dependent work after: load() reads the pixels (and the
// co-located luma) or copies a plane without grain; finish() samples the
// grain LUT with the block's offsets and overlap blends, looks the scaling
// up in LDS, adds the noise and stores.
template <int BPC, int NP> struct PlaneJob {
    using P = typename Px<BPC>::pixel;
    int pl, ssx, ssy, bw0, bh0, lw, x0, bw, bh, is, os, c, row;
    bool grained;
    const P *src;
    P *dst;
    int sv[NP], lv[NP];

    __device__ __forceinline__ void load(const ApplyArgs<BPC> &a, int pl_, int c_, int row_) {
        const Dav1dGpuFilmGrainData &d = a.d;
        pl = pl_;
        c = c_;
        row = row_;
        const int sx = a.layout != 3, sy = a.layout == 1;
        ssx = pl ? sx : 0;
        ssy = pl ? sy : 0;
        const int pw = pl ? (a.w + sx) >> sx : a.w;
        bw0 = 32 >> ssx;
        bh0 = 32 >> ssy;
        lw = 5 - ssx;
        x0 = c * bw0;
        const int y0 = row * bh0;
        bw = min(bw0, pw - x0);
        const int lrows = min(32, a.h - row * 32);
        bh = pl ? (lrows + ssy) >> ssy : lrows;
        is = pl == 0 ? a.is[0] : pl == 1 ? a.is[1] : a.is[2];
        os = pl == 0 ? a.os[0] : pl == 1 ? a.os[1] : a.os[2];
        src = (pl == 0 ? a.in[0] : pl == 1 ? a.in[1] : a.in[2]) + (size_t)y0 * is + x0;
        dst = (pl == 0 ? a.out[0] : pl == 1 ? a.out[1] : a.out[2]) + (size_t)y0 * os + x0;
        grained = pl ? (d.chroma_scaling_from_luma || d.num_uv_points[pl - 1]) : d.num_y_points;
        const P *luma = a.in[0] + (size_t)(row * 32) * a.is[0];
#pragma unroll
        for (int k = 0; k < NP; k++) {
            const int i = threadIdx.x + 256 * k, y = i >> lw, x = i & (bw0 - 1);
            const bool ok = x < bw && y < bh;
            sv[k] = ok ? (int)src[(size_t)y * is + x] : 0;
            lv[k] = 0;
            if (pl && grained && ok) {
                const int lx = (x0 + x) << ssx, ly = y << ssy;
                int avg = luma[(size_t)ly * a.is[0] + min(lx, a.w - 1)];
                if (ssx) avg = (avg + luma[(size_t)ly * a.is[0] + min(lx + 1, a.w - 1)] + 1) >> 1;
                lv[k] = avg;
            }
            if (!grained && ok) dst[(size_t)y * os + x] = (P)sv[k];   // fg_apply_tmpl.c:132-160: copied
        }
    }

    __device__ __forceinline__ void finish(const ApplyArgs<BPC> &a, const int (&off)[2][2], const uint8_t *sc) {
        if (!grained) return;
        const Dav1dGpuFilmGrainData &d = a.d;
        const int bd8 = bd8_of(a.bdmax);
        const int gmin = -(128 << bd8), gmax = (128 << bd8) - 1;
        const int16_t *g = a.grain + pl * kGH * kGW;
        int vmin = 0, vmax = a.bdmax;
        if (d.clip_to_restricted_range) {
            vmin = 16 << bd8;
            vmax = (pl && !a.is_id ? 240 : 235) << bd8;
        }
        const int ys = d.overlap_flag && row ? min(2 >> ssy, bh) : 0;
        const int xs = d.overlap_flag && c ? min(2 >> ssx, bw) : 0;
        // LUT origins of the four (column, row) offset blocks (sample_lut, :155-164)
        int org[2][2];
#pragma unroll
        for (int bx = 0; bx < 2; bx++)
#pragma unroll
            for (int by = 0; by < 2; by++) {
                const int rv = off[bx][by];
                org[bx][by] = (3 + (2 >> ssy) * (3 + (rv & 15)) + bh0 * by) * kGW + 3 + (2 >> ssx) * (3 + (rv >> 4)) +
                              bw0 * bx;
            }
        auto wgt = [&](int ss, int i, int k) -> int { return ss ? (k ? 22 : 23) : ((i == 0) == (k == 0) ? 27 : 17); };
        auto blend = [&](int old, int cur, int w0, int w1) { return min(max(rnd2(old * w0 + cur * w1, 5), gmin), gmax); };
        int gv[NP];
#pragma unroll
        for (int k = 0; k < NP; k++) {   // grain samples (independent loads)
            const int i = threadIdx.x + 256 * k, y = i >> lw, x = i & (bw0 - 1);
            int gr = g[org[0][0] + y * kGW + x];
            if (x < xs) gr = blend(g[org[1][0] + y * kGW + x], gr, wgt(ssx, x, 0), wgt(ssx, x, 1));
            if (y < ys) {
                int top = g[org[0][1] + y * kGW + x];
                if (x < xs) top = blend(g[org[1][1] + y * kGW + x], top, wgt(ssx, x, 0), wgt(ssx, x, 1));
                gr = blend(top, gr, wgt(ssy, y, 0), wgt(ssy, y, 1));
            }
            gv[k] = gr;
        }
#pragma unroll
        for (int k = 0; k < NP; k++) {   // scaling (LDS), noise, store
            const int i = threadIdx.x + 256 * k, y = i >> lw, x = i & (bw0 - 1);
            if (x >= bw || y >= bh) continue;
            int val = sv[k];
            if (pl) {
                val = lv[k];
                if (!d.chroma_scaling_from_luma) {
                    const int comb = lv[k] * d.uv_luma_mult[pl - 1] + sv[k] * d.uv_mult[pl - 1];
                    val = min(max((comb >> 6) + d.uv_offset[pl - 1] * (1 << bd8), 0), a.bdmax);
                }
            }
            const int noise = rnd2(sc[val] * gv[k], d.scaling_shift);
            dst[(size_t)y * os + x] = (P)min(max(sv[k] + noise, vmin), vmax);
        }
    }
};

template <int BPC, int LAYOUT>
__global__ __launch_bounds__(256) void k_grain_apply(ApplyArgs<BPC> a) {
    constexpr int SC = BPC == 8 ? 256 : 4096;
    constexpr int NPC = LAYOUT == 1 ? 1 : LAYOUT == 2 ? 2 : 4;   // chroma pixels per thread
    __shared__ int off[2][2];   // [column: this, previous][row: this, previous]
    __shared__ uint8_t sc[3][SC];
    const Dav1dGpuFilmGrainData &d = a.d;
    // XCD-contiguous block order: workgroups are dealt round-robin over the
    // 8 XCDs, so logical block (b % 8) * (nb / 8) + b / 8 gives each XCD a
    // contiguous run of blocks; a 128-B picture line (4 blocks of one row)
    // is then read and written through one L2 instead of four
    const int cols = (a.w + 31) >> 5, nblk = cols * ((a.h + 31) >> 5);
    const int nb8 = (int)gridDim.x >> 3, b = blockIdx.x;
    const int lb = (b & 7) * nb8 + (b >> 3);
    if (lb >= nblk) return;
    const int c = lb % cols, row = lb / cols;
    // the picture loads of all three planes first (they need no offsets)
    PlaneJob<BPC, 4> jy;
    PlaneJob<BPC, NPC> ju, jv;
    jy.load(a, 0, c, row);
    ju.load(a, 1, c, row);
    jv.load(a, 2, c, row);
    if (threadIdx.x < 4) {
        const int bc = threadIdx.x & 1, br = threadIdx.x >> 1;
        const bool used = (!bc || (d.overlap_flag && c)) && (!br || (d.overlap_flag && row));
        off[bc][br] = used ? fg_offset(d.seed, row - br, c - bc) : 0;
    }
    for (int i = threadIdx.x * 4; i < 3 * SC; i += 1024)   // the scaling LUTs (4 KB apart in the scratch)
        *reinterpret_cast<uint32_t *>(&sc[0][0] + i) =
            *reinterpret_cast<const uint32_t *>(a.scaling + (i / SC) * 4096 + (i % SC));
    __syncthreads();
    int o[2][2] = {{off[0][0], off[0][1]}, {off[1][0], off[1][1]}};
    jy.finish(a, o, sc[0]);
    ju.finish(a, o, d.chroma_scaling_from_luma ? sc[0] : sc[1]);
    jv.finish(a, o, d.chroma_scaling_from_luma ? sc[0] : sc[2]);
}

template <int BPC>
static int launch_grain(const Dav1dGpuFilmGrainBatch *b, hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    constexpr int B = BPC / 8;
    if (!b || b->layout < 1 || b->layout > 3 || !b->scratch) return -1;
    for (int p = 0; p < 3; p++)
        if (!b->in[p].data || !b->out[p].data) return -1;
    const int w = b->in[0].w, h = b->in[0].h;
    if (w <= 0 || h <= 0) return -1;
    GrainArgs g;
    memset(&g, 0, sizeof(g));
    g.d = b->data;
    g.layout = b->layout;
    g.bdmax = BPC == 8 ? 255 : b->bitdepth_max;
    g.grain = (int16_t *)b->scratch;
    g.scaling = (uint8_t *)b->scratch + 3 * kGH * kGW * 2;
    if (g.d.ar_coeff_lag < 0 || g.d.ar_coeff_lag > 3 || g.d.num_y_points > 14 || g.d.num_uv_points[0] > 10 ||
        g.d.num_uv_points[1] > 10)
        return -1;
    k_grain_prep<<<1, 256, 0, stream>>>(g);
    ApplyArgs<BPC> a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) {
        a.in[p] = (const P *)b->in[p].data;
        a.out[p] = (P *)b->out[p].data;
        a.is[p] = (int)(b->in[p].stride / B);
        a.os[p] = (int)(b->out[p].stride / B);
    }
    a.w = w;
    a.h = h;
    a.layout = b->layout;
    a.bdmax = g.bdmax;
    a.is_id = b->is_id;
    a.d = b->data;
    a.grain = g.grain;
    a.scaling = g.scaling;
    const int nblk = ((w + 31) / 32) * ((h + 31) / 32);
    const dim3 grid((unsigned)((nblk + 7) & ~7));
    if (b->layout == 1) k_grain_apply<BPC, 1><<<grid, 256, 0, stream>>>(a);
    else if (b->layout == 2) k_grain_apply<BPC, 2><<<grid, 256, 0, stream>>>(a);
    else k_grain_apply<BPC, 3><<<grid, 256, 0, stream>>>(a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "dav1d-gpu: film grain launch failed: %s\n", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

}  // namespace dgpu

extern "C" int dav1d_gpu_apply_grain_8bpc(const Dav1dGpuFilmGrainBatch *b, void *stream) {
    return dgpu::launch_grain<8>(b, (hipStream_t)stream);
}
extern "C" int dav1d_gpu_apply_grain_16bpc(const Dav1dGpuFilmGrainBatch *b, void *stream) {
    return dgpu::launch_grain<16>(b, (hipStream_t)stream);
}
