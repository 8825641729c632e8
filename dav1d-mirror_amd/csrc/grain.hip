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

__global__ __launch_bounds__(256) void k_grain_prep(GrainArgs a) {
    __shared__ int16_t g[3][kGH][kGW];
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
        const int tmax = (cw - 4) + 4 * (ch - 1);
        for (int t = 3 + 12; t <= tmax; t++) {
            // pixel y = 3 + lane + y0 with x = t - 4y in [3, cw - 3)
            const int ylo = max(3, (t - (cw - 4) + 3) / 4), yhi = min(ch - 1, (t - 3) / 4);
            for (int y = ylo + lane; y <= yhi; y += 64) {
                const int x = t - 4 * y;
                if (x < 3 || x >= cw - 3) continue;
                int sum = 0, k = 0;
                for (int dy = -lag; dy <= 0; dy++)
                    for (int dx = -lag; dx <= lag; dx++) {
                        if (!dx && !dy) {
                            if (p && d.num_y_points) {
                                const int lx = ((x - 3) << sx) + 3, ly = ((y - 3) << sy) + 3;
                                int l = 0;
                                for (int i = 0; i <= sy; i++)
                                    for (int j = 0; j <= sx; j++) l += g[0][ly + i][lx + j];
                                sum += rnd2(l, sx + sy) * cf[k];
                            }
                            dy = 1;   // leave both loops
                            break;
                        }
                        sum += cf[k++] * g[p][y + dy][x + dx];
                    }
                const int v = g[p][y][x] + rnd2(sum, (int)d.ar_coeff_shift);
                g[p][y][x] = (int16_t)min(max(v, gmin), gmax);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    };
    if (wave == 0) ar(0);
    __syncthreads();
    if ((wave == 1 || wave == 2) && need[wave]) ar(wave);
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

// the row seeds' offsets for block column c (the c+1-th 8-bit draw)
__device__ __forceinline__ int fg_offset(const Dav1dGpuFilmGrainData &d, int row, int c) {
    unsigned s = d.seed;
    s ^= (unsigned)((((row) * 37 + 178) & 0xFF) << 8);
    s ^= (unsigned)(((row) * 173 + 105) & 0xFF);
    int v = 0;
    for (int i = 0; i <= c; i++) v = fg_rand(8, s);
    return v;
}

template <int BPC>
__global__ __launch_bounds__(256) void k_grain_apply(ApplyArgs<BPC> a) {
    using P = typename Px<BPC>::pixel;
    const Dav1dGpuFilmGrainData &d = a.d;
    const int c = blockIdx.x, row = blockIdx.y;
    __shared__ int off[2][2];   // [column: this, previous][row: this, previous]
    if (threadIdx.x < 4) {
        const int bc = threadIdx.x & 1, br = threadIdx.x >> 1;
        const bool used = (!bc || (d.overlap_flag && c)) && (!br || (d.overlap_flag && row));
        off[bc][br] = used ? fg_offset(d, row - br, c - bc) : 0;
    }
    __syncthreads();
    const int bd8 = bd8_of(a.bdmax);
    const int gmin = -(128 << bd8), gmax = (128 << bd8) - 1;
    const int sx = a.layout != 3, sy = a.layout == 1;
    for (int pl = 0; pl < 3; pl++) {
        const int ssx = pl ? sx : 0, ssy = pl ? sy : 0;
        const int pw = pl ? (a.w + sx) >> sx : a.w, ph = pl ? (a.h + sy) >> sy : a.h;
        const int bw0 = 32 >> ssx, bh0 = 32 >> ssy;
        const int x0 = c * bw0, y0 = row * bh0;
        const int bw = min(bw0, pw - x0);
        // the strip's rows: luma min(32, h - 32 row), chroma (that + ssy) >> ssy
        const int lrows = min(32, a.h - row * 32);
        const int bh = pl ? (lrows + ssy) >> ssy : lrows;
        if (bw <= 0 || bh <= 0) continue;
        const P *src = a.in[pl] + (size_t)y0 * a.is[pl] + x0;
        P *dst = a.out[pl] + (size_t)y0 * a.os[pl] + x0;
        const bool grained = pl ? (d.chroma_scaling_from_luma || d.num_uv_points[pl - 1]) : d.num_y_points;
        if (!grained) {   // fg_apply_tmpl.c:132-160: the plane is copied
            for (int i = threadIdx.x; i < bw * bh; i += 256) {
                const int y = i / bw, x = i % bw;
                dst[(size_t)y * a.os[pl] + x] = src[(size_t)y * a.is[pl] + x];
            }
            continue;
        }
        const int16_t *g = a.grain + pl * kGH * kGW;
        const uint8_t *sc = a.scaling + (pl && !d.chroma_scaling_from_luma ? pl : 0) * 4096;
        int vmin = 0, vmax = a.bdmax;
        if (d.clip_to_restricted_range) {
            vmin = 16 << bd8;
            vmax = (pl && !a.is_id ? 240 : 235) << bd8;
        }
        const int ys = d.overlap_flag && row ? min(2 >> ssy, bh) : 0;
        const int xs = d.overlap_flag && c ? min(2 >> ssx, bw) : 0;
        // overlap weights: luma {27,17},{17,27}; chroma subsampled {23,22}
        auto wgt = [&](int ss, int i, int k) -> int {
            return ss ? (k ? 22 : 23) : ((i == 0) == (k == 0) ? 27 : 17);
        };
        auto sample = [&](int bx, int by, int x, int y) -> int {
            const int rv = off[bx][by];
            const int ox = 3 + (2 >> ssx) * (3 + (rv >> 4)), oy = 3 + (2 >> ssy) * (3 + (rv & 15));
            return g[(oy + y + bh0 * by) * kGW + ox + x + bw0 * bx];
        };
        auto blend = [&](int old, int cur, int w0, int w1) {
            return min(max(rnd2(old * w0 + cur * w1, 5), gmin), gmax);
        };
        const P *luma = a.in[0] + (size_t)(row * 32) * a.is[0];
        for (int i = threadIdx.x; i < bw * bh; i += 256) {
            const int y = i / bw, x = i % bw;
            int gr = sample(0, 0, x, y);
            if (x < xs) gr = blend(sample(1, 0, x, y), gr, wgt(ssx, x, 0), wgt(ssx, x, 1));
            if (y < ys) {
                int top = sample(0, 1, x, y);
                if (x < xs) top = blend(sample(1, 1, x, y), top, wgt(ssx, x, 0), wgt(ssx, x, 1));
                gr = blend(top, gr, wgt(ssy, y, 0), wgt(ssy, y, 1));
            }
            const int s = src[(size_t)y * a.is[pl] + x];
            int val = s;
            if (pl) {
                const int lx = (x0 + x) << ssx, ly = y << ssy;
                int avg = luma[(size_t)ly * a.is[0] + min(lx, a.w - 1)];
                if (ssx) avg = (avg + luma[(size_t)ly * a.is[0] + min(lx + 1, a.w - 1)] + 1) >> 1;
                val = avg;
                if (!d.chroma_scaling_from_luma) {
                    const int comb = avg * d.uv_luma_mult[pl - 1] + s * d.uv_mult[pl - 1];
                    val = min(max((comb >> 6) + d.uv_offset[pl - 1] * (1 << bd8), 0), a.bdmax);
                }
            }
            const int noise = rnd2(sc[val] * gr, d.scaling_shift);
            dst[(size_t)y * a.os[pl] + x] = (P)min(max(s + noise, vmin), vmax);
        }
    }
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
    k_grain_apply<BPC><<<dim3((w + 31) / 32, (h + 31) / 32), 256, 0, stream>>>(a);
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
