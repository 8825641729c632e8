// cdef.hip -- CDEF on the device (the first post-filter;
// include/dav1d_gpu.h, Dav1dCdefDSPContext and Dav1dGpuCdefFrame).
//
// Frame tier, k_cdef: bytefn(dav1d_cdef_brow) (src/cdef_apply_tmpl.c:97-309)
// over a whole deblocked frame in one launch.  The reference filters in
// place and keeps the pre-filter neighbours its blocks still need in
// cdef_line (two rows per block row, :41-63, :132-139) and lr_bak (two
// columns per block, :65-89, :190-200), so every block reads deblocked,
// pre-CDEF pixels only; the device reads `in` and writes `out` instead.
//   * One 256-thread workgroup per 64x64 luma superblock (the cdef_idx unit,
//     :149): the superblock's pixels and a 2-px ring (4 px left / right, for
//     aligned loads) are staged into LDS as int16, INT16_MIN outside the
//     frame's 8x8 grid (what padding() fills where CDEF_HAVE_* is clear,
//     src/cdef_tmpl.c:44-102).
//   * cdef_find_dir (src/cdef_tmpl.c:238-304) per 8x8 block: wave q computes
//     the costs of directions 2q and 2q+1 for the 64 blocks, one block per
//     lane, the block's 64 pixels held in registers with fully unrolled
//     partial sums; every filter task takes the argmax from LDS.
//   * The filter (cdef_filter_block_c, :104-215): one task per block row, the
//     12 taps read from LDS at the block's direction offsets, thresholds of 0
//     standing for the reference's pri-only / sec-only paths (constrain() is
//     then 0), the min / max clip applied only when both strengths are set.
//   * Blocks the reference skips (cdef_idx -1 or both strengths 0, no coded
//     coefficients, :150-156, :185-189, an adjusted luma strength of 0 with
//     no secondary strength, :237-246) are copied from the staged pixels.
// The kernel is HBM-bound in principle (each pixel read once, written once);
// the filter is ~100 VALU per pixel and 12 LDS reads, see DESIGN.md.
//
// Per-call tier: the Dav1dCdefDSPContext entries (dir, fb[3]) through the
// per-call Stager, one small workgroup per call, the same device filter.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>

#include "dav1d_gpu.h"
#include "dsp_common.hpp"
#include "runtime.hpp"

namespace dgpu {

// Marker for pixels outside the frame's 8x8 grid.  The reference uses
// INT16_MIN (padding(), src/cdef_tmpl.c:44-54); any value whose distance
// from every pixel is at least 2^14 behaves the same (constrain() returns 0
// for it at every strength / damping the format allows: thr << shift < 2^9;
// it never wins the unsigned min or the signed max), and -16384 keeps every
// difference inside int16 for the packed filter below.
constexpr int kNone = -16384;

// (dy, dx) of a direction's two taps: the AV1 CDEF direction set
// (dav1d_cdef_directions, src/tables.c:400-413, as offsets in a 12-wide
// buffer with cyclic padding for dir +- 2).  Held as nibbles (value + 2,
// direction d in bits 4d..4d+3) so a lane-varying direction costs shifts,
// not a memory load:
//   k = 0: dy -1 0 0 0 1 1 1 1, dx 1 1 1 1 1 0 0 0
//   k = 1: dy -2 -1 0 1 2 2 2 2, dx 2 2 2 2 2 1 0 -1
constexpr uint32_t kDy0 = 0x33332221u, kDx0 = 0x22233333u, kDy1 = 0x44443210u, kDx1 = 0x12344444u;
__device__ __forceinline__ int dir_nib(uint32_t c, int d) { return (int)((c >> (4 * d)) & 15) - 2; }
__device__ __forceinline__ int dir_off(int d, int k, int S) {
    return k ? dir_nib(kDy1, d) * S + dir_nib(kDx1, d) : dir_nib(kDy0, d) * S + dir_nib(kDx0, d);
}


__device__ __forceinline__ int ulog2d(unsigned v) { return 31 - __builtin_clz(v); }

// constrain(), src/cdef_tmpl.c:37-42; threshold 0 gives 0 for any shift
__device__ __forceinline__ int constrain(int diff, int thr, int shift) {
    const int ad = abs(diff);
    const int v = min(ad, max(0, thr - (ad >> shift)));
    return diff < 0 ? -v : v;
}

// One block's filter parameters (cdef_filter_block_c's prologue, :119-124)
struct CdefTaps {
    int pri, sec, pri_shift, sec_shift, tap0, tap1;
    int o[2][3];   // [k][primary, secondary dir + 2, secondary dir - 2] LDS offsets
    __device__ void init(int pri_, int sec_, int dir, int damping, int bd8, int S) {
        pri = pri_;
        sec = sec_;
        pri_shift = pri ? max(0, damping - ulog2d((unsigned)pri)) : 0;
        sec_shift = sec ? damping - ulog2d((unsigned)sec) : 0;
        tap0 = 4 - ((pri >> bd8) & 1);
        tap1 = (tap0 & 3) | 2;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            o[k][0] = dir_off(dir, k, S);
            o[k][1] = dir_off((dir + 2) & 7, k, S);
            o[k][2] = dir_off((dir + 6) & 7, k, S);
        }
    }
    // one output pixel from the int16 tile at c (the pixel itself)
    __device__ __forceinline__ int px(const int16_t *c) const {
        const int p = c[0];
        int sum = 0, mn = p, mx = p;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int a = c[o[k][0]], b = c[-o[k][0]];
            const int s0 = c[o[k][1]], s1 = c[-o[k][1]], s2 = c[o[k][2]], s3 = c[-o[k][2]];
            sum += (k ? tap1 : tap0) * (constrain(a - p, pri, pri_shift) + constrain(b - p, pri, pri_shift));
            sum += (2 - k) * (constrain(s0 - p, sec, sec_shift) + constrain(s1 - p, sec, sec_shift) +
                              constrain(s2 - p, sec, sec_shift) + constrain(s3 - p, sec, sec_shift));
            // min over unsigned (INT16_MIN never wins), max over signed (:139-162)
            mn = (int)min(min(min((unsigned)a, (unsigned)b), min((unsigned)s0, (unsigned)s1)),
                          min(min((unsigned)s2, (unsigned)s3), (unsigned)mn));
            mx = max(max(max(a, b), max(s0, s1)), max(max(s2, s3), mx));
        }
        const int v = p + ((sum - (sum < 0) + 8) >> 4);
        return pri && sec ? min(max(v, mn), mx) : v;
    }
    // Two pixels at once (rows y and y + 1 of a column) in packed 16-bit
    // math (v_pk_*), from a pair-interleaved tile whose dword (r, c) holds
    // rows r and r + 1 of column c: a tap of the pair is one 32-bit LDS read.
    // Every value and difference fits int16 with the kNone marker, the sums
    // too (|sum| <= 12 taps * 4 * 240).
    // PRI / SEC: whether the primary / secondary taps run -- the reference's
    // three paths (:119-214: both, primary only, secondary only; a strength
    // of 0 makes every constrain() of its taps 0 and the min / max clamp
    // belongs to the first only), so a wave whose filtering lanes all have
    // sec == 0 (or pri == 0) runs the 4-tap (8-tap) form, exactly
    template <bool PRI = true, bool SEC = true>
    __device__ __forceinline__ void px2(const uint32_t *c, int &o0, int &o1) const {
        typedef short s2 __attribute__((ext_vector_type(2)));
        typedef unsigned short u2 __attribute__((ext_vector_type(2)));
        const s2 zero = { 0, 0 };
        const s2 p = __builtin_bit_cast(s2, c[0]);
        const s2 tp = { (short)pri, (short)pri }, ts = { (short)sec, (short)sec };
        const s2 shp = { (short)pri_shift, (short)pri_shift }, shs = { (short)sec_shift, (short)sec_shift };
        s2 sum = zero, mx = p;
        u2 mn = __builtin_bit_cast(u2, p);
        // constrain(d) = sign(d) * min(|d|, v) with v = max(0, thr - (|d| >> shift))
        // = median(-v, d, v) since v >= 0; v as a saturating unsigned subtract
        auto cons = [&](s2 t, s2 thr, s2 sh) {
            const s2 d = t - p;
            const s2 ad = __builtin_elementwise_max(d, zero - d);
            const s2 v = __builtin_bit_cast(s2, __builtin_elementwise_sub_sat(__builtin_bit_cast(u2, thr),
                                                                                __builtin_bit_cast(u2, (s2)(ad >> sh))));
            return __builtin_elementwise_min(__builtin_elementwise_max(d, zero - v), v);
        };
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if constexpr (PRI) {
                const s2 a = __builtin_bit_cast(s2, c[o[k][0]]), b = __builtin_bit_cast(s2, c[-o[k][0]]);
                const short wp = (short)(k ? tap1 : tap0);
                sum += (s2){ wp, wp } * (cons(a, tp, shp) + cons(b, tp, shp));
                if constexpr (SEC) {
                    mn = __builtin_elementwise_min(mn, __builtin_elementwise_min(__builtin_bit_cast(u2, a),
                                                                                 __builtin_bit_cast(u2, b)));
                    mx = __builtin_elementwise_max(mx, __builtin_elementwise_max(a, b));
                }
            }
            if constexpr (SEC) {
                const s2 s0 = __builtin_bit_cast(s2, c[o[k][1]]), s1 = __builtin_bit_cast(s2, c[-o[k][1]]);
                const s2 s2_ = __builtin_bit_cast(s2, c[o[k][2]]), s3 = __builtin_bit_cast(s2, c[-o[k][2]]);
                const short ws = (short)(2 - k);
                sum += (s2){ ws, ws } * (cons(s0, ts, shs) + cons(s1, ts, shs) + cons(s2_, ts, shs) + cons(s3, ts, shs));
                if constexpr (PRI) {
                    mn = __builtin_elementwise_min(mn, __builtin_elementwise_min(
                             __builtin_elementwise_min(__builtin_bit_cast(u2, s0), __builtin_bit_cast(u2, s1)),
                             __builtin_elementwise_min(__builtin_bit_cast(u2, s2_), __builtin_bit_cast(u2, s3))));
                    mx = __builtin_elementwise_max(mx, __builtin_elementwise_max(__builtin_elementwise_max(s0, s1),
                                                                                 __builtin_elementwise_max(s2_, s3)));
                }
            }
        }
        const s2 neg = (s2)(sum < zero) & (s2){ 1, 1 };
        s2 v = p + ((sum - neg + (s2){ 8, 8 }) >> (s2){ 4, 4 });
        if (PRI && SEC && pri && sec) v = __builtin_elementwise_min(__builtin_elementwise_max(v, __builtin_bit_cast(s2, mn)), mx);
        o0 = v.x;
        o1 = v.y;
    }
};

// The costs of directions 2Q and 2Q+1 (cdef_find_dir_c, :246-291) from the
// block's pixels px >> bd8.  The reference sums px - 128; the partial sums
// here are of px, and each line's 128 * (its pixel count) comes off after.
template <int Q>
__device__ __forceinline__ void cdef_cost_pair(const int (&v)[8][8], unsigned &c0, unsigned &c1) {
    constexpr unsigned div[7] = { 840, 420, 280, 210, 168, 140, 120 };
    int a[15], b[11];
    constexpr auto na = [](int i) {   // pixels on line i of the a / b sets
        int n = 0;
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++)
                n += (Q == 0 ? y + x : Q == 1 ? y : Q == 2 ? 7 + y - x : x) == i;
        return n;
    };
    constexpr auto nb = [](int i) {
        int n = 0;
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++)
                n += (Q == 0 ? y + (x >> 1) : Q == 1 ? 3 + y - (x >> 1) : Q == 2 ? 3 - (y >> 1) + x : (y >> 1) + x) == i;
        return n;
    };
#pragma unroll
    for (int i = 0; i < 15; i++) a[i] = -128 * na(i);
#pragma unroll
    for (int i = 0; i < 11; i++) b[i] = -128 * nb(i);
#pragma unroll
    for (int y = 0; y < 8; y++)
#pragma unroll
        for (int x = 0; x < 8; x++) {
            const int p = v[y][x];
            if (Q == 0) { a[y + x] += p;     b[y + (x >> 1)] += p; }
            if (Q == 1) { a[y] += p;         b[3 + y - (x >> 1)] += p; }
            if (Q == 2) { a[7 + y - x] += p; b[3 - (y >> 1) + x] += p; }
            if (Q == 3) { a[x] += p;         b[(y >> 1) + x] += p; }
        }
    unsigned s = 0;
    if (Q == 0 || Q == 2) {   // diagonals: cost[0] / cost[4]
#pragma unroll
        for (int n = 0; n < 7; n++) s += (unsigned)(a[n] * a[n] + a[14 - n] * a[14 - n]) * div[n];
        s += (unsigned)(a[7] * a[7]) * 105;
    } else {                  // rows / columns: cost[2] / cost[6]
#pragma unroll
        for (int n = 0; n < 8; n++) s += (unsigned)(a[n] * a[n]);
        s *= 105;
    }
    unsigned t = 0;           // the alternate lines: cost[2Q + 1]
#pragma unroll
    for (int m = 0; m < 5; m++) t += (unsigned)(b[3 + m] * b[3 + m]);
    t *= 105;
#pragma unroll
    for (int m = 0; m < 3; m++) t += (unsigned)(b[m] * b[m] + b[10 - m] * b[10 - m]) * div[2 * m + 1];
    c0 = s;
    c1 = t;
}

template <int Q>
__device__ __forceinline__ void cdef_cost_q(const int (&v)[8][8], unsigned *cost, int stride) {
    unsigned c0, c1;
    cdef_cost_pair<Q>(v, c0, c1);
    cost[(2 * Q) * stride] = c0;
    cost[(2 * Q + 1) * stride] = c1;
}

__device__ __forceinline__ void cdef_costs(int q, const int (&v)[8][8], unsigned *cost, int stride) {
    switch (q) {
    case 0: cdef_cost_q<0>(v, cost, stride); break;
    case 1: cdef_cost_q<1>(v, cost, stride); break;
    case 2: cdef_cost_q<2>(v, cost, stride); break;
    default: cdef_cost_q<3>(v, cost, stride); break;
    }
}

// argmax (first maximum, :293-300) and variance (:302)
__device__ __forceinline__ int cdef_best(const unsigned *cost, int stride, unsigned &var) {
    unsigned c[8];
#pragma unroll
    for (int n = 0; n < 8; n++) c[n] = cost[n * stride];
    int best = 0;
    unsigned bc = c[0];
#pragma unroll
    for (int n = 1; n < 8; n++)
        if (c[n] > bc) { bc = c[n]; best = n; }
    unsigned opp = c[0];
#pragma unroll
    for (int n = 1; n < 8; n++)
        if (n == (best ^ 4)) opp = c[n];
    var = (bc - opp) >> 10;
    return best;
}

// adjust_strength, src/cdef_apply_tmpl.c:91-95
__device__ __forceinline__ int adjust_strength(int strength, unsigned var) {
    if (!var) return 0;
    const int i = var >> 6 ? min(ulog2d(var >> 6), 12) : 0;
    return (strength * (4 + i) + 8) >> 4;
}

// 4 pixels <-> int16 / pixel vectors
template <int BPC> struct Quad;
template <> struct Quad<8> {
    static __device__ __forceinline__ void load(const uint8_t *p, int16_t *d) {
        const uint32_t v = *reinterpret_cast<const uint32_t *>(p);
        d[0] = (int16_t)(v & 0xff); d[1] = (int16_t)((v >> 8) & 0xff);
        d[2] = (int16_t)((v >> 16) & 0xff); d[3] = (int16_t)(v >> 24);
    }
    static __device__ __forceinline__ void store(uint8_t *p, const int *v) {
        *reinterpret_cast<uint32_t *>(p) = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) |
                                           ((uint32_t)v[3] << 24);
    }
};
template <> struct Quad<16> {
    static __device__ __forceinline__ void load(const uint16_t *p, int16_t *d) {
        const uint2 v = *reinterpret_cast<const uint2 *>(p);
        d[0] = (int16_t)(v.x & 0xffff); d[1] = (int16_t)(v.x >> 16);
        d[2] = (int16_t)(v.y & 0xffff); d[3] = (int16_t)(v.y >> 16);
    }
    static __device__ __forceinline__ void store(uint16_t *p, const int *v) {
        uint2 o;
        o.x = (uint32_t)v[0] | ((uint32_t)v[1] << 16);
        o.y = (uint32_t)v[2] | ((uint32_t)v[3] << 16);
        *reinterpret_cast<uint2 *>(p) = o;
    }
};

template <int BPC> struct CdefArgs {
    using P = typename Px<BPC>::pixel;
    const P *in[3];
    P *out[3];
    int is[3], os[3];          // strides in pixels
    const int8_t *idx;
    const uint8_t *noskip;
    int gw, gh;                // luma grid (8x8 blocks) in pixels
    int sbw, sbh, b8w, b8h;
    int sby0, sbr;             // the superblock rows run: [sby0, sby0 + sbr)
    int bdmax, damping;
    uint8_t ys[8], uvs[8];
};

// Stage rows [y0 - 2, y0 + H + 2) and columns [x0 - 4, x0 + W + 4) of one
// plane into an int16 tile of row stride W + 8; INT16_MIN outside the grid
// (gw x gh: multiples of 4, so a 4-px group is wholly in or out).  load()
// issues every global load of the thread; store() writes the tile, so the
// three planes' loads are all in flight before the first store waits.
template <int BPC, int W, int H>
struct Stage {
    // pair-interleaved: dword (r, c) = rows r and r + 1 of column c, for the
    // H + 3 pairs of the H + 4 staged rows
    static constexpr int G = (W + 8) / 4, R = H + 3, S = W + 8, N = (G * R + 255) / 256;
    using Raw = typename std::conditional<BPC == 8, uint32_t, uint2>::type;
    Raw raw[N], raw2[N];
    bool ok[N], ok2[N];
    __device__ __forceinline__ void load(const typename Px<BPC>::pixel *src, int stride, int x0, int y0, int gw,
                                         int gh) {
#pragma unroll
        for (int n = 0; n < N; n++) {
            const int i = threadIdx.x + 256 * n, r = i / G, g = i - r * G;
            const int Y = y0 - 2 + r, X = x0 - 4 + 4 * g;
            const bool col = i < G * R && X >= 0 && X < gw;
            ok[n] = col && Y >= 0 && Y < gh;
            ok2[n] = col && Y + 1 >= 0 && Y + 1 < gh;
            if (ok[n]) raw[n] = *reinterpret_cast<const Raw *>(src + (size_t)Y * stride + X);
            if (ok2[n]) raw2[n] = *reinterpret_cast<const Raw *>(src + (size_t)(Y + 1) * stride + X);
        }
    }
    static __device__ __forceinline__ uint32_t px(const Raw &w, bool ok, int k) {
        if (!ok) return 0xc000u;   // kNone
        if constexpr (BPC == 8) return (w >> (8 * k)) & 0xff;
        else return ((k < 2 ? w.x : w.y) >> (16 * (k & 1))) & 0xffff;
    }
    __device__ __forceinline__ void store(uint32_t *t) const {
#pragma unroll
        for (int n = 0; n < N; n++) {
            const int i = threadIdx.x + 256 * n, r = i / G, g = i - r * G;
            if (i >= G * R) break;
            uint4 v;
            v.x = px(raw[n], ok[n], 0) | (px(raw2[n], ok2[n], 0) << 16);
            v.y = px(raw[n], ok[n], 1) | (px(raw2[n], ok2[n], 1) << 16);
            v.z = px(raw[n], ok[n], 2) | (px(raw2[n], ok2[n], 2) << 16);
            v.w = px(raw[n], ok[n], 3) | (px(raw2[n], ok2[n], 3) << 16);
            *reinterpret_cast<uint4 *>(&t[r * S + 4 * g]) = v;
        }
    }
};

// Filter (FILT) or copy one column of BH pixels of a block from its pair tile.
template <int BPC, int BH, bool FILT, bool PRI = true, bool SEC = true>
__device__ __forceinline__ void col_out(typename Px<BPC>::pixel *dst, int ds, const uint32_t *c, int S,
                                        const CdefTaps &tp) {
    using P = typename Px<BPC>::pixel;
#pragma unroll
    for (int y = 0; y < BH; y += 2) {
        int v0 = (int)(c[y * S] & 0xffff), v1 = (int)(c[y * S] >> 16);
        if (FILT) tp.px2<PRI, SEC>(c + y * S, v0, v1);
        dst[y * ds] = (P)v0;
        dst[(y + 1) * ds] = (P)v1;
    }
}
template <int BPC, int BH>
__device__ __forceinline__ void col_out(typename Px<BPC>::pixel *dst, int ds, const uint32_t *c, int S,
                                        const CdefTaps &tp, bool filt) {
    if (filt) {
        // (the votes run over the filtering lanes: the copying ones are masked off here)
        // (the primary-only / secondary-only forms for waves that need only one)
        if (__all(tp.sec == 0)) col_out<BPC, BH, true, true, false>(dst, ds, c, S, tp);
        else if (__all(tp.pri == 0)) col_out<BPC, BH, true, false, true>(dst, ds, c, S, tp);
        else col_out<BPC, BH, true>(dst, ds, c, S, tp);
    } else {
        col_out<BPC, BH, false>(dst, ds, c, S, tp);
    }
}

// Measured: the round-4 ablations (41.6 us whole, 41.0 without
// the direction search, 16.1 without the filter); two superblocks per
// workgroup with the second one's loads in flight (48.2 us) and a forced 6 /
// 7 waves per SIMD (42.5 / 46.8, then 38.2 against 36.1 us with a spill)
// were slower; the register allocator keeps its own choice.
template <int BPC, int LAYOUT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
void k_cdef(CdefArgs<BPC> a) {
    using P = typename Px<BPC>::pixel;
    constexpr int SX = LAYOUT == 1 || LAYOUT == 2, SY = LAYOUT == 1;
    constexpr int LS = 64 + 8;                      // luma tile stride
    constexpr int CW = 64 >> SX, CH = 64 >> SY, CS = CW + 8;
    constexpr int CBW = 8 >> SX, CBH = 8 >> SY;     // chroma block
    // pair tiles: luma first, then the two chroma tiles in the same LDS once
    // the luma blocks are filtered (the chroma loads wait in registers), so a
    // workgroup needs max(luma, chroma) instead of their sum: 21.6 KB at
    // 4:2:0, seven workgroups per CU instead of four
    constexpr int TL = (64 + 3) * LS, TC = LAYOUT ? (CH + 3) * CS : 0;
    __shared__ __attribute__((aligned(16))) uint32_t tile[TL > 2 * TC ? TL : 2 * TC];
    uint32_t *const tl = tile;
    __shared__ unsigned cost[8][64];
    __shared__ uint8_t skip[64];
    __shared__ uint8_t bdir[64], bpri[64];   // per block: direction, adjusted luma strength (<= 240)

    // XCD-contiguous superblock order: workgroups are dealt round-robin over
    // the 8 XCDs, so logical superblock (b % 8) * (n / 8) + b / 8 keeps a run
    // of neighbours (which share their border lines) in one L2
    const int nsb = a.sbw * a.sbr, nb8 = (int)gridDim.x >> 3, b = blockIdx.x;
    const int sb = (b & 7) * nb8 + (b >> 3);
    if (sb >= nsb) return;
    const int sbx = sb % a.sbw, sby = a.sby0 + sb / a.sbw;
    const int idx = a.idx[sby * a.sbw + sbx];   // (the frame's superblock index, row ranges included)
    const int ylvl = idx >= 0 ? a.ys[idx] : 0, uvlvl = idx >= 0 && LAYOUT ? a.uvs[idx] : 0;
    const bool active = ylvl || uvlvl;   // :150-156
    const int bd8 = BPC == 8 ? 0 : bits_of(a.bdmax) - 8;
    const int ypri = (ylvl >> 2) << bd8, ysec = ((ylvl & 3) + ((ylvl & 3) == 3)) << bd8;
    const int uvpri = (uvlvl >> 2) << bd8, uvsec = ((uvlvl & 3) + ((uvlvl & 3) == 3)) << bd8;
    const int damping = a.damping + bd8;

    const int x0 = sbx * 64, y0 = sby * 64;
    Stage<BPC, CW, CH> su, sv;   // every plane's loads in flight together
    {
        Stage<BPC, 64, 64> sy;
        sy.load(a.in[0], a.is[0], x0, y0, a.gw, a.gh);
        if (LAYOUT) {
            su.load(a.in[1], a.is[1], x0 >> SX, y0 >> SY, a.gw >> SX, a.gh >> SY);
            sv.load(a.in[2], a.is[2], x0 >> SX, y0 >> SY, a.gw >> SX, a.gh >> SY);
        }
        if (threadIdx.x < 64) {   // the superblock's skip flags (:185-189)
            const int gx8 = sbx * 8 + (threadIdx.x & 7), gy8 = sby * 8 + (threadIdx.x >> 3);
            skip[threadIdx.x] = gx8 < a.b8w && gy8 < a.b8h ? !a.noskip[gy8 * a.b8w + gx8] : 1;
        }
        sy.store(tl);
    }
    __syncthreads();

    // directions: wave q, lane = block (8 x 8 blocks of 8x8)
    const bool need_dir = active && (ypri || uvpri);
    if (need_dir) {
        const int q = threadIdx.x >> 6, blk = threadIdx.x & 63;
        const int bx8 = blk & 7, by8 = blk >> 3;
        if (sbx * 8 + bx8 < a.b8w && sby * 8 + by8 < a.b8h) {
            int v[8][8];
            const uint32_t *c = &tl[(by8 * 8 + 2) * LS + bx8 * 8 + 4];
#pragma unroll
            for (int y = 0; y < 8; y += 2) {   // one pair row gives two block rows
                const uint4 r0 = *reinterpret_cast<const uint4 *>(c + y * LS);
                const uint4 r1 = *reinterpret_cast<const uint4 *>(c + y * LS + 4);
                const uint32_t w[8] = { r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w };
#pragma unroll
                for (int x = 0; x < 8; x++) {   // (the - 128 is folded into cdef_cost_pair)
                    v[y][x] = BPC == 8 ? (int)(w[x] & 0xffff) : (int)(w[x] & 0xffff) >> bd8;
                    v[y + 1][x] = BPC == 8 ? (int)(w[x] >> 16) : (int)(w[x] >> 16) >> bd8;
                }
            }
            cdef_costs(q, v, &cost[0][blk], 64);
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            unsigned var;
            const int d = cdef_best(&cost[0][threadIdx.x], 64, var);
            bdir[threadIdx.x] = (uint8_t)d;
            bpri[threadIdx.x] = (uint8_t)(ypri ? adjust_strength(ypri, var) : 0);   // :237-246
        }
        __syncthreads();
    }

    // Column tasks: the lanes of a wave take consecutive columns of one row
    // of blocks and walk them down, so a tap instruction reads 64
    // consecutive int16 (plus each block's direction offset).  (A row per
    // lane put the lanes' rows 72 int16 apart, 8 lanes per LDS bank.)
    // luma: 8 rows of blocks x 64 columns
    for (int t = threadIdx.x; t < 8 * 64; t += 256) {
        const int by8 = t >> 6, l = t & 63, bx8 = l >> 3, x = l & 7, blk = by8 * 8 + bx8;
        const int gx8 = sbx * 8 + bx8, gy8 = sby * 8 + by8;
        if (gx8 >= a.b8w || gy8 >= a.b8h) continue;
        const uint32_t *c = &tl[(by8 * 8 + 2) * LS + bx8 * 8 + 4 + x];
        P *dst = a.out[0] + (size_t)(gy8 * 8) * a.os[0] + gx8 * 8 + x;
        CdefTaps tp;
        bool filt = false;
        if (active && !skip[blk]) {
            const int pri = ypri ? bpri[blk] : 0;
            if (pri || ysec) {
                tp.init(pri, ysec, ypri ? bdir[blk] : 0, damping, bd8, LS);
                filt = true;
            }
        }
        col_out<BPC, 8>(dst, a.os[0], c, LS, tp, filt);
    }
    if (!LAYOUT) return;
    __syncthreads();   // the luma tile is free: the chroma tiles go there
    su.store(tile);
    sv.store(tile + TC);
    __syncthreads();
    // chroma: 2 planes x 8 rows of blocks x 8 * CBW columns (:248-286)
    constexpr int LB = 8 * CBW;
    for (int t = threadIdx.x; t < 2 * 8 * LB; t += 256) {
        const int pl = t / (8 * LB), r = t - pl * 8 * LB;
        const int by8 = r / LB, l = r - by8 * LB, bx8 = l / CBW, x = l - bx8 * CBW, blk = by8 * 8 + bx8;
        const int gx8 = sbx * 8 + bx8, gy8 = sby * 8 + by8;
        if (gx8 >= a.b8w || gy8 >= a.b8h) continue;
        const uint32_t *c = &tile[pl * TC + (by8 * CBH + 2) * CS + bx8 * CBW + 4 + x];
        P *dst = a.out[1 + pl] + (size_t)(gy8 * CBH) * a.os[1 + pl] + gx8 * CBW + x;
        CdefTaps tp;
        bool filt = false;
        if (uvlvl && !skip[blk]) {
            int dir = 0;
            if (uvpri) {
                dir = bdir[blk];
                if (LAYOUT == 2) dir = (int)((0x66654207u >> (4 * dir)) & 15);   // uv_dirs[1], :115-117
            }
            tp.init(uvpri, uvsec, dir, damping - 1, bd8, CS);
            filt = true;
        }
        col_out<BPC, CBH>(dst, a.os[1 + pl], c, CS, tp, filt);
    }
}

template <int BPC>
static int launch_cdef(const Dav1dGpuCdefFrame *f, hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    constexpr int B = BPC / 8;
    if (!f || f->layout < 0 || f->layout > 3 || !f->cdef_idx || !f->noskip) return -1;
    const int np = f->layout ? 3 : 1;
    CdefArgs<BPC> a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < np; p++) {
        if (!f->in[p].data || !f->out[p].data || f->in[p].data == f->out[p].data) return -1;
        // 4-pixel groups are loaded and stored whole
        if (((uintptr_t)f->in[p].data | (uintptr_t)f->out[p].data | (uintptr_t)f->in[p].stride |
             (uintptr_t)f->out[p].stride) & (4 * B - 1))
            return -4;
        a.in[p] = (const P *)f->in[p].data;
        a.out[p] = (P *)f->out[p].data;
        a.is[p] = (int)(f->in[p].stride / B);
        a.os[p] = (int)(f->out[p].stride / B);
    }
    const int w = f->in[0].w, h = f->in[0].h;
    if (w <= 0 || h <= 0 || f->damping < 3 || f->damping > 6) return -1;
    for (int i = 0; i < 8; i++)
        if (f->y_strength[i] > 63 || f->uv_strength[i] > 63) return -1;
    const int bw = ((w + 7) >> 3) << 1, bh = ((h + 7) >> 3) << 1;   // f->bw, f->bh (src/decode.c:3598)
    a.gw = bw * 4;
    a.gh = bh * 4;
    a.b8w = bw >> 1;
    a.b8h = bh >> 1;
    a.sbw = (bw + 15) >> 4;
    a.sbh = (bh + 15) >> 4;
    a.idx = f->cdef_idx;
    a.noskip = f->noskip;
    a.bdmax = BPC == 8 ? 255 : f->bitdepth_max;
    a.damping = f->damping;
    memcpy(a.ys, f->y_strength, 8);
    memcpy(a.uvs, f->uv_strength, 8);
    // a row range (luma rows, multiples of 64): its superblock rows
    const int r0 = f->row_start, r1 = f->row_end;
    if (r0 < 0 || r1 < 0 || (r0 & 63) || (r1 & 63) || (r1 && r1 <= r0)) return -1;
    a.sby0 = r0 >> 6;
    a.sbr = min(a.sbh, r1 ? r1 >> 6 : a.sbh) - a.sby0;
    if (a.sbr <= 0) return 0;   // (a range past the picture)
    const dim3 grid((unsigned)((a.sbw * a.sbr + 7) & ~7));
    switch (f->layout) {
    case 0: k_cdef<BPC, 0><<<grid, 256, 0, stream>>>(a); break;
    case 1: k_cdef<BPC, 1><<<grid, 256, 0, stream>>>(a); break;
    case 2: k_cdef<BPC, 2><<<grid, 256, 0, stream>>>(a); break;
    default: k_cdef<BPC, 3><<<grid, 256, 0, stream>>>(a); break;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "dav1d-gpu: cdef launch failed: %s\n", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

// ---- per-call tier -------------------------------------------------------
// cdef_filter_block_{8x8,4x8,4x4}_c (src/cdef_tmpl.c:217-236): the 12x12
// neighbourhood assembled in LDS from dst / left / top / bottom as padding()
// does, then one pixel per lane.
template <int BPC>
__global__ __launch_bounds__(64) void k_cdef_fb(typename Px<BPC>::pixel *dst, ptrdiff_t ds,
                                                const typename Px<BPC>::pixel *src, ptrdiff_t ss,
                                                const typename Px<BPC>::pixel *left,
                                                const typename Px<BPC>::pixel *top, ptrdiff_t ts,
                                                const typename Px<BPC>::pixel *bot, ptrdiff_t bs, int pri, int sec,
                                                int dir, int damping, int edges, int w, int h, int bdmax) {
    constexpr int S = 12;
    __shared__ int16_t t[12 * S];
    for (int i = threadIdx.x; i < (h + 4) * (w + 4); i += 64) {
        const int y = i / (w + 4) - 2, x = i % (w + 4) - 2;
        const bool have = (y >= 0 || (edges & DGPU_CDEF_HAVE_TOP)) && (y < h || (edges & DGPU_CDEF_HAVE_BOTTOM)) &&
                          (x >= 0 || (edges & DGPU_CDEF_HAVE_LEFT)) && (x < w || (edges & DGPU_CDEF_HAVE_RIGHT));
        int v = kNone;
        if (have) {
            if (y < 0) v = top[(y + 2) * ts + x];
            else if (y >= h) v = bot[(y - h) * bs + x];
            else if (x < 0) v = left[y * 2 + 2 + x];
            else v = src[y * ss + x];
        }
        t[(y + 2) * S + x + 2] = (int16_t)v;
    }
    __syncthreads();
    if ((int)threadIdx.x >= w * h) return;
    const int y = threadIdx.x / w, x = threadIdx.x % w;
    CdefTaps tp;
    tp.init(pri, sec, dir, damping, bits_of(bdmax) - 8, S);
    dst[y * ds + x] = (typename Px<BPC>::pixel)tp.px(&t[(y + 2) * S + x + 2]);
}

// cdef_find_dir_c (:238-304): lane q computes directions 2q, 2q+1
template <int BPC>
__global__ __launch_bounds__(64) void k_cdef_dir(const typename Px<BPC>::pixel *img, ptrdiff_t is, int32_t *res,
                                                 int bdmax) {
    __shared__ unsigned cost[8];
    const int q = threadIdx.x, bd8 = bits_of(bdmax) - 8;
    if (q < 4) {
        int v[8][8];
#pragma unroll
        for (int y = 0; y < 8; y++)
#pragma unroll
            for (int x = 0; x < 8; x++) v[y][x] = ((int)img[y * is + x] >> bd8) - 128;
        cdef_costs(q, v, cost, 1);
    }
    __syncthreads();
    if (q == 0) {
        unsigned var;
        res[0] = cdef_best(cost, 1, var);
        res[1] = (int32_t)var;
    }
}

template <int BPC, int W, int H>
static bool cdef_fb_t(typename Px<BPC>::pixel *dst, ptrdiff_t stride, const typename Px<BPC>::pixel (*left)[2],
                      const typename Px<BPC>::pixel *top, const typename Px<BPC>::pixel *bottom, int pri, int sec,
                      int dir, int damping, int edges, int bdmax) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    const long xs = (edges & DGPU_CDEF_HAVE_LEFT) ? -2 : 0, xe = W + ((edges & DGPU_CDEF_HAVE_RIGHT) ? 2 : 0);
    Stager st;
    // dst is read over [0, xe) (padding() reads 2 px past a present right
    // edge) but written over [0, W) only
    const int id = st.in(dst, stride, 0, xe * B, 0, H);
    const int od = st.out(dst, stride, 0, W * B, 0, H);
    const int il = (edges & DGPU_CDEF_HAVE_LEFT) ? st.in1(left, 2 * H * B) : -1;
    const int it = (edges & DGPU_CDEF_HAVE_TOP) ? st.in(top, stride, xs * B, xe * B, 0, 2) : -1;
    const int ib = (edges & DGPU_CDEF_HAVE_BOTTOM) ? st.in(bottom, stride, xs * B, xe * B, 0, 2) : -1;
    if (!st.upload()) return false;
    k_cdef_fb<BPC><<<1, 64, 0, st.stream()>>>(
        st.origin<P>(od), st.pitch(od) / B, st.origin<const P>(id), st.pitch(id) / B,
        il >= 0 ? st.origin<const P>(il) : nullptr, it >= 0 ? st.origin<const P>(it) : nullptr,
        it >= 0 ? st.pitch(it) / B : 0, ib >= 0 ? st.origin<const P>(ib) : nullptr, ib >= 0 ? st.pitch(ib) / B : 0,
        pri, sec, dir, damping, edges, W, H, bdmax);
    return st.finish();
}

template <int BPC>
static bool cdef_dir_t(const typename Px<BPC>::pixel *img, ptrdiff_t stride, unsigned *var, int *dir, int bdmax) {
    using P = typename Px<BPC>::pixel;
    constexpr long B = sizeof(P);
    int32_t res[2] = { 0, 0 };
    Stager st;
    const int ii = st.in(img, stride, 0, 8 * B, 0, 8);
    const int orr = st.out1(res, sizeof(res));
    if (!st.upload()) return false;
    k_cdef_dir<BPC><<<1, 64, 0, st.stream()>>>(st.origin<const P>(ii), st.pitch(ii) / B, st.origin<int32_t>(orr),
                                               bdmax);
    if (!st.finish()) return false;
    *var = (unsigned)res[1];
    *dir = res[0];
    return true;
}

// The caller's entries before dav1d_cdef_dsp_init_gpu_* overwrote them (run
// when the GPU path fails: runtime.hpp's error contract).
static Dav1dCdefDSPContext_8bpc g_fb8;
static Dav1dCdefDSPContext_16bpc g_fb16;

#define CDEF_ENTRIES(BPC, P, BDP, BDV)                                                                    \
template <int W, int H>                                                                                   \
static void cdef_fb_##BPC(P *d, ptrdiff_t s, const P (*l)[2], const P *t, const P *b, int pri, int sec,  \
                          int dir, int damping, int edges BDP)                                            \
{ DGPU_OR_FALLBACK((cdef_fb_t<BPC, W, H>(d, s, l, t, b, pri, sec, dir, damping, edges, BDV)),            \
                   g_fb##BPC.fb[W == 8 ? 0 : H == 8 ? 1 : 2], d, s, l, t, b, pri, sec, dir, damping,     \
                   edges BDV##_ARG); }                                                                    \
static int cdef_dir_##BPC(const P *img, ptrdiff_t s, unsigned *var BDP)                                   \
{                                                                                                         \
    int dir = 0;                                                                                          \
    if (cdef_dir_t<BPC>(img, s, var, &dir, BDV)) return dir;                                              \
    return g_fb##BPC.dir ? g_fb##BPC.dir(img, s, var BDV##_ARG) : 0;                                      \
}

#define BD8_PARAM
#define BD8_VAL 255
#define BD8_VAL_ARG
#define BD16_PARAM , int bitdepth_max
#define BD16_VAL bitdepth_max
#define BD16_VAL_ARG , bitdepth_max
CDEF_ENTRIES(8, uint8_t, BD8_PARAM, BD8_VAL)
CDEF_ENTRIES(16, uint16_t, BD16_PARAM, BD16_VAL)

#define FILL_CDEF(BPC, c)                     \
    do {                                      \
        c->dir = cdef_dir_##BPC;              \
        c->fb[0] = cdef_fb_##BPC<8, 8>;       \
        c->fb[1] = cdef_fb_##BPC<4, 8>;       \
        c->fb[2] = cdef_fb_##BPC<4, 4>;       \
    } while (0)

}  // namespace dgpu

using namespace dgpu;

// bitfn(dav1d_cdef_dsp_init) replacement, src/cdef_tmpl.c:316-331
// The _gpu_ hooks keep the caller's previous entries as fallbacks.
extern "C" void dav1d_cdef_dsp_init_gpu_8bpc(Dav1dCdefDSPContext_8bpc *c) {
    Dav1dCdefDSPContext_8bpc g{}, *gp = &g;
    FILL_CDEF(8, gp);
    save_fallback(&g_fb8, c, gp);
    FILL_CDEF(8, c);
}
extern "C" void dav1d_cdef_dsp_init_gpu_16bpc(Dav1dCdefDSPContext_16bpc *c) {
    Dav1dCdefDSPContext_16bpc g{}, *gp = &g;
    FILL_CDEF(16, gp);
    save_fallback(&g_fb16, c, gp);
    FILL_CDEF(16, c);
}
extern "C" void dav1d_cdef_dsp_init_8bpc(Dav1dCdefDSPContext_8bpc *c) { FILL_CDEF(8, c); }
extern "C" void dav1d_cdef_dsp_init_16bpc(Dav1dCdefDSPContext_16bpc *c) { FILL_CDEF(16, c); }

extern "C" int dav1d_gpu_cdef_frame_8bpc(const Dav1dGpuCdefFrame *f, void *stream) {
    return launch_cdef<8>(f, (hipStream_t)stream);
}
extern "C" int dav1d_gpu_cdef_frame_16bpc(const Dav1dGpuCdefFrame *f, void *stream) {
    return launch_cdef<16>(f, (hipStream_t)stream);
}
