// dsp_common.hpp -- device-side building blocks shared by the per-call
// kernels and the fused batch kernel (gfx950, wave64).
//
// Pixel ABI traits follow include/common/bitdepth.h:36-91 of the reference:
// 8bpc = uint8 pixels / int16 coefs, 16bpc = uint16 pixels / int32 coefs with
// a run-time bitdepth_max.  MC intermediate precision and prep bias follow
// src/mc_tmpl.c:39-49.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DSPT_QUAL __constant__ static const
#include "dsp_tables.h"
#undef DSPT_QUAL

namespace dgpu {

template <int BPC> struct Px;
template <> struct Px<8> {
    using pixel = uint8_t;
    using coef = int16_t;
    static constexpr int PBIAS = 0;
    __device__ __host__ static constexpr int ibits(int) { return 4; }
};
template <> struct Px<16> {
    using pixel = uint16_t;
    using coef = int32_t;
    static constexpr int PBIAS = 8192;
    __device__ __host__ static int ibits(int bdmax) { return 14 - (32 - __builtin_clz((unsigned)bdmax)); }
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }
__device__ __forceinline__ int rnd_sh(int v, int sh) { return (v + ((1 << sh) >> 1)) >> sh; }
__device__ __forceinline__ int bits_of(int bdmax) { return 32 - __builtin_clz((unsigned)bdmax); }

// 8-tap sub-pel kernel row for 1-D filter type t at sub-pel m (1..15) over a
// block extent `len`: 4-tap banks for len <= 4, sharp -> regular there
// (src/mc_tmpl.c:99-107).  Returns nullptr for m == 0.
__device__ __forceinline__ const signed char *subpel_kernel(int t, int m, int len) {
    if (!m) return nullptr;
    const int bank = len > 4 ? t : 3 + (t & 1);
    return &dspt_subpel[(bank * 15 + m - 1) * 8];
}

// ---------------------------------------------------------------------------
// 1-D inverse transforms on register arrays (src/itx_1d.c semantics).
// Every function works in place on c[0], c[S], ..., c[(N-1)*S] with a
// compile-time stride so that after inlining the array lives in VGPRs.
// The (k - 4096) spellings mirror the reference's overflow-free forms
// (src/itx_1d.c:39-63) so results are identical for any 32-bit input.
// ---------------------------------------------------------------------------
struct Clip {
    int lo, hi;
    __device__ __forceinline__ int operator()(int v) const { return min(max(v, lo), hi); }
};

__device__ __forceinline__ int r12(int v) { return (v + 2048) >> 12; }
__device__ __forceinline__ int r11(int v) { return (v + 1024) >> 11; }
__device__ __forceinline__ int r8s(int v) { return (v * 181 + 128) >> 8; }

// 8-bit (D2) forms of the rounded product sums: every value a 1-D transform
// multiplies is then an int16 (an input, or a clipped stage output: the 8-bit
// clips are int16's range), so a sum of two products with the rounding
// constant is one v_dot2_i32_i16 of the packed pair, exact in int32 (|K| <
// 2^15).  drN<SH, K...>(v...) = (sum K_i v_i + (1 << SH >> 1)) >> SH; the
// reference's '- 4096' overflow-free forms (10/12-bit) fold back in
// (tools/gen_itx_d2.py wrote each D2SEL next to its original expression).
#define D2SEL(d2, orig) (D2 ? (d2) : (orig))
typedef short dgpu_v2i16 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int dot2c(uint32_t v, uint32_t k, int acc) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(dgpu_v2i16, v), __builtin_bit_cast(dgpu_v2i16, k), acc, false);
}
__device__ __forceinline__ uint32_t pk2(int a, int b) {   // (lo16(a), lo16(b))
    return __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x05040100u);
}
__host__ __device__ constexpr uint32_t kp2(int ka, int kb) { return (uint32_t)(uint16_t)ka | (uint32_t)(uint16_t)kb << 16; }
template <int SH, int KA> __device__ __forceinline__ int dr1(int a) {   // the high half meets a zero constant
    return dot2c((uint32_t)a, kp2(KA, 0), 1 << (SH - 1)) >> SH;
}
template <int SH> __device__ __forceinline__ int dr1v(int a, int ka) {
    return dot2c((uint32_t)a, kp2(ka, 0), 1 << (SH - 1)) >> SH;
}
template <int SH, int KA, int KB> __device__ __forceinline__ int dr2(int a, int b) {
    return dot2c(pk2(a, b), kp2(KA, KB), 1 << (SH - 1)) >> SH;
}
template <int SH, int KA, int KB, int KC> __device__ __forceinline__ int dr3(int a, int b, int c) {
    return dot2c((uint32_t)c, kp2(KC, 0), dot2c(pk2(a, b), kp2(KA, KB), 1 << (SH - 1))) >> SH;
}
template <int SH, int KA, int KB, int KC, int KD> __device__ __forceinline__ int dr4(int a, int b, int c, int d) {
    return dot2c(pk2(c, d), kp2(KC, KD), dot2c(pk2(a, b), kp2(KA, KB), 1 << (SH - 1))) >> SH;
}

template <int S, bool HALF, bool D2 = false>
__device__ __forceinline__ void dct4(int *c, Clip cl) {
    int a, b, p, q;
    if (HALF) {
        a = b = D2SEL((dr1<8, 181>(c[0])), (r8s(c[0])));
        p = D2SEL((dr1<12, 1567>(c[S])), (r12(c[S] * 1567)));
        q = D2SEL((dr1<12, 3784>(c[S])), (r12(c[S] * 3784)));
    } else {
        const int i0 = c[0], i1 = c[S], i2 = c[2 * S], i3 = c[3 * S];
        a = D2SEL((dr2<8, 181, 181>(i0, i2)), (r8s(i0 + i2)));
        b = D2SEL((dr2<8, 181, -181>(i0, i2)), (r8s(i0 - i2)));
        p = D2SEL((dr2<12, 1567, -3784>(i1, i3)), (r12(i1 * 1567 - i3 * (3784 - 4096)) - i3));
        q = D2SEL((dr2<12, 3784, 1567>(i1, i3)), (r12(i1 * (3784 - 4096) + i3 * 1567) + i1));
    }
    c[0] = cl(a + q);
    c[S] = cl(b + p);
    c[2 * S] = cl(b - p);
    c[3 * S] = cl(a - q);
}

template <int S, bool HALF, bool D2 = false>
__device__ __forceinline__ void dct8(int *c, Clip cl) {
    dct4<2 * S, HALF, D2>(c, cl);
    const int i1 = c[S], i3 = c[3 * S];
    int u4, u5, u6, u7;
    if (HALF) {
        u4 = D2SEL((dr1<12, 799>(i1)), (r12(i1 * 799)));
        u5 = D2SEL((dr1<12, -2276>(i3)), (r12(i3 * -2276)));
        u6 = D2SEL((dr1<12, 3406>(i3)), (r12(i3 * 3406)));
        u7 = D2SEL((dr1<12, 4017>(i1)), (r12(i1 * 4017)));
    } else {
        const int i5 = c[5 * S], i7 = c[7 * S];
        u4 = D2SEL((dr2<12, 799, -4017>(i1, i7)), (r12(i1 * 799 - i7 * (4017 - 4096)) - i7));
        u5 = D2SEL((dr2<11, 1703, -1138>(i5, i3)), (r11(i5 * 1703 - i3 * 1138)));
        u6 = D2SEL((dr2<11, 1138, 1703>(i5, i3)), (r11(i5 * 1138 + i3 * 1703)));
        u7 = D2SEL((dr2<12, 4017, 799>(i1, i7)), (r12(i1 * (4017 - 4096) + i7 * 799) + i1));
    }
    const int v4 = cl(u4 + u5), v5 = cl(u4 - u5), v7 = cl(u7 + u6), v6 = cl(u7 - u6);
    const int w5 = D2SEL((dr2<8, 181, -181>(v6, v5)), (r8s(v6 - v5))), w6 = D2SEL((dr2<8, 181, 181>(v6, v5)), (r8s(v6 + v5)));
    const int e0 = c[0], e1 = c[2 * S], e2 = c[4 * S], e3 = c[6 * S];
    c[0] = cl(e0 + v7);
    c[S] = cl(e1 + w6);
    c[2 * S] = cl(e2 + w5);
    c[3 * S] = cl(e3 + v4);
    c[4 * S] = cl(e3 - v4);
    c[5 * S] = cl(e2 - w5);
    c[6 * S] = cl(e1 - w6);
    c[7 * S] = cl(e0 - v7);
}

template <int S, bool HALF, bool D2 = false>
__device__ __forceinline__ void dct16(int *c, Clip cl) {
    dct8<2 * S, HALF, D2>(c, cl);
    const int i1 = c[S], i3 = c[3 * S], i5 = c[5 * S], i7 = c[7 * S];
    int a8, a9, a10, a11, a12, a13, a14, a15;
    if (HALF) {
        a8 = D2SEL((dr1<12, 401>(i1)), (r12(i1 * 401)));   a9 = D2SEL((dr1<12, -2598>(i7)), (r12(i7 * -2598)));
        a10 = D2SEL((dr1<12, 1931>(i5)), (r12(i5 * 1931))); a11 = D2SEL((dr1<12, -1189>(i3)), (r12(i3 * -1189)));
        a12 = D2SEL((dr1<12, 3920>(i3)), (r12(i3 * 3920))); a13 = D2SEL((dr1<12, 3612>(i5)), (r12(i5 * 3612)));
        a14 = D2SEL((dr1<12, 3166>(i7)), (r12(i7 * 3166))); a15 = D2SEL((dr1<12, 4076>(i1)), (r12(i1 * 4076)));
    } else {
        const int i9 = c[9 * S], i11 = c[11 * S], i13 = c[13 * S], i15 = c[15 * S];
        a8 = D2SEL((dr2<12, 401, -4076>(i1, i15)), (r12(i1 * 401 - i15 * (4076 - 4096)) - i15));
        a9 = D2SEL((dr2<11, 1583, -1299>(i9, i7)), (r11(i9 * 1583 - i7 * 1299)));
        a10 = D2SEL((dr2<12, 1931, -3612>(i5, i11)), (r12(i5 * 1931 - i11 * (3612 - 4096)) - i11));
        a11 = D2SEL((dr2<12, 3920, -1189>(i13, i3)), (r12(i13 * (3920 - 4096) - i3 * 1189) + i13));
        a12 = D2SEL((dr2<12, 1189, 3920>(i13, i3)), (r12(i13 * 1189 + i3 * (3920 - 4096)) + i3));
        a13 = D2SEL((dr2<12, 3612, 1931>(i5, i11)), (r12(i5 * (3612 - 4096) + i11 * 1931) + i5));
        a14 = D2SEL((dr2<11, 1299, 1583>(i9, i7)), (r11(i9 * 1299 + i7 * 1583)));
        a15 = D2SEL((dr2<12, 4076, 401>(i1, i15)), (r12(i1 * (4076 - 4096) + i15 * 401) + i1));
    }
    const int b8 = cl(a8 + a9), b9 = cl(a8 - a9), b10 = cl(a11 - a10), b11 = cl(a11 + a10);
    const int b12 = cl(a12 + a13), b13 = cl(a12 - a13), b14 = cl(a15 - a14), b15 = cl(a15 + a14);
    const int r9 = D2SEL((dr2<12, 1567, -3784>(b14, b9)), (r12(b14 * 1567 - b9 * (3784 - 4096)) - b9));
    const int r14 = D2SEL((dr2<12, 3784, 1567>(b14, b9)), (r12(b14 * (3784 - 4096) + b9 * 1567) + b14));
    const int r10 = D2SEL((dr2<12, -3784, -1567>(b13, b10)), (r12(-(b13 * (3784 - 4096) + b10 * 1567)) - b13));
    const int r13 = D2SEL((dr2<12, 1567, -3784>(b13, b10)), (r12(b13 * 1567 - b10 * (3784 - 4096)) - b10));
    const int d8 = cl(b8 + b11), d9 = cl(r9 + r10), d10 = cl(r9 - r10), d11 = cl(b8 - b11);
    const int d12 = cl(b15 - b12), d13 = cl(r14 - r13), d14 = cl(r14 + r13), d15 = cl(b15 + b12);
    const int odd[8] = { d15, d14, D2SEL((dr2<8, 181, 181>(d13, d10)), (r8s(d13 + d10))), D2SEL((dr2<8, 181, 181>(d12, d11)), (r8s(d12 + d11))),
                         D2SEL((dr2<8, 181, -181>(d12, d11)), (r8s(d12 - d11))), D2SEL((dr2<8, 181, -181>(d13, d10)), (r8s(d13 - d10))), d9, d8 };
    int ev[8];
#pragma unroll
    for (int i = 0; i < 8; i++) ev[i] = c[2 * i * S];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c[i * S] = cl(ev[i] + odd[i]);
        c[(15 - i) * S] = cl(ev[i] - odd[i]);
    }
}

// The 32-point odd half: rotation constants {cos, sin}-pairs per input pair.
template <int S, bool HALF, bool D2 = false>
__device__ __forceinline__ void dct32(int *c, Clip cl) {
    dct16<2 * S, HALF, D2>(c, cl);
    int t[32];
    if (HALF) {
        t[16] = D2SEL((dr1<12, 201>(c[1 * S])), (r12(c[1 * S] * 201)));   t[17] = D2SEL((dr1<12, -2751>(c[15 * S])), (r12(c[15 * S] * -2751)));
        t[18] = D2SEL((dr1<12, 1751>(c[9 * S])), (r12(c[9 * S] * 1751)));  t[19] = D2SEL((dr1<12, -1380>(c[7 * S])), (r12(c[7 * S] * -1380)));
        t[20] = D2SEL((dr1<12, 995>(c[5 * S])), (r12(c[5 * S] * 995)));   t[21] = D2SEL((dr1<12, -2106>(c[11 * S])), (r12(c[11 * S] * -2106)));
        t[22] = D2SEL((dr1<12, 2440>(c[13 * S])), (r12(c[13 * S] * 2440))); t[23] = D2SEL((dr1<12, -601>(c[3 * S])), (r12(c[3 * S] * -601)));
        t[24] = D2SEL((dr1<12, 4052>(c[3 * S])), (r12(c[3 * S] * 4052)));  t[25] = D2SEL((dr1<12, 3290>(c[13 * S])), (r12(c[13 * S] * 3290)));
        t[26] = D2SEL((dr1<12, 3513>(c[11 * S])), (r12(c[11 * S] * 3513))); t[27] = D2SEL((dr1<12, 3973>(c[5 * S])), (r12(c[5 * S] * 3973)));
        t[28] = D2SEL((dr1<12, 3857>(c[7 * S])), (r12(c[7 * S] * 3857)));  t[29] = D2SEL((dr1<12, 3703>(c[9 * S])), (r12(c[9 * S] * 3703)));
        t[30] = D2SEL((dr1<12, 3035>(c[15 * S])), (r12(c[15 * S] * 3035))); t[31] = D2SEL((dr1<12, 4091>(c[1 * S])), (r12(c[1 * S] * 4091)));
    } else {
        const int i1 = c[1 * S], i3 = c[3 * S], i5 = c[5 * S], i7 = c[7 * S];
        const int i9 = c[9 * S], i11 = c[11 * S], i13 = c[13 * S], i15 = c[15 * S];
        const int i17 = c[17 * S], i19 = c[19 * S], i21 = c[21 * S], i23 = c[23 * S];
        const int i25 = c[25 * S], i27 = c[27 * S], i29 = c[29 * S], i31 = c[31 * S];
        t[16] = D2SEL((dr2<12, 201, -4091>(i1, i31)), (r12(i1 * 201 - i31 * (4091 - 4096)) - i31));
        t[17] = D2SEL((dr2<12, 3035, -2751>(i17, i15)), (r12(i17 * (3035 - 4096) - i15 * 2751) + i17));
        t[18] = D2SEL((dr2<12, 1751, -3703>(i9, i23)), (r12(i9 * 1751 - i23 * (3703 - 4096)) - i23));
        t[19] = D2SEL((dr2<12, 3857, -1380>(i25, i7)), (r12(i25 * (3857 - 4096) - i7 * 1380) + i25));
        t[20] = D2SEL((dr2<12, 995, -3973>(i5, i27)), (r12(i5 * 995 - i27 * (3973 - 4096)) - i27));
        t[21] = D2SEL((dr2<12, 3513, -2106>(i21, i11)), (r12(i21 * (3513 - 4096) - i11 * 2106) + i21));
        t[22] = D2SEL((dr2<11, 1220, -1645>(i13, i19)), (r11(i13 * 1220 - i19 * 1645)));
        t[23] = D2SEL((dr2<12, 4052, -601>(i29, i3)), (r12(i29 * (4052 - 4096) - i3 * 601) + i29));
        t[24] = D2SEL((dr2<12, 601, 4052>(i29, i3)), (r12(i29 * 601 + i3 * (4052 - 4096)) + i3));
        t[25] = D2SEL((dr2<11, 1645, 1220>(i13, i19)), (r11(i13 * 1645 + i19 * 1220)));
        t[26] = D2SEL((dr2<12, 2106, 3513>(i21, i11)), (r12(i21 * 2106 + i11 * (3513 - 4096)) + i11));
        t[27] = D2SEL((dr2<12, 3973, 995>(i5, i27)), (r12(i5 * (3973 - 4096) + i27 * 995) + i5));
        t[28] = D2SEL((dr2<12, 1380, 3857>(i25, i7)), (r12(i25 * 1380 + i7 * (3857 - 4096)) + i7));
        t[29] = D2SEL((dr2<12, 3703, 1751>(i9, i23)), (r12(i9 * (3703 - 4096) + i23 * 1751) + i9));
        t[30] = D2SEL((dr2<12, 2751, 3035>(i17, i15)), (r12(i17 * 2751 + i15 * (3035 - 4096)) + i15));
        t[31] = D2SEL((dr2<12, 4091, 201>(i1, i31)), (r12(i1 * (4091 - 4096) + i31 * 201) + i1));
    }
    int u[32];
#pragma unroll
    for (int g = 16; g < 32; g += 4) {
        u[g] = cl(t[g] + t[g + 1]);
        u[g + 1] = cl(t[g] - t[g + 1]);
        u[g + 2] = cl(t[g + 3] - t[g + 2]);
        u[g + 3] = cl(t[g + 3] + t[g + 2]);
    }
    const int v17 = D2SEL((dr2<12, 799, -4017>(u[30], u[17])), (r12(u[30] * 799 - u[17] * (4017 - 4096)) - u[17]));
    const int v30 = D2SEL((dr2<12, 4017, 799>(u[30], u[17])), (r12(u[30] * (4017 - 4096) + u[17] * 799) + u[30]));
    const int v18 = D2SEL((dr2<12, -4017, -799>(u[29], u[18])), (r12(-(u[29] * (4017 - 4096) + u[18] * 799)) - u[29]));
    const int v29 = D2SEL((dr2<12, 799, -4017>(u[29], u[18])), (r12(u[29] * 799 - u[18] * (4017 - 4096)) - u[18]));
    const int v21 = D2SEL((dr2<11, 1703, -1138>(u[26], u[21])), (r11(u[26] * 1703 - u[21] * 1138)));
    const int v26 = D2SEL((dr2<11, 1138, 1703>(u[26], u[21])), (r11(u[26] * 1138 + u[21] * 1703)));
    const int v22 = D2SEL((dr2<11, -1138, -1703>(u[25], u[22])), (r11(-(u[25] * 1138 + u[22] * 1703))));
    const int v25 = D2SEL((dr2<11, 1703, -1138>(u[25], u[22])), (r11(u[25] * 1703 - u[22] * 1138)));
    const int w16 = cl(u[16] + u[19]), w17 = cl(v17 + v18), w18 = cl(v17 - v18), w19 = cl(u[16] - u[19]);
    const int w20 = cl(u[23] - u[20]), w21 = cl(v22 - v21), w22 = cl(v22 + v21), w23 = cl(u[23] + u[20]);
    const int w24 = cl(u[24] + u[27]), w25 = cl(v25 + v26), w26 = cl(v25 - v26), w27 = cl(u[24] - u[27]);
    const int w28 = cl(u[31] - u[28]), w29 = cl(v30 - v29), w30 = cl(v30 + v29), w31 = cl(u[31] + u[28]);
    const int x18 = D2SEL((dr2<12, 1567, -3784>(w29, w18)), (r12(w29 * 1567 - w18 * (3784 - 4096)) - w18));
    const int x29 = D2SEL((dr2<12, 3784, 1567>(w29, w18)), (r12(w29 * (3784 - 4096) + w18 * 1567) + w29));
    const int x19 = D2SEL((dr2<12, 1567, -3784>(w28, w19)), (r12(w28 * 1567 - w19 * (3784 - 4096)) - w19));
    const int x28 = D2SEL((dr2<12, 3784, 1567>(w28, w19)), (r12(w28 * (3784 - 4096) + w19 * 1567) + w28));
    const int x20 = D2SEL((dr2<12, -3784, -1567>(w27, w20)), (r12(-(w27 * (3784 - 4096) + w20 * 1567)) - w27));
    const int x27 = D2SEL((dr2<12, 1567, -3784>(w27, w20)), (r12(w27 * 1567 - w20 * (3784 - 4096)) - w20));
    const int x21 = D2SEL((dr2<12, -3784, -1567>(w26, w21)), (r12(-(w26 * (3784 - 4096) + w21 * 1567)) - w26));
    const int x26 = D2SEL((dr2<12, 1567, -3784>(w26, w21)), (r12(w26 * 1567 - w21 * (3784 - 4096)) - w21));
    const int y16 = cl(w16 + w23), y17 = cl(w17 + w22), y18 = cl(x18 + x21), y19 = cl(x19 + x20);
    const int y20 = cl(x19 - x20), y21 = cl(x18 - x21), y22 = cl(w17 - w22), y23 = cl(w16 - w23);
    const int y24 = cl(w31 - w24), y25 = cl(w30 - w25), y26 = cl(x29 - x26), y27 = cl(x28 - x27);
    const int y28 = cl(x28 + x27), y29 = cl(x29 + x26), y30 = cl(w30 + w25), y31 = cl(w31 + w24);
    const int odd[16] = { y31, y30, y29, y28,
                          D2SEL((dr2<8, 181, 181>(y27, y20)), (r8s(y27 + y20))), D2SEL((dr2<8, 181, 181>(y26, y21)), (r8s(y26 + y21))), D2SEL((dr2<8, 181, 181>(y25, y22)), (r8s(y25 + y22))), D2SEL((dr2<8, 181, 181>(y24, y23)), (r8s(y24 + y23))),
                          D2SEL((dr2<8, 181, -181>(y24, y23)), (r8s(y24 - y23))), D2SEL((dr2<8, 181, -181>(y25, y22)), (r8s(y25 - y22))), D2SEL((dr2<8, 181, -181>(y26, y21)), (r8s(y26 - y21))), D2SEL((dr2<8, 181, -181>(y27, y20)), (r8s(y27 - y20))),
                          y19, y18, y17, y16 };
    int ev[16];
#pragma unroll
    for (int i = 0; i < 16; i++) ev[i] = c[2 * i * S];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        c[i * S] = cl(ev[i] + odd[i]);
        c[(31 - i) * S] = cl(ev[i] - odd[i]);
    }
}

// 64-point DCT; only inputs 0..31 may be non-zero (src/itx_1d.c:436-781).
template <int S, bool D2 = false>
__device__ __forceinline__ void dct64(int *c, Clip cl) {
    dct32<2 * S, true, D2>(c, cl);
    constexpr int idx[32] = { 1, 31, 17, 15, 9, 23, 25, 7, 5, 27, 21, 11, 13, 19, 29, 3,
                              3, 29, 19, 13, 11, 21, 27, 5, 7, 25, 23, 9, 15, 17, 31, 1 };
    constexpr int mul[32] = { 101, -2824, 1660, -1474, 897, -2191, 2359, -700,
                              501, -2520, 2019, -1092, 1285, -1842, 2675, -301,
                              4085, 3102, 3659, 3889, 3948, 3564, 3229, 4065,
                              4036, 3349, 3461, 3996, 3822, 3745, 2967, 4095 };
    int a[32];  // a[k] holds t(32+k)
#pragma unroll
    for (int k = 0; k < 32; k++) a[k] = D2SEL((dr1v<12>(c[idx[k] * S], mul[k])), (r12(c[idx[k] * S] * mul[k])));
    int b[32];
#pragma unroll
    for (int g = 0; g < 32; g += 4) {
        b[g] = cl(a[g] + a[g + 1]);
        b[g + 1] = cl(a[g] - a[g + 1]);
        b[g + 2] = cl(a[g + 3] - a[g + 2]);
        b[g + 3] = cl(a[g + 3] + a[g + 2]);
    }
    // first rotation stage (indices relative to 32)
    int r[32];
#pragma unroll
    for (int k = 0; k < 32; k++) r[k] = b[k];
    r[1] = D2SEL((dr2<12, -4076, 401>(b[1], b[30])), (r12(b[1] * (4096 - 4076) + b[30] * 401) - b[1]));
    r[2] = D2SEL((dr2<12, -401, -4076>(b[2], b[29])), (r12(b[2] * -401 + b[29] * (4096 - 4076)) - b[29]));
    r[5] = D2SEL((dr2<11, -1299, 1583>(b[5], b[26])), (r11(b[5] * -1299 + b[26] * 1583)));
    r[6] = D2SEL((dr2<11, -1583, -1299>(b[6], b[25])), (r11(b[6] * -1583 + b[25] * -1299)));
    r[9] = D2SEL((dr2<12, -3612, 1931>(b[9], b[22])), (r12(b[9] * (4096 - 3612) + b[22] * 1931) - b[9]));
    r[10] = D2SEL((dr2<12, -1931, -3612>(b[10], b[21])), (r12(b[10] * -1931 + b[21] * (4096 - 3612)) - b[21]));
    r[13] = D2SEL((dr2<12, -1189, 3920>(b[13], b[18])), (r12(b[13] * -1189 + b[18] * (3920 - 4096)) + b[18]));
    r[14] = D2SEL((dr2<12, -3920, -1189>(b[14], b[17])), (r12(b[14] * (4096 - 3920) + b[17] * -1189) - b[14]));
    r[17] = D2SEL((dr2<12, -1189, 3920>(b[14], b[17])), (r12(b[14] * -1189 + b[17] * (3920 - 4096)) + b[17]));
    r[18] = D2SEL((dr2<12, 3920, 1189>(b[13], b[18])), (r12(b[13] * (3920 - 4096) + b[18] * 1189) + b[13]));
    r[21] = D2SEL((dr2<12, -3612, 1931>(b[10], b[21])), (r12(b[10] * (4096 - 3612) + b[21] * 1931) - b[10]));
    r[22] = D2SEL((dr2<12, 1931, 3612>(b[9], b[22])), (r12(b[9] * 1931 + b[22] * (3612 - 4096)) + b[22]));
    r[25] = D2SEL((dr2<11, -1299, 1583>(b[6], b[25])), (r11(b[6] * -1299 + b[25] * 1583)));
    r[26] = D2SEL((dr2<11, 1583, 1299>(b[5], b[26])), (r11(b[5] * 1583 + b[26] * 1299)));
    r[29] = D2SEL((dr2<12, -4076, 401>(b[2], b[29])), (r12(b[2] * (4096 - 4076) + b[29] * 401) - b[2]));
    r[30] = D2SEL((dr2<12, 401, 4076>(b[1], b[30])), (r12(b[1] * 401 + b[30] * (4076 - 4096)) + b[30]));
    int d[32];
#pragma unroll
    for (int g = 0; g < 32; g += 8) {
        d[g] = cl(r[g] + r[g + 3]);
        d[g + 1] = cl(r[g + 1] + r[g + 2]);
        d[g + 2] = cl(r[g + 1] - r[g + 2]);
        d[g + 3] = cl(r[g] - r[g + 3]);
        d[g + 4] = cl(r[g + 7] - r[g + 4]);
        d[g + 5] = cl(r[g + 6] - r[g + 5]);
        d[g + 6] = cl(r[g + 6] + r[g + 5]);
        d[g + 7] = cl(r[g + 7] + r[g + 4]);
    }
    int e[32];
#pragma unroll
    for (int k = 0; k < 32; k++) e[k] = d[k];
    e[2] = D2SEL((dr2<12, -4017, 799>(d[2], d[29])), (r12(d[2] * (4096 - 4017) + d[29] * 799) - d[2]));
    e[3] = D2SEL((dr2<12, -4017, 799>(d[3], d[28])), (r12(d[3] * (4096 - 4017) + d[28] * 799) - d[3]));
    e[4] = D2SEL((dr2<12, -799, -4017>(d[4], d[27])), (r12(d[4] * -799 + d[27] * (4096 - 4017)) - d[27]));
    e[5] = D2SEL((dr2<12, -799, -4017>(d[5], d[26])), (r12(d[5] * -799 + d[26] * (4096 - 4017)) - d[26]));
    e[10] = D2SEL((dr2<11, -1138, 1703>(d[10], d[21])), (r11(d[10] * -1138 + d[21] * 1703)));
    e[11] = D2SEL((dr2<11, -1138, 1703>(d[11], d[20])), (r11(d[11] * -1138 + d[20] * 1703)));
    e[12] = D2SEL((dr2<11, -1703, -1138>(d[12], d[19])), (r11(d[12] * -1703 + d[19] * -1138)));
    e[13] = D2SEL((dr2<11, -1703, -1138>(d[13], d[18])), (r11(d[13] * -1703 + d[18] * -1138)));
    e[18] = D2SEL((dr2<11, -1138, 1703>(d[13], d[18])), (r11(d[13] * -1138 + d[18] * 1703)));
    e[19] = D2SEL((dr2<11, -1138, 1703>(d[12], d[19])), (r11(d[12] * -1138 + d[19] * 1703)));
    e[20] = D2SEL((dr2<11, 1703, 1138>(d[11], d[20])), (r11(d[11] * 1703 + d[20] * 1138)));
    e[21] = D2SEL((dr2<11, 1703, 1138>(d[10], d[21])), (r11(d[10] * 1703 + d[21] * 1138)));
    e[26] = D2SEL((dr2<12, -4017, 799>(d[5], d[26])), (r12(d[5] * (4096 - 4017) + d[26] * 799) - d[5]));
    e[27] = D2SEL((dr2<12, -4017, 799>(d[4], d[27])), (r12(d[4] * (4096 - 4017) + d[27] * 799) - d[4]));
    e[28] = D2SEL((dr2<12, 799, 4017>(d[3], d[28])), (r12(d[3] * 799 + d[28] * (4017 - 4096)) + d[28]));
    e[29] = D2SEL((dr2<12, 799, 4017>(d[2], d[29])), (r12(d[2] * 799 + d[29] * (4017 - 4096)) + d[29]));
    int f[32];
#pragma unroll
    for (int g = 0; g < 32; g += 16) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            f[g + i] = cl(e[g + i] + e[g + 7 - i]);
            f[g + 7 - i] = cl(e[g + i] - e[g + 7 - i]);
            f[g + 8 + i] = cl(e[g + 15 - i] - e[g + 8 + i]);
            f[g + 15 - i] = cl(e[g + 15 - i] + e[g + 8 + i]);
        }
    }
    int q[32];
#pragma unroll
    for (int k = 0; k < 32; k++) q[k] = f[k];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int lo = 4 + i, hi = 27 - i;       // t36..t39 / t59..t56
        q[lo] = D2SEL((dr2<12, -3784, 1567>(f[lo], f[hi])), (r12(f[lo] * (4096 - 3784) + f[hi] * 1567) - f[lo]));
        q[hi] = D2SEL((dr2<12, 1567, 3784>(f[lo], f[hi])), (r12(f[lo] * 1567 + f[hi] * (3784 - 4096)) + f[hi]));
        const int lo2 = 8 + i, hi2 = 23 - i;     // t40..t43 / t55..t52
        q[lo2] = D2SEL((dr2<12, -1567, -3784>(f[lo2], f[hi2])), (r12(f[lo2] * -1567 + f[hi2] * (4096 - 3784)) - f[hi2]));
        q[hi2] = D2SEL((dr2<12, -3784, 1567>(f[lo2], f[hi2])), (r12(f[lo2] * (4096 - 3784) + f[hi2] * 1567) - f[lo2]));
    }
    int g2[32];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        g2[i] = cl(q[i] + q[15 - i]);
        g2[15 - i] = cl(q[i] - q[15 - i]);
        g2[16 + i] = cl(q[31 - i] - q[16 + i]);
        g2[31 - i] = cl(q[31 - i] + q[16 + i]);
    }
    int h2[32];
#pragma unroll
    for (int k = 0; k < 32; k++) h2[k] = g2[k];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int lo = 8 + i, hi = 23 - i;
        h2[lo] = D2SEL((dr2<8, 181, -181>(g2[hi], g2[lo])), (r8s(g2[hi] - g2[lo])));
        h2[hi] = D2SEL((dr2<8, 181, 181>(g2[hi], g2[lo])), (r8s(g2[hi] + g2[lo])));
    }
    int ev[32];
#pragma unroll
    for (int i = 0; i < 32; i++) ev[i] = c[2 * i * S];
#pragma unroll
    for (int i = 0; i < 32; i++) {
        c[i * S] = cl(ev[i] + h2[31 - i]);
        c[(63 - i) * S] = cl(ev[i] - h2[31 - i]);
    }
}

// ADSTs read every input before writing; FLIP writes the outputs reversed
// (src/itx_1d.c:964-975).
template <int S, bool FLIP, bool D2 = false>
__device__ __forceinline__ void adst4(int *c) {
    const int a = c[0], b = c[S], d2 = c[2 * S], d3 = c[3 * S];
    int o[4];
    o[0] = D2SEL((dr4<12, 1321, 3803, 2482, 3344>(a, d2, d3, b)), (r12(1321 * a + (3803 - 4096) * d2 + (2482 - 4096) * d3 + (3344 - 4096) * b) + d2 + d3 + b));
    o[1] = D2SEL((dr4<12, 2482, -1321, -3803, 3344>(a, d2, d3, b)), (r12((2482 - 4096) * a - 1321 * d2 - (3803 - 4096) * d3 + (3344 - 4096) * b) + a - d3 + b));
    o[2] = (209 * (a - d2 + d3) + 128) >> 8;
    o[3] = D2SEL((dr4<12, 3803, 2482, -1321, -3344>(a, d2, d3, b)), (r12((3803 - 4096) * a + (2482 - 4096) * d2 - 1321 * d3 - (3344 - 4096) * b) + a + d2 - b));
#pragma unroll
    for (int k = 0; k < 4; k++) c[(FLIP ? 3 - k : k) * S] = o[k];
}

template <int S, bool FLIP, bool D2 = false>
__device__ __forceinline__ void adst8(int *c, Clip cl) {
    int i[8];
#pragma unroll
    for (int k = 0; k < 8; k++) i[k] = c[k * S];
    const int t0a = D2SEL((dr2<12, 4076, 401>(i[7], i[0])), (r12((4076 - 4096) * i[7] + 401 * i[0]) + i[7]));
    const int t1a = D2SEL((dr2<12, 401, -4076>(i[7], i[0])), (r12(401 * i[7] - (4076 - 4096) * i[0]) - i[0]));
    const int t2a = D2SEL((dr2<12, 3612, 1931>(i[5], i[2])), (r12((3612 - 4096) * i[5] + 1931 * i[2]) + i[5]));
    const int t3a = D2SEL((dr2<12, 1931, -3612>(i[5], i[2])), (r12(1931 * i[5] - (3612 - 4096) * i[2]) - i[2]));
    const int t4a = D2SEL((dr2<11, 1299, 1583>(i[3], i[4])), (r11(1299 * i[3] + 1583 * i[4])));
    const int t5a = D2SEL((dr2<11, 1583, -1299>(i[3], i[4])), (r11(1583 * i[3] - 1299 * i[4])));
    const int t6a = D2SEL((dr2<12, 1189, 3920>(i[1], i[6])), (r12(1189 * i[1] + (3920 - 4096) * i[6]) + i[6]));
    const int t7a = D2SEL((dr2<12, 3920, -1189>(i[1], i[6])), (r12((3920 - 4096) * i[1] - 1189 * i[6]) + i[1]));
    const int t0 = cl(t0a + t4a), t1 = cl(t1a + t5a), t2 = cl(t2a + t6a), t3 = cl(t3a + t7a);
    const int t4 = cl(t0a - t4a), t5 = cl(t1a - t5a), t6 = cl(t2a - t6a), t7 = cl(t3a - t7a);
    const int u4 = D2SEL((dr2<12, 3784, 1567>(t4, t5)), (r12((3784 - 4096) * t4 + 1567 * t5) + t4));
    const int u5 = D2SEL((dr2<12, 1567, -3784>(t4, t5)), (r12(1567 * t4 - (3784 - 4096) * t5) - t5));
    const int u6 = D2SEL((dr2<12, 3784, -1567>(t7, t6)), (r12((3784 - 4096) * t7 - 1567 * t6) + t7));
    const int u7 = D2SEL((dr2<12, 1567, 3784>(t7, t6)), (r12(1567 * t7 + (3784 - 4096) * t6) + t6));
    int o[8];
    o[0] = cl(t0 + t2);
    o[7] = -cl(t1 + t3);
    const int v2 = cl(t0 - t2), v3 = cl(t1 - t3);
    o[1] = -cl(u4 + u6);
    o[6] = cl(u5 + u7);
    const int v6 = cl(u4 - u6), v7 = cl(u5 - u7);
    o[3] = -D2SEL((dr2<8, 181, 181>(v2, v3)), (r8s(v2 + v3)));
    o[4] = D2SEL((dr2<8, 181, -181>(v2, v3)), (r8s(v2 - v3)));
    o[2] = D2SEL((dr2<8, 181, 181>(v6, v7)), (r8s(v6 + v7)));
    o[5] = -D2SEL((dr2<8, 181, -181>(v6, v7)), (r8s(v6 - v7)));
#pragma unroll
    for (int k = 0; k < 8; k++) c[(FLIP ? 7 - k : k) * S] = o[k];
}

template <int S, bool FLIP, bool D2 = false>
__device__ __forceinline__ void adst16(int *c, Clip cl) {
    int i[16];
#pragma unroll
    for (int k = 0; k < 16; k++) i[k] = c[k * S];
    const int t0 = D2SEL((dr2<12, 4091, 201>(i[15], i[0])), (r12(i[15] * (4091 - 4096) + i[0] * 201) + i[15]));
    const int t1 = D2SEL((dr2<12, 201, -4091>(i[15], i[0])), (r12(i[15] * 201 - i[0] * (4091 - 4096)) - i[0]));
    const int t2 = D2SEL((dr2<12, 3973, 995>(i[13], i[2])), (r12(i[13] * (3973 - 4096) + i[2] * 995) + i[13]));
    const int t3 = D2SEL((dr2<12, 995, -3973>(i[13], i[2])), (r12(i[13] * 995 - i[2] * (3973 - 4096)) - i[2]));
    const int t4 = D2SEL((dr2<12, 3703, 1751>(i[11], i[4])), (r12(i[11] * (3703 - 4096) + i[4] * 1751) + i[11]));
    const int t5 = D2SEL((dr2<12, 1751, -3703>(i[11], i[4])), (r12(i[11] * 1751 - i[4] * (3703 - 4096)) - i[4]));
    const int t6 = D2SEL((dr2<11, 1645, 1220>(i[9], i[6])), (r11(i[9] * 1645 + i[6] * 1220)));
    const int t7 = D2SEL((dr2<11, 1220, -1645>(i[9], i[6])), (r11(i[9] * 1220 - i[6] * 1645)));
    const int t8 = D2SEL((dr2<12, 2751, 3035>(i[7], i[8])), (r12(i[7] * 2751 + i[8] * (3035 - 4096)) + i[8]));
    const int t9 = D2SEL((dr2<12, 3035, -2751>(i[7], i[8])), (r12(i[7] * (3035 - 4096) - i[8] * 2751) + i[7]));
    const int t10 = D2SEL((dr2<12, 2106, 3513>(i[5], i[10])), (r12(i[5] * 2106 + i[10] * (3513 - 4096)) + i[10]));
    const int t11 = D2SEL((dr2<12, 3513, -2106>(i[5], i[10])), (r12(i[5] * (3513 - 4096) - i[10] * 2106) + i[5]));
    const int t12 = D2SEL((dr2<12, 1380, 3857>(i[3], i[12])), (r12(i[3] * 1380 + i[12] * (3857 - 4096)) + i[12]));
    const int t13 = D2SEL((dr2<12, 3857, -1380>(i[3], i[12])), (r12(i[3] * (3857 - 4096) - i[12] * 1380) + i[3]));
    const int t14 = D2SEL((dr2<12, 601, 4052>(i[1], i[14])), (r12(i[1] * 601 + i[14] * (4052 - 4096)) + i[14]));
    const int t15 = D2SEL((dr2<12, 4052, -601>(i[1], i[14])), (r12(i[1] * (4052 - 4096) - i[14] * 601) + i[1]));
    const int a0 = cl(t0 + t8), a1 = cl(t1 + t9), a2 = cl(t2 + t10), a3 = cl(t3 + t11);
    const int a4 = cl(t4 + t12), a5 = cl(t5 + t13), a6 = cl(t6 + t14), a7 = cl(t7 + t15);
    const int a8 = cl(t0 - t8), a9 = cl(t1 - t9), a10 = cl(t2 - t10), a11 = cl(t3 - t11);
    const int a12 = cl(t4 - t12), a13 = cl(t5 - t13), a14 = cl(t6 - t14), a15 = cl(t7 - t15);
    const int b8 = D2SEL((dr2<12, 4017, 799>(a8, a9)), (r12(a8 * (4017 - 4096) + a9 * 799) + a8));
    const int b9 = D2SEL((dr2<12, 799, -4017>(a8, a9)), (r12(a8 * 799 - a9 * (4017 - 4096)) - a9));
    const int b10 = D2SEL((dr2<12, 2276, 3406>(a10, a11)), (r12(a10 * 2276 + a11 * (3406 - 4096)) + a11));
    const int b11 = D2SEL((dr2<12, 3406, -2276>(a10, a11)), (r12(a10 * (3406 - 4096) - a11 * 2276) + a10));
    const int b12 = D2SEL((dr2<12, 4017, -799>(a13, a12)), (r12(a13 * (4017 - 4096) - a12 * 799) + a13));
    const int b13 = D2SEL((dr2<12, 799, 4017>(a13, a12)), (r12(a13 * 799 + a12 * (4017 - 4096)) + a12));
    const int b14 = D2SEL((dr2<12, 2276, -3406>(a15, a14)), (r12(a15 * 2276 - a14 * (3406 - 4096)) - a14));
    const int b15 = D2SEL((dr2<12, 3406, 2276>(a15, a14)), (r12(a15 * (3406 - 4096) + a14 * 2276) + a15));
    const int c0 = cl(a0 + a4), c1 = cl(a1 + a5), c2 = cl(a2 + a6), c3 = cl(a3 + a7);
    const int c4 = cl(a0 - a4), c5 = cl(a1 - a5), c6 = cl(a2 - a6), c7 = cl(a3 - a7);
    const int c8 = cl(b8 + b12), c9 = cl(b9 + b13), c10 = cl(b10 + b14), c11 = cl(b11 + b15);
    const int c12 = cl(b8 - b12), c13 = cl(b9 - b13), c14 = cl(b10 - b14), c15 = cl(b11 - b15);
    const int d4 = D2SEL((dr2<12, 3784, 1567>(c4, c5)), (r12(c4 * (3784 - 4096) + c5 * 1567) + c4));
    const int d5 = D2SEL((dr2<12, 1567, -3784>(c4, c5)), (r12(c4 * 1567 - c5 * (3784 - 4096)) - c5));
    const int d6 = D2SEL((dr2<12, 3784, -1567>(c7, c6)), (r12(c7 * (3784 - 4096) - c6 * 1567) + c7));
    const int d7 = D2SEL((dr2<12, 1567, 3784>(c7, c6)), (r12(c7 * 1567 + c6 * (3784 - 4096)) + c6));
    const int d12 = D2SEL((dr2<12, 3784, 1567>(c12, c13)), (r12(c12 * (3784 - 4096) + c13 * 1567) + c12));
    const int d13 = D2SEL((dr2<12, 1567, -3784>(c12, c13)), (r12(c12 * 1567 - c13 * (3784 - 4096)) - c13));
    const int d14 = D2SEL((dr2<12, 3784, -1567>(c15, c14)), (r12(c15 * (3784 - 4096) - c14 * 1567) + c15));
    const int d15 = D2SEL((dr2<12, 1567, 3784>(c15, c14)), (r12(c15 * 1567 + c14 * (3784 - 4096)) + c14));
    int o[16];
    o[0] = cl(c0 + c2);
    o[15] = -cl(c1 + c3);
    const int e2 = cl(c0 - c2), e3 = cl(c1 - c3);
    o[3] = -cl(d4 + d6);
    o[12] = cl(d5 + d7);
    const int e6 = cl(d4 - d6), e7 = cl(d5 - d7);
    o[1] = -cl(c8 + c10);
    o[14] = cl(c9 + c11);
    const int e10 = cl(c8 - c10), e11 = cl(c9 - c11);
    o[2] = cl(d12 + d14);
    o[13] = -cl(d13 + d15);
    const int e14 = cl(d12 - d14), e15 = cl(d13 - d15);
    o[7] = -D2SEL((dr2<8, 181, 181>(e2, e3)), (r8s(e2 + e3)));
    o[8] = D2SEL((dr2<8, 181, -181>(e2, e3)), (r8s(e2 - e3)));
    o[4] = D2SEL((dr2<8, 181, 181>(e6, e7)), (r8s(e6 + e7)));
    o[11] = -D2SEL((dr2<8, 181, -181>(e6, e7)), (r8s(e6 - e7)));
    o[6] = D2SEL((dr2<8, 181, 181>(e10, e11)), (r8s(e10 + e11)));
    o[9] = -D2SEL((dr2<8, 181, -181>(e10, e11)), (r8s(e10 - e11)));
    o[5] = -D2SEL((dr2<8, 181, 181>(e14, e15)), (r8s(e14 + e15)));
    o[10] = D2SEL((dr2<8, 181, -181>(e14, e15)), (r8s(e14 - e15)));
#pragma unroll
    for (int k = 0; k < 16; k++) c[(FLIP ? 15 - k : k) * S] = o[k];
}

// identity scalings, src/itx_1d.c:983-1017
template <int N, int S, bool D2 = false>
__device__ __forceinline__ void identity(int *c) {
#pragma unroll
    for (int k = 0; k < N; k++) {
        const int v = c[k * S];
        if (N == 4) c[k * S] = v + D2SEL((dr1<12, 1697>(v)), (r12(v * 1697)));
        else if (N == 8) c[k * S] = v * 2;
        else if (N == 16) c[k * S] = 2 * v + D2SEL((dr1<11, 1697>(v)), (r11(v * 1697)));
        else c[k * S] = v * 4;
    }
}

// Walsh-Hadamard, src/itx_1d.c:1023-1038
template <int S>
__device__ __forceinline__ void wht4(int *c) {
    const int a = c[0], b = c[S], d2 = c[2 * S], d3 = c[3 * S];
    const int t0 = a + b, t2 = d2 - d3, t4 = (t0 - t2) >> 1, t3 = t4 - d3, t1 = t4 - b;
    c[0] = t0 - t3;
    c[S] = t3;
    c[2 * S] = t1;
    c[3 * S] = t2 + t1;
}

// WHT_WHT (lossless 4x4) for the batch kernels, src/itx_tmpl.c:166-185: both
// passes in one lane's int32 registers from the compact coefficient region
// (column-major, nzh rows; zeros outside it), coef >> 2 first, no clip and no
// shift anywhere.  t[] is the residual, row-major.  A batch kernel keeps an
// 8-bit residual in int16: saturating it there changes no output pixel (a
// residual beyond +-32767 clips the same way for any pixel in [0, bdmax]),
// whereas the row pass's int16 intermediate would not be exact for extreme
// coefficients, which is why this does not reuse the kernels' row / column
// passes.
template <typename C>
__device__ __forceinline__ void wht4x4(const C *cs, int nzw, int nzh, int *t) {
#pragma unroll
    for (int y = 0; y < 4; y++) {
#pragma unroll
        for (int x = 0; x < 4; x++) t[4 * y + x] = (x < nzw && y < nzh) ? (int)cs[x * nzh + y] >> 2 : 0;
        wht4<1>(&t[4 * y]);
    }
#pragma unroll
    for (int x = 0; x < 4; x++) wht4<4>(&t[x]);
}

enum Kind1D { K_DCT = 0, K_ADST = 1, K_FLIPADST = 2, K_IDENTITY = 3 };

// Run-time kind, compile-time length.  Unsupported (kind, N) pairs never
// occur: the tables only reference the instantiations the reference has.
template <int N, int S, bool D2 = false>
__device__ __forceinline__ void tx1d(int kind, int *c, Clip cl) {
    if (kind == K_DCT) {
        if constexpr (N == 4) dct4<S, false, D2>(c, cl);
        else if constexpr (N == 8) dct8<S, false, D2>(c, cl);
        else if constexpr (N == 16) dct16<S, false, D2>(c, cl);
        else if constexpr (N == 32) dct32<S, false, D2>(c, cl);
        else dct64<S, D2>(c, cl);
    } else if (kind == K_IDENTITY) {
        if constexpr (N <= 32) identity<N, S, D2>(c);
    } else {
        // ADST and FLIPADST share one body (lanes of a wave may mix them);
        // the flip is an in-register reversal by selects
        if constexpr (N == 4) adst4<S, false, D2>(c);
        else if constexpr (N == 8) adst8<S, false, D2>(c, cl);
        else if constexpr (N == 16) adst16<S, false, D2>(c, cl);
        if constexpr (N <= 16) {
            const bool f = kind == K_FLIPADST;
#pragma unroll
            for (int i = 0; i < N / 2; i++) {
                const int lo = c[i * S], hi = c[(N - 1 - i) * S];
                c[i * S] = f ? hi : lo;
                c[(N - 1 - i) * S] = f ? lo : hi;
            }
        }
    }
}

// {vertical, horizontal} 1-D kinds per TxfmType, 2 bits per type
// (src/itx_tmpl.c:210-242: the type's first word is the vertical transform)
//   v: 0 1 0 1 2 0 2 1 2 3 0 3 1 3 2 3   h: 0 0 1 1 0 2 2 2 1 3 3 0 3 1 3 2
__device__ __host__ __forceinline__ int kind_v(int txtp) { return (0xedce6244u >> (2 * txtp)) & 3; }
__device__ __host__ __forceinline__ int kind_h(int txtp) { return (0xb73da850u >> (2 * txtp)) & 3; }

// width, height, shift per RectTxfmSize (src/itx_tmpl.c:142-160)
struct TxInfo { unsigned char w, h, shift; };
__device__ __host__ constexpr TxInfo tx_info(int tx) {
    constexpr TxInfo t[19] = {
        { 4, 4, 0 }, { 8, 8, 1 }, { 16, 16, 2 }, { 32, 32, 2 }, { 64, 64, 2 },
        { 4, 8, 0 }, { 8, 4, 0 }, { 8, 16, 1 }, { 16, 8, 1 }, { 16, 32, 1 },
        { 32, 16, 1 }, { 32, 64, 1 }, { 64, 32, 1 }, { 4, 16, 1 }, { 16, 4, 1 },
        { 8, 32, 2 }, { 32, 8, 2 }, { 16, 64, 2 }, { 64, 16, 2 },
    };
    return t[tx];
}

template <int BPC> struct ItxClip;
template <> struct ItxClip<8> {
    __device__ static Clip row(int) { return { -32768, 32767 }; }
    __device__ static Clip col(int) { return { -32768, 32767 }; }
};
template <> struct ItxClip<16> {  // src/itx_tmpl.c:72-76
    __device__ static Clip row(int bdmax) {
        const int lo = (int)((unsigned)~bdmax << 7);
        return { lo, ~lo };
    }
    __device__ static Clip col(int bdmax) {
        const int lo = (int)((unsigned)~bdmax << 5);
        return { lo, ~lo };
    }
};

}  // namespace dgpu
