// recon_kernel.hpp -- the batch tier: one grid launch per class group
// reconstructs a frame's worth of transform-block units (Dav1dGpuUnit).
//
// Per unit the work the reference does in recon_b_inter / recon_b_intra
// (src/recon_tmpl.c:1598, :1195) for one transform block: the prediction
// (mc put, or mct x2 + avg, src/recon_tmpl.c:957-1059, :1845; or intra_pred,
// :1294) then inv_txfm_add (:816 / :1347), fused so the prediction never
// round-trips through HBM.
//
// Mapping (wave64, v2).  Units are sorted by transform size class.  A wave
// owns U = 64 / G units of one class, G lanes each (G grows with the unit so
// each lane has a handful of pixels).  Every phase is element-parallel over
// the unit's G lanes -- no lane walks a whole column serially:
//   P1  reference footprint(s): a fixed, unrolled count of dword loads per
//       lane (all issued before any is consumed), kept at their byte skew
//       in LDS; intra edges likewise; coefficient rows for P3 are loaded too
//   P2  intra: directional / filter-intra edge preparation, then the
//       prediction of every pixel into an LDS tile
//   P3  row transforms (lane y < min(h,32)), transposed into LDS
//   P4  column transforms (lane x < w) -> residual tile in LDS
//   P5  mc horizontal pass: one 8-tap sum per (row, x) -- packed-byte
//       v_dot4 on 8bpc -- into an int16 intermediate tile
//   P6  mc vertical pass / compound average / intra tile, + residual, clip,
//       into the output tile
//   P7  output rows stored with aligned 4..16-byte stores
// Every LDS hand-off stays inside one wave (no workgroup barrier).
#pragma once
#include "dav1d_gpu.h"
#include "dsp_common.hpp"

namespace dgpu {

constexpr int kSegments = 16;   // spatial segments per class (task ordering)

template <int BPC> struct ReconArgs {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    P *dst[3];
    int dst_stride[3];                   // pixels
    const P *ref[DGPU_MAX_REFS][3];
    int ref_stride[DGPU_MAX_REFS][3];    // pixels
    const Dav1dGpuUnit *units;
    C *coef;
    const P *edges;
    int class_start[DGPU_N_RECT_TX_SIZES + 1];
    // wave schedule: waves are ordered (segment, class); seg_wave[s * NC + c]
    // is the first wave of (segment s, class c), a running prefix.
    int seg_wave[kSegments * DGPU_N_RECT_TX_SIZES + 1];
    int nwaves;
    int bdmax;
    int zero_coefs;
    int ablate;   // debug-only phase mask (DAV1D_GPU_ABLATE); 0 in production
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }
__host__ __device__ constexpr int cmin(int a, int b) { return a < b ? a : b; }
__host__ __device__ constexpr int a16(int v) { return (v + 15) & ~15; }

// size-class shape: lanes per unit G = clamp(w*h/4, 8, 64), at least
// max(w, min(h,32)) so the 1-D transforms have a lane per line
__host__ __device__ constexpr int lanes_per_unit(int tx) {
    const int w = tx_info(tx).w, h = tx_info(tx).h, sh = cmin(h, 32);
    return cmax(cmax(cmin(cmax(w * h / 4, 8), 64), w), sh);
}
// class groups, each its own kernel (own register / LDS budget)
enum { GROUP_SMALL = 0, GROUP_LARGE = 1, GROUP_HUGE = 2 };
__host__ __device__ constexpr int class_group(int tx) {
    const int w = tx_info(tx).w, h = tx_info(tx).h;
    return (w == 64 || h == 64) ? GROUP_HUGE : (w * h <= 128 ? GROUP_SMALL : GROUP_LARGE);
}

template <int TX> struct Cls {
    static constexpr int W = tx_info(TX).w, H = tx_info(TX).h, SHIFT = tx_info(TX).shift;
    static constexpr int SW = cmin(W, 32), SH = cmin(H, 32);
    static constexpr int G = lanes_per_unit(TX);
    static constexpr int U = 64 / G;
    static constexpr bool RECT2 = W * 2 == H || H * 2 == W;
};

template <int BPC> struct Tmp { using T = int32_t; };
template <> struct Tmp<8> { using T = int16_t; };  // 8-bit column range is int16

// LDS slot of one unit (bytes).  TMP holds the transposed row results, then
// (aliased, consumed in program order) the residual tile and the output tile.
template <int BPC, int TX> struct Slot {
    using CL = Cls<TX>;
    static constexpr int W = CL::W, H = CL::H, B = BPC / 8;
    static constexpr int TP = CL::SH + 1;
    static constexpr int TMP = a16(cmax(W * TP * (int)sizeof(typename Tmp<BPC>::T), W * H * 2));
    static constexpr int NDW = (3 + (W + 7) * B + 3) / 4;           // dwords per footprint row
    static constexpr int FPB = NDW * 4;
    static constexpr int FP = a16((H + 7) * FPB);
    static constexpr int MID = a16((H + 7) * W * 2);
    static constexpr int EDGE = 2 * H + 2 * W + 1;                   // topleft[-2h..2w]
    static constexpr int INTRA = a16(2 * EDGE * 2 + W * H * 2);
    static constexpr int SRC = cmax(2 * FP + 2 * MID, INTRA);
    static constexpr int BYTES = TMP + SRC;
    static constexpr int WAVE = CL::U * BYTES;
};

// ---------------------------------------------------------------- intra ---

__device__ __forceinline__ int ip_strength(int wh, int angle, int is_sm) {  // ipred_tmpl.c:327
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
__device__ __forceinline__ int ip_upsample(int wh, int angle, int is_sm) {
    return angle < 40 && wh <= (16 >> is_sm);
}
// filter_edge element (src/ipred_tmpl.c:362-385), `in` indexed from 0
__device__ __forceinline__ int ip_smooth(const int16_t *in, int i, int lim_from, int lim_to, int from,
                                         int to, int st) {
    if (i < lim_from || i >= lim_to) return in[clampi(i, from, to - 1)];
    const int k0 = st == 3 ? 2 : 0, k1 = st == 2 ? 5 : 4, k2 = st == 1 ? 8 : st == 2 ? 6 : 4;
    const int s = k0 * (in[clampi(i - 2, from, to - 1)] + in[clampi(i + 2, from, to - 1)]) +
                  k1 * (in[clampi(i - 1, from, to - 1)] + in[clampi(i + 1, from, to - 1)]) +
                  k2 * in[clampi(i, from, to - 1)];
    return (s + 8) >> 4;
}
// upsample_edge element (src/ipred_tmpl.c:391-406)
__device__ __forceinline__ int ip_up(const int16_t *in, int o, int hsz, int from, int to, int bdmax) {
    const int i = o >> 1;
    if (!(o & 1) || i >= hsz - 1) return in[clampi(i, from, to - 1)];
    const int s = -in[clampi(i - 1, from, to - 1)] + 9 * in[clampi(i, from, to - 1)] +
                  9 * in[clampi(i + 1, from, to - 1)] - in[clampi(i + 2, from, to - 1)];
    return clampi((s + 8) >> 4, 0, bdmax);
}

// intra prediction of one unit into `ptile` (int16, W x H), all G lanes.
// e: topleft[-2h..2w] staged as int16; fe: scratch edge.
template <int BPC, int TX>
__device__ __forceinline__ void intra_unit(const Dav1dGpuUnit &u, int16_t *e, int16_t *fe, int16_t *ptile,
                                           int l, int bdmax) {
    using CL = Cls<TX>;
    constexpr int W = CL::W, H = CL::H, G = CL::G;
    const int16_t *tl = e + 2 * H;   // topleft[0]
    const int mode = u.p.intra.mode;
    const int ang = u.p.intra.angle & 511, is_sm = (u.p.intra.angle >> 9) & 1, filt = u.p.intra.angle >> 10;
    int up = 0, upl = 0, d1 = 0, d2 = 0, maxb = 0, dc = 0;
    if (mode == DGPU_Z1_PRED) {   // src/ipred_tmpl.c:408-443
        d1 = dspt_dr_deriv[ang >> 1];
        up = filt ? ip_upsample(W + H, 90 - ang, is_sm) : 0;
        const int st = (!up && filt) ? ip_strength(W + H, 90 - ang, is_sm) : 0;
        if (up) {
            for (int o = l; o < 2 * (W + H) - 1; o += G) fe[o] = ip_up(tl + 1, o, W + H, -1, W + cmin(W, H), bdmax);
            maxb = 2 * (W + H) - 2;
            d1 <<= 1;
        } else if (st) {
            for (int i = l; i < W + H; i += G) fe[i] = ip_smooth(tl + 1, i, 0, W + H, -1, W + cmin(W, H), st);
            maxb = W + H - 1;
        } else {
            for (int i = l; i < W + cmin(W, H); i += G) fe[i] = tl[1 + i];
            maxb = W + cmin(W, H) - 1;
        }
    } else if (mode == DGPU_Z3_PRED) {   // src/ipred_tmpl.c:542-581; fe[maxb - i] == left[-i]
        d1 = dspt_dr_deriv[(270 - ang) >> 1];
        up = filt ? ip_upsample(W + H, ang - 180, is_sm) : 0;
        const int st = (!up && filt) ? ip_strength(W + H, ang - 180, is_sm) : 0;
        if (up) {
            for (int o = l; o < 2 * (W + H) - 1; o += G)
                fe[o] = ip_up(tl - (W + H), o, W + H, cmax(W - H, 0), W + H + 1, bdmax);
            maxb = 2 * (W + H) - 2;
            d1 <<= 1;
        } else if (st) {
            for (int i = l; i < W + H; i += G)
                fe[i] = ip_smooth(tl - (W + H), i, 0, W + H, cmax(W - H, 0), W + H + 1, st);
            maxb = W + H - 1;
        } else {
            maxb = H + cmin(W, H) - 1;
            for (int i = l; i <= maxb; i += G) fe[i] = tl[-1 - maxb + i];
        }
    } else if (mode == DGPU_Z2_PRED) {   // src/ipred_tmpl.c:462-513
        d2 = dspt_dr_deriv[(ang - 90) >> 1];   // dy
        d1 = dspt_dr_deriv[(180 - ang) >> 1];  // dx
        upl = filt ? ip_upsample(W + H, 180 - ang, is_sm) : 0;
        up = filt ? ip_upsample(W + H, ang - 90, is_sm) : 0;
        int16_t *c = fe + 2 * H;   // corner
        if (up) {
            for (int o = l; o < 2 * W + 1; o += G) c[o] = ip_up(tl, o, W + 1, 0, W + 1, bdmax);
        } else {
            const int st = filt ? ip_strength(W + H, ang - 90, is_sm) : 0;
            for (int i = l; i < W; i += G)
                c[1 + i] = st ? ip_smooth(tl + 1, i, 0, u.p.intra.max_w, -1, W, st) : tl[1 + i];
        }
        if (upl) {
            for (int o = l; o < 2 * H + 1; o += G) c[-2 * H + o] = ip_up(tl - H, o, H + 1, 0, H + 1, bdmax);
        } else {
            const int st = filt ? ip_strength(W + H, 180 - ang, is_sm) : 0;
            for (int i = l; i < H; i += G)
                c[-H + i] = st ? ip_smooth(tl - H, i, H - u.p.intra.max_h, H, 0, H + 1, st) : tl[-H + i];
        }
        wave_sync();
        if (l == 0) c[0] = tl[0];
        if (up) d1 <<= 1;
        if (upl) d2 <<= 1;
    } else if (mode == DGPU_FILTER_PRED) {   // src/ipred_tmpl.c:617-655, cells in anti-diagonal waves
        if constexpr (W <= 32 && H <= 32) {
            const signed char *taps = &dspt_filter_intra[(u.p.intra.angle & 511) * 56];
            constexpr int cw = W / 4, ch = H / 2;
            for (int step = 0; step < cw + ch - 1; step++) {
                for (int cidx = l; cidx < cw * ch; cidx += G) {
                    const int cx = cidx % cw, cy = cidx / cw;
                    if (cx + cy != step) continue;
                    const int x = cx * 4, y = cy * 2;
                    int p0, p1, p2, p3, p4, p5, p6;
                    if (y == 0) {
                        p0 = x == 0 ? tl[0] : tl[x];
                        p1 = tl[1 + x]; p2 = tl[2 + x]; p3 = tl[3 + x]; p4 = tl[4 + x];
                    } else {
                        const int16_t *upr = ptile + (y - 1) * W + x;
                        p0 = x == 0 ? tl[-y] : upr[-1];
                        p1 = upr[0]; p2 = upr[1]; p3 = upr[2]; p4 = upr[3];
                    }
                    p5 = x == 0 ? tl[-(y + 1)] : ptile[y * W + x - 1];
                    p6 = x == 0 ? tl[-(y + 2)] : ptile[(y + 1) * W + x - 1];
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        const signed char *tk = taps + k * 7;
                        const int acc = tk[0] * p0 + tk[1] * p1 + tk[2] * p2 + tk[3] * p3 + tk[4] * p4 +
                                        tk[5] * p5 + tk[6] * p6;
                        ptile[(y + (k >> 2)) * W + x + (k & 3)] = clampi((acc + 8) >> 4, 0, bdmax);
                    }
                }
                wave_sync();
            }
        }
        return;
    } else if (mode != DGPU_VERT_PRED && mode != DGPU_HOR_PRED && mode <= DGPU_DC_128_PRED) {
        // DC family: group reduction of the edge sums (src/ipred_tmpl.c:86-166)
        unsigned st = 0, sl = 0;
        for (int i = l; i < W; i += G) st += tl[1 + i];
        for (int i = l; i < H; i += G) sl += tl[-1 - i];
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            st += __shfl_xor(st, off, 64);
            sl += __shfl_xor(sl, off, 64);
        }
        unsigned s;
        if (mode == DGPU_DC_128_PRED) s = (bdmax + 1) >> 1;
        else if (mode == DGPU_TOP_DC_PRED) s = (st + (W >> 1)) >> __builtin_ctz(W);
        else if (mode == DGPU_LEFT_DC_PRED) s = (sl + (H >> 1)) >> __builtin_ctz(H);
        else {
            s = (st + sl + ((W + H) >> 1)) >> __builtin_ctz(W + H);
            if (W != H) {
                const bool r4 = W > 2 * H || H > 2 * W;
                if (BPC == 8) s = (s * (r4 ? 0x3334u : 0x5556u)) >> 16;
                else s = (s * (r4 ? 0x6667u : 0xAAABu)) >> 17;
            }
        }
        dc = (int)s;
    }
    wave_sync();
    for (int i = l; i < W * H; i += G) {
        const int x = i % W, y = i / W;
        const int top = tl[1 + x], left = tl[-(1 + y)];
        int v;
        switch (mode) {
        case DGPU_VERT_PRED: v = top; break;
        case DGPU_HOR_PRED: v = left; break;
        case DGPU_PAETH_PRED: {   // src/ipred_tmpl.c:244-265
            const int c0 = tl[0], base = left + top - c0;
            const int dl = abs(left - base), dt = abs(top - base), dd = abs(c0 - base);
            v = (dl <= dt && dl <= dd) ? left : dt <= dd ? top : c0;
            break;
        }
        case DGPU_SMOOTH_PRED: {   // src/ipred_tmpl.c:267-325
            const int wv = dspt_sm_weights[H + y], wh = dspt_sm_weights[W + x];
            v = (wv * top + (256 - wv) * tl[-H] + wh * left + (256 - wh) * tl[W] + 256) >> 9;
            break;
        }
        case DGPU_SMOOTH_V_PRED: {
            const int wv = dspt_sm_weights[H + y];
            v = (wv * top + (256 - wv) * tl[-H] + 128) >> 8;
            break;
        }
        case DGPU_SMOOTH_H_PRED: {
            const int wh = dspt_sm_weights[W + x];
            v = (wh * left + (256 - wh) * tl[W] + 128) >> 8;
            break;
        }
        case DGPU_Z1_PRED: {
            const int xpos = (y + 1) * d1, frac = xpos & 0x3e;
            const int base = (xpos >> 6) + x * (1 + up);
            v = base < maxb ? (fe[base] * (64 - frac) + fe[base + 1] * frac + 32) >> 6 : fe[maxb];
            break;
        }
        case DGPU_Z3_PRED: {
            const int ypos = (x + 1) * d1, frac = ypos & 0x3e;
            const int base = (ypos >> 6) + y * (1 + up);
            v = base < maxb ? (fe[maxb - base] * (64 - frac) + fe[maxb - base - 1] * frac + 32) >> 6 : fe[0];
            break;
        }
        case DGPU_Z2_PRED: {
            const int16_t *c = fe + 2 * H;
            const int xpos = ((1 + up) << 6) - (y + 1) * d1;
            const int bx = (xpos >> 6) + x * (1 + up);
            int t;
            if (bx >= 0) {
                const int fx = xpos & 0x3e;
                t = c[bx] * (64 - fx) + c[bx + 1] * fx;
            } else {
                const int ypos = (y << (6 + upl)) - (x + 1) * d2;
                const int by = ypos >> 6, fy = ypos & 0x3e;
                const int16_t *lft = c - (1 + upl);
                t = lft[-by] * (64 - fy) + lft[-(by + 1)] * fy;
            }
            v = (t + 32) >> 6;
            break;
        }
        default: v = dc; break;   // DC family
        }
        ptile[i] = (int16_t)v;
    }
}

// ------------------------------------------------------------------ mc -----

// 8-tap kernel as two packed dwords (signed bytes), or {0,0} for m == 0
struct Taps { uint32_t lo, hi; const signed char *k; };
__device__ __forceinline__ Taps get_taps(int t, int m, int len) {
    Taps r{0, 0, nullptr};
    const signed char *k = subpel_kernel(t, m, len);
    r.k = k;
    if (k) {
        r.lo = (uint8_t)k[0] | (uint32_t)(uint8_t)k[1] << 8 | (uint32_t)(uint8_t)k[2] << 16 | (uint32_t)(uint8_t)k[3] << 24;
        r.hi = (uint8_t)k[4] | (uint32_t)(uint8_t)k[5] << 8 | (uint32_t)(uint8_t)k[6] << 16 | (uint32_t)(uint8_t)k[7] << 24;
    }
    return r;
}

// Horizontal 8-tap sum over footprint bytes [boff, boff+8) of an 8bpc row
// (dword-aligned row start): v_alignbyte to the window, then two v_dot4 on
// bias-shifted bytes (p ^ 0x80 == p - 128; taps sum to 64 -> + 128 * 64).
__device__ __forceinline__ int hsum8(const uint8_t *row, int boff, const Taps &t) {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(row) + (boff >> 2);
    const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
    const int s = boff & 3;
    const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, s) ^ 0x80808080u;
    const uint32_t w1 = __builtin_amdgcn_alignbyte(d2, d1, s) ^ 0x80808080u;
    int acc = __builtin_amdgcn_sdot4((int)w0, (int)t.lo, 0, false);
    acc = __builtin_amdgcn_sdot4((int)w1, (int)t.hi, acc, false);
    return acc + 128 * 64;
}
__device__ __forceinline__ int hsum16(const uint16_t *row, const Taps &t) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += t.k[i] * (int)row[i];
    return s;
}

// ---------------------------------------------------------------- kernel --

template <int BPC, int TX>
__device__ __forceinline__ void recon_units(const ReconArgs<BPC> &a, int first, int count, uint8_t *wave_lds) {
    using CL = Cls<TX>;
    using SL = Slot<BPC, TX>;
    using P = typename Px<BPC>::pixel;
    using TT = typename Tmp<BPC>::T;
    constexpr int W = CL::W, H = CL::H, SH = CL::SH, G = CL::G, B = BPC / 8;
    const int lane = threadIdx.x & 63;
    const int g = lane / G, l = lane % G;
    if (g >= count) return;

    const Dav1dGpuUnit u = a.units[first + g];
    uint8_t *slot = wave_lds + g * SL::BYTES;
    TT *tmp = reinterpret_cast<TT *>(slot);
    int16_t *restile = reinterpret_cast<int16_t *>(slot);     // aliases tmp (read before written)
    P *otile = reinterpret_cast<P *>(slot);                    // aliases restile, same index order
    uint8_t *srcl = slot + SL::TMP;
    const int plane = u.plane;
    const int bdmax = a.bdmax;
    const int ib = Px<BPC>::ibits(bdmax);
    const int PB = Px<BPC>::PBIAS;
    const int pred = u.pred;
    const bool inter = pred == DGPU_PRED_INTER || pred == DGPU_PRED_INTER_AVG;
    const bool comp = pred == DGPU_PRED_INTER_AVG;
    const int txtp = u.txtp;
    const bool nores = txtp == DGPU_NO_RESIDUAL;
    const bool dconly = !nores && u.nzw == 0;

    // ---------------- P1: issue every global load of the unit ----------------
    int sk0 = 0, sk1 = 0;   // byte skew of each footprint in its LDS rows
    if (inter && !(a.ablate & 1)) {
        constexpr int TOT = (H + 7) * SL::NDW;
        constexpr int NIT = (TOT + G - 1) / G;
        uint32_t v0[NIT], v1[NIT];
        uintptr_t base[2];
        int rsb[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int r = k ? u.p.inter.ref[1] : u.p.inter.ref[0];
            const int rs = a.ref_stride[r][plane];
            const P *org = a.ref[r][plane] + (k ? u.p.inter.src_off[1] : u.p.inter.src_off[0]) - 3 * rs - 3;
            const uintptr_t ad = reinterpret_cast<uintptr_t>(org);
            base[k] = ad & ~(uintptr_t)3;
            rsb[k] = rs * B;
            if (k) sk1 = (int)(ad & 3); else sk0 = (int)(ad & 3);
        }
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int i = l + it * G;
            const int row = i / SL::NDW, d = i - row * SL::NDW;
            if (i < TOT) {
                v0[it] = reinterpret_cast<const uint32_t *>(base[0] + (intptr_t)row * rsb[0])[d];
                if (comp) v1[it] = reinterpret_cast<const uint32_t *>(base[1] + (intptr_t)row * rsb[1])[d];
            }
        }
        uint32_t *f0 = reinterpret_cast<uint32_t *>(srcl);
        uint32_t *f1 = reinterpret_cast<uint32_t *>(srcl + SL::FP);
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int i = l + it * G;
            if (i < TOT) {
                f0[i] = v0[it];
                if (comp) f1[i] = v1[it];
            }
        }
    }
    int16_t *e = reinterpret_cast<int16_t *>(srcl);            // intra: topleft[-2h..2w]
    int16_t *fe = e + SL::EDGE;                                  // prepared edge
    int16_t *ptile = fe + SL::EDGE;                              // intra prediction W x H
    if (pred == DGPU_PRED_INTRA) {
        const P *es = a.edges + u.p.intra.edge_off - 2 * H;
        for (int i = l; i < SL::EDGE; i += G) e[i] = es[i];
    }
    // coefficient row for P3 (lane y owns row y), compact column-major region
    typename Px<BPC>::coef *cf = a.coef + u.coef_off;
    int c[W];
    const bool rowlane = !nores && !dconly && l < SH && !(a.ablate & 8);
    if (rowlane) {
        const int nzw = u.nzw, nzh = u.nzh;
#pragma unroll
        for (int x = 0; x < W; x++) {
            int v = (x < nzw && l < nzh) ? (int)cf[l + x * nzh] : 0;
            c[x] = CL::RECT2 ? r8s(v) : v;
        }
        if (a.zero_coefs && l < nzh)
            for (int x = 0; x < nzw; x++) cf[l + x * nzh] = 0;
    }
    int dcres = 0;
    if (dconly) {  // src/itx_tmpl.c:53-65
        int dc = cf[0];
        if (CL::RECT2) dc = r8s(dc);
        dc = r8s(dc);
        dc = (dc + ((1 << CL::SHIFT) >> 1)) >> CL::SHIFT;
        dcres = (dc * 181 + 128 + 2048) >> 12;
    }
    wave_sync();
    if (dconly && a.zero_coefs && l == 0) cf[0] = 0;

    // ---------------- P2: intra prediction into ptile ----------------
    if (pred == DGPU_PRED_INTRA && !(a.ablate & 4)) {
        intra_unit<BPC, TX>(u, e, fe, ptile, l, bdmax);
        wave_sync();
    }

    // ---------------- P3 / P4: inverse transform -> residual tile --------------
    const Clip rc = ItxClip<BPC>::row(bdmax), cc = ItxClip<BPC>::col(bdmax);
    if (rowlane) {
        tx1d<W, 1>(kind_h(txtp), c, rc);
        constexpr int RND = (1 << CL::SHIFT) >> 1;
#pragma unroll
        for (int x = 0; x < W; x++) tmp[x * SL::TP + l] = (TT)cc((c[x] + RND) >> CL::SHIFT);
    }
    wave_sync();
    const bool haveres = !nores && !dconly && !(a.ablate & 8);
    if (haveres && l < W) {
        int col[H];
#pragma unroll
        for (int y = 0; y < H; y++) col[y] = y < SH ? (int)tmp[l * SL::TP + y] : 0;
        tx1d<H, 1>(kind_v(txtp), col, cc);
#pragma unroll
        for (int y = 0; y < H; y++) restile[y * W + l] = (int16_t)((col[y] + 8) >> 4);
    }
    wave_sync();

    // ---------------- P5: mc horizontal pass -> int16 intermediate tiles ----------
    const int f2d = inter ? u.p.inter.filter2d : 0;
    const bool bil = f2d == DGPU_FILTER_2D_BILINEAR;
    // filter_type = type_h | type_v << 2 per Filter2d (src/mc_tmpl.c:376-384)
    const int ftype = bil ? 0 : (int)((0x951a62840ull >> (4 * f2d)) & 15);
    const int bw = u.bw4 * 4, bh = u.bh4 * 4;
    constexpr int FPP = SL::FPB / B;   // footprint pitch in pixels
    int16_t *mid0 = reinterpret_cast<int16_t *>(srcl + 2 * SL::FP);
    int16_t *mid1 = reinterpret_cast<int16_t *>(srcl + 2 * SL::FP + SL::MID);
    Taps th0{}, tv0{}, th1{}, tv1{};
    int mx0 = 0, my0 = 0, mx1 = 0, my1 = 0;
    if (inter) {
        mx0 = u.p.inter.mx[0]; my0 = u.p.inter.my[0];
        mx1 = u.p.inter.mx[1]; my1 = u.p.inter.my[1];
        if (!bil) {
            th0 = get_taps(ftype & 3, mx0, bw); tv0 = get_taps(ftype >> 2, my0, bh);
            th1 = get_taps(ftype & 3, mx1, bw); tv1 = get_taps(ftype >> 2, my1, bh);
        }
    }
    if (inter && !bil && !(a.ablate & 2)) {
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (k == 1 && !comp) break;
            const Taps &th = k ? th1 : th0;
            const Taps &tv = k ? tv1 : tv0;
            if (!th.k) continue;
            const uint8_t *F = srcl + k * SL::FP;
            const int skp = (k ? sk1 : sk0);
            int16_t *M = k ? mid1 : mid0;
            // rows needed: all H+7 for hv, rows 3..H+2 for h-only
            const int r0 = tv.k ? 0 : 3;
            const int nrows = tv.k ? H + 7 : H;
            constexpr int NE = ((H + 7) * W + G - 1) / G;
#pragma unroll
            for (int it = 0; it < NE; it++) {
                const int i = l + it * G;
                if (i < nrows * W) {
                    const int r = r0 + i / W, x = i % W;
                    int s;
                    if constexpr (BPC == 8) s = hsum8(F + r * SL::FPB, skp + x, th);
                    else s = hsum16(reinterpret_cast<const uint16_t *>(F + r * SL::FPB) + (skp >> 1) + x, th);
                    int m;
                    if (tv.k) m = rnd_sh(s, 6 - ib);                                   // hv intermediate
                    else if (comp) m = rnd_sh(s, 6 - ib) - PB;                         // prep h-only
                    else m = clampi((s + 32 + ((1 << (6 - ib)) >> 1)) >> 6, 0, bdmax); // put h-only
                    M[r * W + x] = (int16_t)m;
                }
            }
        }
        wave_sync();
    }

    // ---------------- P6: vertical pass / blend / add residual -> output tile -------
    {
        constexpr int NO = (W * H + G - 1) / G;
        P *dstp = a.dst[plane] + u.dst_off;
        const int ds = a.dst_stride[plane];
#pragma unroll
        for (int it = 0; it < NO; it++) {
            const int i = l + it * G;
            if (i >= W * H) break;
            const int y = i / W, x = i % W;
            int p;
            if (inter) {
                int o[2];
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    if (k == 1 && !comp) { o[1] = 0; break; }
                    const int mx = k ? mx1 : mx0, my = k ? my1 : my0;
                    const Taps &th = k ? th1 : th0;
                    const Taps &tv = k ? tv1 : tv0;
                    const P *F = reinterpret_cast<const P *>(srcl + k * SL::FP) + ((k ? sk1 : sk0) / B);
                    const int16_t *M = k ? mid1 : mid0;
                    int v;
                    if (a.ablate & 2) {
                        v = F[(y + 3) * FPP + x + 3];
                    } else if (bil) {   // put_bilin_c / prep_bilin_c, src/mc_tmpl.c:395-546
                        const P *s0 = F + (y + 3) * FPP + x + 3;
                        if (mx && my) {
                            const int m0 = (int16_t)rnd_sh(16 * s0[0] + mx * (s0[1] - s0[0]), 4 - ib);
                            const int m1 = (int16_t)rnd_sh(16 * s0[FPP] + mx * (s0[FPP + 1] - s0[FPP]), 4 - ib);
                            const int t = 16 * m0 + my * (m1 - m0);
                            v = comp ? rnd_sh(t, 4) - PB : clampi(rnd_sh(t, 4 + ib), 0, bdmax);
                        } else if (mx) {
                            const int px = rnd_sh(16 * s0[0] + mx * (s0[1] - s0[0]), 4 - ib);
                            v = comp ? px - PB : clampi(rnd_sh(px, ib), 0, bdmax);
                        } else if (my) {
                            const int t = 16 * s0[0] + my * (s0[FPP] - s0[0]);
                            v = comp ? rnd_sh(t, 4 - ib) - PB : clampi(rnd_sh(t, 4), 0, bdmax);
                        } else {
                            v = comp ? ((int)s0[0] << ib) - PB : (int)s0[0];
                        }
                    } else if (th.k && tv.k) {   // put/prep_8tap_c hv, src/mc_tmpl.c:126-150, :232-258
                        const int16_t *mc = M + y * W + x;
                        int t = 0;
#pragma unroll
                        for (int q = 0; q < 8; q++) t += tv.k[q] * mc[q * W];
                        v = comp ? rnd_sh(t, 6) - PB : clampi(rnd_sh(t, 6 + ib), 0, bdmax);
                    } else if (th.k) {           // h-only, already final in M
                        v = M[(y + 3) * W + x];
                    } else if (tv.k) {           // v-only, src/mc_tmpl.c:161-168, :270-279
                        const P *s0 = F + y * FPP + x + 3;
                        int t = 0;
#pragma unroll
                        for (int q = 0; q < 8; q++) t += tv.k[q] * (int)s0[q * FPP];
                        v = comp ? rnd_sh(t, 6 - ib) - PB : clampi(rnd_sh(t, 6), 0, bdmax);
                    } else {                     // integer position
                        const int s0 = F[(y + 3) * FPP + x + 3];
                        v = comp ? (s0 << ib) - PB : s0;
                    }
                    o[k] = v;
                }
                // avg_c, src/mc_tmpl.c:587-602
                p = comp ? clampi((o[0] + o[1] + (1 << ib) + 2 * PB) >> (ib + 1), 0, bdmax) : o[0];
            } else if (pred == DGPU_PRED_INTRA) {
                p = ptile[i];
            } else {
                p = dstp[y * ds + x];   // PRED_NONE: residual onto the picture
            }
            const int r = haveres ? restile[i] : dcres;
            otile[i] = (P)clampi(p + r, 0, bdmax);
        }
    }
    wave_sync();

    // ---------------- P7: store the finished unit rows ----------------
    {
        constexpr int RB = W * B;                       // bytes per row
        constexpr int CB = RB >= 16 ? 16 : RB;          // bytes per store
        constexpr int NC = RB / CB;                     // stores per row
        constexpr int NS = (H * NC + G - 1) / G;
        uint8_t *dbase = reinterpret_cast<uint8_t *>(a.dst[plane] + u.dst_off);
        const int dsb = a.dst_stride[plane] * B;
        const uint8_t *ob = reinterpret_cast<const uint8_t *>(otile);
#pragma unroll
        for (int it = 0; it < NS; it++) {
            const int i = l + it * G;
            if (i >= H * NC) break;
            const int y = i / NC, cx = i % NC;
            uint8_t *dp = dbase + (intptr_t)y * dsb + cx * CB;
            const uint8_t *sp = ob + y * RB + cx * CB;
            if constexpr (CB == 16) *reinterpret_cast<uint4 *>(dp) = *reinterpret_cast<const uint4 *>(sp);
            else if constexpr (CB == 8) *reinterpret_cast<uint2 *>(dp) = *reinterpret_cast<const uint2 *>(sp);
            else *reinterpret_cast<uint32_t *>(dp) = *reinterpret_cast<const uint32_t *>(sp);
        }
    }
}

}  // namespace dgpu
