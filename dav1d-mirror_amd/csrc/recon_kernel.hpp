// recon_kernel.hpp -- the batch tier: one grid launch reconstructs a frame's
// worth of transform-block units (include/dav1d_gpu.h, Dav1dGpuUnit).
//
// Per unit the work the reference does in recon_b_inter / recon_b_intra
// (src/recon_tmpl.c:1598, :1195) for one transform block: the prediction
// (mc put, or mct x2 + avg, src/recon_tmpl.c:957-1059, :1845; or intra_pred,
// :1294) followed by inv_txfm_add (:816 / :1347), fused so the prediction
// never round-trips through HBM.
//
// Mapping (wave64).  Units are sorted by transform size class on the host.
// A wave owns U = 64 / G units of one class, G = max(w, min(h, 32)) lanes
// each:
//   A  stage the unit's source: the (w+7) x (h+7) reference footprint(s)
//      (dword loads, kept at their byte skew) or the intra edge array,
//      into this unit's LDS slot; directional / filter-intra edges are
//      then prepared in LDS.
//   B  row pass: lane y (< min(h,32)) loads coefficient row y, runs the
//      horizontal 1-D transform in VGPRs, rounds/clips to the column range
//      and writes the row transposed into LDS.
//   C  column pass: lane x (< w) pulls column x from LDS, runs the vertical
//      1-D transform, then streams the prediction of column x (an 8-tap
//      vertical window over per-row horizontal sums, or the intra formula),
//      adds the residual, clips, and stores the finished pixels once.
// No workgroup barrier is needed: every LDS hand-off is inside one wave.
#pragma once
#include "dav1d_gpu.h"
#include "dsp_common.hpp"

namespace dgpu {

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
    int wave_start[DGPU_N_RECT_TX_SIZES + 1];   // cumulative waves per class
    int bdmax;
    int zero_coefs;
    int ablate;   // debug-only phase mask (DAV1D_GPU_ABLATE); 0 in production
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int TX> struct Cls {
    static constexpr int W = tx_info(TX).w, H = tx_info(TX).h, SHIFT = tx_info(TX).shift;
    static constexpr int SW = W < 32 ? W : 32, SH = H < 32 ? H : 32;
    static constexpr int G = W > SH ? W : SH;
    static constexpr int U = 64 / G;
    static constexpr bool RECT2 = W * 2 == H || H * 2 == W;
    static constexpr bool BIG = W == 64 || H == 64;
};

template <int BPC> struct Tmp { using T = int32_t; };
template <> struct Tmp<8> { using T = int16_t; };  // 8-bit column range is int16

// LDS slot layout of one unit (bytes)
template <int BPC, int TX> struct Slot {
    using CL = Cls<TX>;
    static constexpr int B = BPC / 8;
    static constexpr int TP = CL::SH + 1;                           // tmp pitch (elements)
    static constexpr int TMP = ((CL::W * TP * (int)sizeof(typename Tmp<BPC>::T)) + 15) & ~15;
    static constexpr int FPB = ((CL::W + 7) * B + 6 + 3) & ~3;       // footprint pitch (bytes), room for a 3-byte skew
    static constexpr int FP = (((CL::H + 7) * FPB) + 15) & ~15;      // one footprint
    static constexpr int EDGE = 2 * CL::H + 2 * CL::W + 1;          // topleft[-2h..2w]
    static constexpr int INTRA = ((2 * EDGE + 2 * EDGE + 2 * CL::W * CL::H) + 15) & ~15;
    static constexpr int SRC = 2 * FP > INTRA ? 2 * FP : INTRA;
    static constexpr int BYTES = TMP + SRC;
    static constexpr int WAVE = CL::U * BYTES;
};

template <int BPC, int... TX> struct MaxWave;
template <int BPC, int T0> struct MaxWave<BPC, T0> { static constexpr int v = Slot<BPC, T0>::WAVE; };
template <int BPC, int T0, int... TR> struct MaxWave<BPC, T0, TR...> {
    static constexpr int a = Slot<BPC, T0>::WAVE, b = MaxWave<BPC, TR...>::v;
    static constexpr int v = a > b ? a : b;
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

// Intra unit state prepared in phase A.
struct IntraPrep {
    int mode, ang, is_sm, filt;
    int up, upl, d1, d2, maxb, dc;
};

// ---------------------------------------------------------------- kernel --

template <int BPC, int TX>
__device__ __forceinline__ void recon_units(const ReconArgs<BPC> &a, int first, int count, uint8_t *wave_lds) {
    using CL = Cls<TX>;
    using SL = Slot<BPC, TX>;
    using P = typename Px<BPC>::pixel;
    using TT = typename Tmp<BPC>::T;
    constexpr int W = CL::W, H = CL::H, SH = CL::SH, G = CL::G;
    constexpr int B = BPC / 8;
    const int lane = threadIdx.x & 63;
    const int g = lane / G, l = lane % G;
    const bool active = g < count;
    if (!active) return;

    const Dav1dGpuUnit u = a.units[first + g];
    uint8_t *slot = wave_lds + g * SL::BYTES;
    TT *tmp = reinterpret_cast<TT *>(slot);
    uint8_t *srcl = slot + SL::TMP;
    const int plane = u.plane;
    const int bdmax = a.bdmax;
    const int ib = Px<BPC>::ibits(bdmax);

    // ---------------- phase A: stage sources ----------------
    const int nref = u.pred == DGPU_PRED_INTER_AVG ? 2 : u.pred == DGPU_PRED_INTER ? 1 : 0;
    int skew0 = 0, skew1 = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        if (k >= nref || (a.ablate & 1)) break;
        const int r = k ? u.p.inter.ref[1] : u.p.inter.ref[0];
        const int rs = a.ref_stride[r][plane];
        const P *org = a.ref[r][plane] + (k ? u.p.inter.src_off[1] : u.p.inter.src_off[0]) - 3 * rs - 3;
        const uintptr_t ad = reinterpret_cast<uintptr_t>(org);
        const uintptr_t a0 = ad & ~(uintptr_t)3;
        const int sk = (int)(ad - a0) / B;
        if (k) skew1 = sk; else skew0 = sk;
        const int ndw = ((int)(ad - a0) + (W + 7) * B + 3) >> 2;
        const float inv = 1.0f / (float)ndw;
        uint32_t *dstl = reinterpret_cast<uint32_t *>(srcl + k * SL::FP);
        const int total = (H + 7) * ndw;
        for (int i = l; i < total; i += G) {
            const int row = (int)(((float)i + 0.5f) * inv), d = i - row * ndw;
            const uint32_t *s = reinterpret_cast<const uint32_t *>(a0 + (intptr_t)row * rs * B);
            dstl[row * (SL::FPB / 4) + d] = s[d];
        }
    }
    int16_t *e = reinterpret_cast<int16_t *>(srcl);             // topleft[-2h..2w] -> e[0..]
    int16_t *fe = e + SL::EDGE;                                   // filtered / upsampled edge
    int16_t *ftile = fe + SL::EDGE;                               // filter-intra W x H
    const int16_t *tl = e + 2 * H;                                // topleft[0]
    IntraPrep ip{};
    if (u.pred == DGPU_PRED_INTRA) {
        const P *es = a.edges + u.p.intra.edge_off;
        for (int i = l; i < SL::EDGE; i += G) e[i] = es[i - 2 * H];
        ip.mode = u.p.intra.mode;
        ip.ang = u.p.intra.angle & 511;
        ip.is_sm = (u.p.intra.angle >> 9) & 1;
        ip.filt = u.p.intra.angle >> 10;
    }
    wave_sync();
    if (u.pred == DGPU_PRED_INTRA) {
        const int mode = ip.mode;
        if (mode == DGPU_Z1_PRED) {   // src/ipred_tmpl.c:408-443
            ip.d1 = dspt_dr_deriv[ip.ang >> 1];
            ip.up = ip.filt ? ip_upsample(W + H, 90 - ip.ang, ip.is_sm) : 0;
            const int st = (!ip.up && ip.filt) ? ip_strength(W + H, 90 - ip.ang, ip.is_sm) : 0;
            if (ip.up) {
                for (int o = l; o < 2 * (W + H) - 1; o += G) fe[o] = ip_up(tl + 1, o, W + H, -1, W + min(W, H), bdmax);
                ip.maxb = 2 * (W + H) - 2;
                ip.d1 <<= 1;
            } else if (st) {
                for (int i = l; i < W + H; i += G) fe[i] = ip_smooth(tl + 1, i, 0, W + H, -1, W + min(W, H), st);
                ip.maxb = W + H - 1;
            } else {
                for (int i = l; i < W + min(W, H); i += G) fe[i] = tl[1 + i];
                ip.maxb = W + min(W, H) - 1;
            }
        } else if (mode == DGPU_Z3_PRED) {   // src/ipred_tmpl.c:542-581
            ip.d1 = dspt_dr_deriv[(270 - ip.ang) >> 1];
            ip.up = ip.filt ? ip_upsample(W + H, ip.ang - 180, ip.is_sm) : 0;
            const int st = (!ip.up && ip.filt) ? ip_strength(W + H, ip.ang - 180, ip.is_sm) : 0;
            // fe holds the left edge bottom-up as the reference's left_out,
            // with fe[maxb] = the element read as left[-maxb]
            if (ip.up) {
                for (int o = l; o < 2 * (W + H) - 1; o += G)
                    fe[o] = ip_up(tl - (W + H), o, W + H, max(W - H, 0), W + H + 1, bdmax);
                ip.maxb = 2 * (W + H) - 2;
                ip.d1 <<= 1;
            } else if (st) {
                for (int i = l; i < W + H; i += G)
                    fe[i] = ip_smooth(tl - (W + H), i, 0, W + H, max(W - H, 0), W + H + 1, st);
                ip.maxb = W + H - 1;
            } else {
                ip.maxb = H + min(W, H) - 1;
                for (int i = l; i <= ip.maxb; i += G) fe[i] = tl[-1 - ip.maxb + i];
            }
        } else if (mode == DGPU_Z2_PRED) {   // src/ipred_tmpl.c:462-513
            ip.d2 = dspt_dr_deriv[(ip.ang - 90) >> 1];   // dy
            ip.d1 = dspt_dr_deriv[(180 - ip.ang) >> 1];  // dx
            ip.upl = ip.filt ? ip_upsample(W + H, 180 - ip.ang, ip.is_sm) : 0;
            ip.up = ip.filt ? ip_upsample(W + H, ip.ang - 90, ip.is_sm) : 0;
            int16_t *c = fe + 2 * H;   // corner
            if (ip.up) {
                for (int o = l; o < 2 * W + 1; o += G) c[o] = ip_up(tl, o, W + 1, 0, W + 1, bdmax);
            } else {
                const int st = ip.filt ? ip_strength(W + H, ip.ang - 90, ip.is_sm) : 0;
                for (int i = l; i < W; i += G)
                    c[1 + i] = st ? ip_smooth(tl + 1, i, 0, u.p.intra.max_w, -1, W, st) : tl[1 + i];
            }
            if (ip.upl) {
                for (int o = l; o < 2 * H + 1; o += G) c[-2 * H + o] = ip_up(tl - H, o, H + 1, 0, H + 1, bdmax);
            } else {
                const int st = ip.filt ? ip_strength(W + H, 180 - ip.ang, ip.is_sm) : 0;
                for (int i = l; i < H; i += G)
                    c[-H + i] = st ? ip_smooth(tl - H, i, H - u.p.intra.max_h, H, 0, H + 1, st) : tl[-H + i];
            }
            wave_sync();
            if (l == 0) c[0] = tl[0];
            if (ip.up) ip.d1 <<= 1;
            if (ip.upl) ip.d2 <<= 1;
        } else if (mode == DGPU_FILTER_PRED) {   // src/ipred_tmpl.c:617-655
            const signed char *taps = &dspt_filter_intra[(u.p.intra.angle & 511) * 56];
            constexpr int cw = W / 4, ch = H / 2;
            if constexpr (W <= 32 && H <= 32) {
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
                            const int16_t *up = ftile + (y - 1) * W + x;
                            p0 = x == 0 ? tl[-y] : up[-1];
                            p1 = up[0]; p2 = up[1]; p3 = up[2]; p4 = up[3];
                        }
                        p5 = x == 0 ? tl[-(y + 1)] : ftile[y * W + x - 1];
                        p6 = x == 0 ? tl[-(y + 2)] : ftile[(y + 1) * W + x - 1];
#pragma unroll
                        for (int k = 0; k < 8; k++) {
                            const signed char *tk = taps + k * 7;
                            const int acc = tk[0] * p0 + tk[1] * p1 + tk[2] * p2 + tk[3] * p3 +
                                            tk[4] * p4 + tk[5] * p5 + tk[6] * p6;
                            ftile[(y + (k >> 2)) * W + x + (k & 3)] = clampi((acc + 8) >> 4, 0, bdmax);
                        }
                    }
                    wave_sync();
                }
            }
        } else if (mode <= DGPU_DC_128_PRED && mode != DGPU_VERT_PRED && mode != DGPU_HOR_PRED) {
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
            ip.dc = (int)s;
        }
        wave_sync();
    }

    // intra prediction of the whole unit into the LDS tile, all G lanes
    // (src/ipred_tmpl.c:93-599); FILTER_PRED already filled it above
    if (u.pred == DGPU_PRED_INTRA && ip.mode != DGPU_FILTER_PRED && !(a.ablate & 4)) {
        const int mode = ip.mode;
        for (int i = l; i < W * H; i += G) {
            const int x = i % W, y = i / W;
            const int top = tl[1 + x], left = tl[-(1 + y)];
            int v;
            switch (mode) {
            case DGPU_VERT_PRED: v = top; break;
            case DGPU_HOR_PRED: v = left; break;
            case DGPU_PAETH_PRED: {
                const int c0 = tl[0], base = left + top - c0;
                const int dl = abs(left - base), dt = abs(top - base), dc = abs(c0 - base);
                v = (dl <= dt && dl <= dc) ? left : dt <= dc ? top : c0;
                break;
            }
            case DGPU_SMOOTH_PRED: {
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
                const int xpos = (y + 1) * ip.d1, frac = xpos & 0x3e;
                const int base = (xpos >> 6) + x * (1 + ip.up);
                v = base < ip.maxb ? (fe[base] * (64 - frac) + fe[base + 1] * frac + 32) >> 6 : fe[ip.maxb];
                break;
            }
            case DGPU_Z3_PRED: {
                const int ypos = (x + 1) * ip.d1, frac = ypos & 0x3e;
                const int base = (ypos >> 6) + y * (1 + ip.up);
                // left[-i] == fe[maxb - i]
                v = base < ip.maxb
                        ? (fe[ip.maxb - base] * (64 - frac) + fe[ip.maxb - base - 1] * frac + 32) >> 6
                        : fe[0];
                break;
            }
            case DGPU_Z2_PRED: {
                const int16_t *c = fe + 2 * H;
                const int xpos = ((1 + ip.up) << 6) - (y + 1) * ip.d1;
                const int bx = (xpos >> 6) + x * (1 + ip.up);
                int t;
                if (bx >= 0) {
                    const int fx = xpos & 0x3e;
                    t = c[bx] * (64 - fx) + c[bx + 1] * fx;
                } else {
                    const int ypos = (y << (6 + ip.upl)) - (x + 1) * ip.d2;
                    const int by = ypos >> 6, fy = ypos & 0x3e;
                    const int16_t *lft = c - (1 + ip.upl);
                    t = lft[-by] * (64 - fy) + lft[-(by + 1)] * fy;
                }
                v = (t + 32) >> 6;
                break;
            }
            default:  // DC family
                v = ip.dc;
                break;
            }
            ftile[y * W + x] = (int16_t)v;
        }
        wave_sync();
    }

    // ---------------- phase B: row transforms ----------------
    const int txtp = u.txtp;
    const bool nores = txtp == DGPU_NO_RESIDUAL;
    const bool dconly = !nores && u.nzw == 0;
    const Clip rc = ItxClip<BPC>::row(bdmax), cc = ItxClip<BPC>::col(bdmax);
    typename Px<BPC>::coef *cf = a.coef + u.coef_off;
    if (!nores && !dconly && l < SH && !(a.ablate & 8)) {
        const int nzw = u.nzw, nzh = u.nzh;
        int c[W];
#pragma unroll
        for (int x = 0; x < W; x++) {
            int v = (x < nzw && l < nzh) ? (int)cf[l + x * nzh] : 0;
            c[x] = CL::RECT2 ? r8s(v) : v;
        }
        if (a.zero_coefs && l < nzh)
            for (int x = 0; x < nzw; x++) cf[l + x * nzh] = 0;
        tx1d<W, 1>(kind_h(txtp), c, rc);
        constexpr int RND = (1 << CL::SHIFT) >> 1;
#pragma unroll
        for (int x = 0; x < W; x++) tmp[x * SL::TP + l] = (TT)cc((c[x] + RND) >> CL::SHIFT);
    }
    wave_sync();

    // ---------------- phase C: column transform + prediction + store -------
    if (l >= W) return;
    int res[H];
    if (nores || (a.ablate & 8)) {
#pragma unroll
        for (int y = 0; y < H; y++) res[y] = (a.ablate & 8) ? (int)tmp[y] : 0;
    } else if (dconly) {  // src/itx_tmpl.c:53-65
        int dc = cf[0];
        if (a.zero_coefs) {
            wave_sync();
            if (l == 0) cf[0] = 0;
        }
        if (CL::RECT2) dc = r8s(dc);
        dc = r8s(dc);
        dc = (dc + ((1 << CL::SHIFT) >> 1)) >> CL::SHIFT;
        dc = (dc * 181 + 128 + 2048) >> 12;
#pragma unroll
        for (int y = 0; y < H; y++) res[y] = dc;
    } else {
#pragma unroll
        for (int y = 0; y < H; y++) res[y] = y < SH ? (int)tmp[l * SL::TP + y] : 0;
        tx1d<H, 1>(kind_v(txtp), res, cc);
#pragma unroll
        for (int y = 0; y < H; y++) res[y] = (res[y] + 8) >> 4;
    }

    const int x = l;
    P *d = a.dst[plane] + u.dst_off + x;
    const int ds = a.dst_stride[plane];

    if (u.pred == DGPU_PRED_INTER || u.pred == DGPU_PRED_INTER_AVG) {
        const int f2d = u.p.inter.filter2d;
        const bool bil = f2d == DGPU_FILTER_2D_BILINEAR;
        // filter_type = type_h | type_v << 2 per Filter2d (src/mc_tmpl.c:376-384)
        const int ftype = bil ? 0 : (int)((0x951a62840ull >> (4 * f2d)) & 15);
        const int bw = u.bw4 * 4, bh = u.bh4 * 4;
        const bool comp = u.pred == DGPU_PRED_INTER_AVG;
        const int PB = Px<BPC>::PBIAS;
        int p0[H];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (k == 1 && !comp) break;
            const int mx = k ? u.p.inter.mx[1] : u.p.inter.mx[0];
            const int my = k ? u.p.inter.my[1] : u.p.inter.my[0];
            const signed char *fh = subpel_kernel(ftype & 3, mx, bw);
            const signed char *fv = subpel_kernel(ftype >> 2, my, bh);
            const P *F = reinterpret_cast<const P *>(srcl + k * SL::FP) + (k ? skew1 : skew0) + x;
            constexpr int FPP = SL::FPB / B;   // footprint pitch in pixels
            auto hsum = [&](int r) {           // 8-tap horizontal sum of footprint row r
                int s = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) s += fh[t] * (int)F[r * FPP + t];
                return s;
            };
            auto vsum_src = [&](int y) {
                int s = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) s += fv[t] * (int)F[(y + t) * FPP + 3];
                return s;
            };
            int out[H];
            if (a.ablate & 2) {
#pragma unroll
                for (int y = 0; y < H; y++) out[y] = F[y * FPP];
            } else if (bil) {        // put_bilin_c / prep_bilin_c, src/mc_tmpl.c:395-546
                auto bl = [&](int r, int c0, int c1, int m) {
                    const int p = F[r * FPP + c0], q = F[r * FPP + c1];
                    return 16 * p + m * (q - p);
                };
#pragma unroll
                for (int y = 0; y < H; y++) {
                    int v;
                    if (mx && my) {
                        const int m0 = (int16_t)rnd_sh(bl(y + 3, 3, 4, mx), 4 - ib);
                        const int m1 = (int16_t)rnd_sh(bl(y + 4, 3, 4, mx), 4 - ib);
                        const int s = 16 * m0 + my * (m1 - m0);
                        v = comp ? rnd_sh(s, 4) - PB : clampi(rnd_sh(s, 4 + ib), 0, bdmax);
                    } else if (mx) {
                        const int px = rnd_sh(bl(y + 3, 3, 4, mx), 4 - ib);
                        v = comp ? px - PB : clampi(rnd_sh(px, ib), 0, bdmax);
                    } else if (my) {
                        const int p = F[(y + 3) * FPP + 3], q = F[(y + 4) * FPP + 3];
                        const int s = 16 * p + my * (q - p);
                        v = comp ? rnd_sh(s, 4 - ib) - PB : clampi(rnd_sh(s, 4), 0, bdmax);
                    } else {
                        const int p = F[(y + 3) * FPP + 3];
                        v = comp ? (p << ib) - PB : p;
                    }
                    out[y] = v;
                }
            } else if (fh && fv) {   // put/prep_8tap_c hv paths
                int win[8];
#pragma unroll
                for (int t = 0; t < 7; t++) win[t] = (int16_t)rnd_sh(hsum(t), 6 - ib);
#pragma unroll
                for (int y = 0; y < H; y++) {
                    win[7] = (int16_t)rnd_sh(hsum(y + 7), 6 - ib);
                    int s = 0;
#pragma unroll
                    for (int t = 0; t < 8; t++) s += fv[t] * win[t];
                    out[y] = comp ? rnd_sh(s, 6) - PB : clampi(rnd_sh(s, 6 + ib), 0, bdmax);
#pragma unroll
                    for (int t = 0; t < 7; t++) win[t] = win[t + 1];
                }
            } else if (fh) {
#pragma unroll
                for (int y = 0; y < H; y++) {
                    const int s = hsum(y + 3);
                    out[y] = comp ? rnd_sh(s, 6 - ib) - PB
                                  : clampi((s + 32 + ((1 << (6 - ib)) >> 1)) >> 6, 0, bdmax);
                }
            } else if (fv) {
#pragma unroll
                for (int y = 0; y < H; y++) {
                    const int s = vsum_src(y);
                    out[y] = comp ? rnd_sh(s, 6 - ib) - PB : clampi(rnd_sh(s, 6), 0, bdmax);
                }
            } else {
#pragma unroll
                for (int y = 0; y < H; y++) {
                    const int v = F[(y + 3) * FPP + 3];
                    out[y] = comp ? (v << ib) - PB : v;
                }
            }
            if (k == 0) {
#pragma unroll
                for (int y = 0; y < H; y++) p0[y] = out[y];
            } else {  // avg_c, src/mc_tmpl.c:587-602
#pragma unroll
                for (int y = 0; y < H; y++)
                    p0[y] = clampi((p0[y] + out[y] + (1 << ib) + 2 * PB) >> (ib + 1), 0, bdmax);
            }
        }
#pragma unroll
        for (int y = 0; y < H; y++) d[y * ds] = (P)clampi(p0[y] + res[y], 0, bdmax);
        return;
    }

    if (u.pred == DGPU_PRED_INTRA) {
#pragma unroll
        for (int y = 0; y < H; y++) d[y * ds] = (P)clampi(ftile[y * W + x] + res[y], 0, bdmax);
        return;
    }

    // DGPU_PRED_NONE: residual onto the existing pixels
#pragma unroll
    for (int y = 0; y < H; y++) d[y * ds] = (P)clampi((int)d[y * ds] + res[y], 0, bdmax);
}

}  // namespace dgpu
