// tile_kernel.hpp -- the superblock-tile batch kernel (Dav1dGpuTileBatch).
//
// One workgroup (4 waves) reconstructs one tile: a plane's rectangle of at
// most 64x64 pixels, i.e. what recon_b_inter / recon_b_intra produce for
// the blocks of one superblock (src/recon_tmpl.c:1598, :1195).
//
//   P0  staging: the tile's coefficients and intra edges (16-B chunks into
//       LDS), a zeroed residual tile `acc`, and the lane maps (lane -> tx
//       record, lane -> pred record) from the producer's lane bases.
//   P1  inverse transforms (src/itx_tmpl.c:40-100): a transform block owns
//       max(w, min(h, 32)) lanes; lane r runs row r (rows >= nzh are zero
//       and skipped) into the tile, then lane x runs column x, in place.
//       Residuals land at their picture position in `acc` (int16 at 8 bpc).
//   P2  predictions, added to the residual and clipped in `acc`:
//       * cooperative groups (INTRA, CFL): edge preparation and DC sums over
//         the group's lanes, then 4x2 tasks;
//       * independent 4 x R tasks (mc put / compound, PAL, NONE, WARP,
//         inter-intra), R = 8 (8 bpc, h >= 8) or 4.  The mc filter runs as a
//         sliding window in registers: R + 7 footprint rows, each one aligned
//         16-byte load (+ v_alignbyte), 4 horizontal outputs per row by two
//         v_dot4 each, then the 8 vertical taps by v_dot2 on row pairs.
//         Lanes of one block take adjacent 4-column quads, so a footprint
//         row is one cache line for the whole block's lanes.  Footprints that
//         leave the reference plane are clamped to it (emu_edge_c,
//         src/mc_tmpl.c:827-875, applied as recon_tmpl.c:986-999 does).
//   P3  one store of the tile: whole rows, 16 bytes per lane.
// Workgroup barriers separate the phases; inside P1 and the cooperative
// groups every LDS hand-off stays within one wave.
#pragma once
#include "recon_kernel.hpp"

namespace dgpu {

// DGPU_TILE_TRACE builds: per tile and wave, s_memtime at the phase
// boundaries into TileArgs::trace ([tile][wave][8]; tools/tile_trace.py)
#ifndef DGPU_TILE_TRACE
#define DGPU_TILE_TRACE 0
#endif

constexpr int kTileThreads = 256;
constexpr int kTileMaxLanesTx = 1024;    // sum of max(w, min(h,32)) over a 64x64 tile's tx blocks
constexpr int kTileMaxLanesPred = 1024;  // cooperative (<= 512 + pad) + task (<= 256) lanes

// residual / output tile: int16 at 8 bpc (every row-pass value and residual
// fits: both are clipped to int16), int32 at 16 bpc.  Row strides are odd
// in dwords so lanes walking rows (row pass, column pass) hit distinct banks.
template <int BPC> struct TAcc { using T = int16_t; static constexpr int S = 66; };
template <> struct TAcc<16> { using T = int32_t; static constexpr int S = 65; };

// transform lanes of a tx size: one per row (row pass) and one per column
// (column pass) of the same group
__host__ __device__ constexpr int tile_tx_lanes(int tx) {
    return cmax(tx_info(tx).w, cmin(tx_info(tx).h, 32));
}

// LDS layout of one workgroup (bytes)
template <int BPC> struct TileLds {
    using A = typename TAcc<BPC>::T;
    static constexpr int B = BPC / 8;
    static constexpr int CB = sizeof(typename Px<BPC>::coef);
    static constexpr int ACC = a16(64 * TAcc<BPC>::S * (int)sizeof(A));
    // staged coefficients (P1), then the prepared intra edges (P2: int16,
    // one per raw edge pixel, at the raw edge's index)
    static constexpr int CF = a16(cmax(4096 * CB + 32, DGPU_TILE_MAX_EDGE * 2 + 32));
    static constexpr int EDGE = a16(DGPU_TILE_MAX_EDGE * B + 32);
    static constexpr int TXMAP = kTileMaxLanesTx;
    static constexpr int PMAP = kTileMaxLanesPred;
    static constexpr int WARPT = 193 * 8 + 8;
    static constexpr int O_ACC = 0, O_CF = ACC, O_EDGE = O_CF + CF, O_TXMAP = O_EDGE + EDGE;
    static constexpr int O_PMAP = O_TXMAP + TXMAP, O_WARP = O_PMAP + PMAP;
    static constexpr int BYTES = a16(O_WARP + WARPT);
};

template <int BPC> struct TileArgs {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    P *dst[3];
    int dst_stride[3];                       // pixels
    const P *ref[DGPU_MAX_REFS * 3];
    int ref_stride[DGPU_MAX_REFS * 3];       // pixels
    int ref_w[DGPU_MAX_REFS * 3], ref_h[DGPU_MAX_REFS * 3];
    const Dav1dGpuTile *tiles;
    const Dav1dGpuPred *preds;
    const Dav1dGpuTx *txs;
    C *coef;
    const P *edges;
    const uint8_t *aux_pool;
    const P *cfl_luma;
    int cfl_luma_stride;   // pixels
    int cfl_ss;
    unsigned long long *trace;   // DGPU_TILE_TRACE builds only
    int tile0, n_tiles;   // this launch's tile range
    int bdmax;
    int zero_coefs;
#if DGPU_BOUNDS
    int bnd_noclamp;   // DAV1D_GPU_BND_NOCLAMP self-test: the round-3 lane maps (no padding init, raw indices)
#endif
};

// A record index read from the tile's LDS lane maps (pmap / txmap), clamped
// to the tile's record count.  DGPU_BOUNDS builds report every index at or
// past the count before clamping it (the stale-map mechanism of the round-3 /
// round-4 faults), and with the NOCLAMP self-test use it raw, so the range
// table sees where such a read would have landed.
#if DGPU_BOUNDS
static __device__ int g_dgpu_tile_index_hits;   // printed at most 256 times per process (its own count)
__device__ __noinline__ int tile_index(int i, int n, int noclamp, int which, int line) {
    if (i >= n && atomicAdd(&g_dgpu_tile_index_hits, 1) < 256)
        printf("DGPU_TILE_INDEX %s line %d index %d of %d block %d lane %d\n", which ? "pred" : "tx", line, i, n,
               (int)blockIdx.x, (int)(threadIdx.x & 63));
    return noclamp ? i : min(i, n - 1);
}
#define DGPU_TILE_INDEX(i, n, which) tile_index(i, n, a.bnd_noclamp, which, __LINE__)
#else
#define DGPU_TILE_INDEX(i, n, which) min(i, (n) - 1)
#endif

// the reference planes of a workgroup in LDS (lane-varying ref slots index it)
template <int BPC> struct TileRefTab {
    using P = typename Px<BPC>::pixel;
    const P *ref[DGPU_MAX_REFS * 3];
    int stride[DGPU_MAX_REFS * 3];
    int w[DGPU_MAX_REFS * 3], h[DGPU_MAX_REFS * 3];
};

// per-workgroup view of the tile
template <int BPC> struct TileCtx {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    using A = typename TAcc<BPC>::T;
    A *acc;                  // [64][S]
    const C *cf;             // staged coefficients (tile coef0 at index 0)
    const P *ed;             // staged edges (tile edge0 at index 0)
    int16_t *fe;             // prepared edges, parallel to ed
    const uint2 *wtab;       // warp filter table in LDS (tiles with WARP preds)
    const TileRefTab<BPC> *rt;
    int plane, bdmax, ib;
};

// ------------------------------------------------------------ transforms ---

// Row pass of one row: coefficients (compact, column-major, stride nzh) ->
// W-point transform (src/itx_tmpl.c:79-88) -> intermediate clip -> tile row.
template <int BPC, int W>
__device__ __forceinline__ void tile_row(const typename Px<BPC>::coef *cs, int nzw, int nzh, int r, int kind, int shift,
                                         bool rect2, Clip rc, Clip cc, typename TAcc<BPC>::T *arow) {
    constexpr int SW = W < 32 ? W : 32;
    int c[W];
#pragma unroll
    for (int x = 0; x < W; x++) {
        int v = 0;
        if (x < SW && x < nzw) v = cs[x * nzh + r];
        c[x] = rect2 ? r8s(v) : v;
    }
    tx1d<W, 1, BPC == 8>(kind, c, rc);
    const int rnd = (1 << shift) >> 1;
#pragma unroll
    for (int x = 0; x < W; x++) c[x] = cc((c[x] + rnd) >> shift);
    if constexpr (BPC == 8) {
#pragma unroll
        for (int x = 0; x < W; x += 2) *reinterpret_cast<uint32_t *>(arow + x) = pack16(c[x], c[x + 1]);
    } else {
#pragma unroll
        for (int x = 0; x < W; x++) arow[x] = c[x];
    }
}

// Column pass of one column, in place: rows >= nzh are zero (the row pass
// did not write them), the H-point transform, then (v + 8) >> 4.
template <int BPC, int H>
__device__ __forceinline__ void tile_col(typename TAcc<BPC>::T *acol, int nzh, int kind, Clip cc) {
    constexpr int S = TAcc<BPC>::S;
    constexpr int SH = H < 32 ? H : 32;
    int col[H];
#pragma unroll
    for (int y = 0; y < H; y++) col[y] = (y < SH && y < nzh) ? (int)acol[y * S] : 0;
    tx1d<H, 1, BPC == 8>(kind, col, cc);
#pragma unroll
    for (int y = 0; y < H; y++) acol[y * S] = (col[y] + 8) >> 4;
}

// --------------------------------------------------------------- output ---

// 4 predicted pixels of one row + the residual in `acc` -> clipped pixels in `acc`
template <int BPC>
__device__ __forceinline__ void acc_put4(typename TAcc<BPC>::T *a, const int *pv, int bdmax) {
    if constexpr (BPC == 8) {
        uint32_t *d = reinterpret_cast<uint32_t *>(a);
        const uint32_t r0 = d[0], r1 = d[1];
        const int o0 = clampi(pv[0] + (int)(int16_t)(r0 & 0xffff), 0, bdmax);
        const int o1 = clampi(pv[1] + ((int)r0 >> 16), 0, bdmax);
        const int o2 = clampi(pv[2] + (int)(int16_t)(r1 & 0xffff), 0, bdmax);
        const int o3 = clampi(pv[3] + ((int)r1 >> 16), 0, bdmax);
        d[0] = (uint32_t)o0 | (uint32_t)o1 << 16;
        d[1] = (uint32_t)o2 | (uint32_t)o3 << 16;
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) a[i] = clampi(pv[i] + a[i], 0, bdmax);
    }
}

// ------------------------------------------------------------------ intra --
// Run-time-size versions of the batch kernel's intra code: the lanes of a
// wave may belong to groups of different block sizes.

template <int BPC, typename P>
__device__ __forceinline__ IntraState tintra_prep(const Dav1dGpuPred &p, int W, int H, int G, const P *tl, int16_t *fe,
                                                  int l, int bdmax) {
    IntraState s{p.p.intra.mode, 0, 0, 0, 0, 0, 0};
    const int ang = p.p.intra.angle & 511, is_sm = (p.p.intra.angle >> 9) & 1, filt = p.p.intra.angle >> 10;
    if (s.mode == DGPU_Z1_PRED) {   // src/ipred_tmpl.c:408-443
        s.d1 = dspt_dr_deriv[ang >> 1];
        s.up = filt ? ip_upsample(W + H, 90 - ang, is_sm) : 0;
        const int st = (!s.up && filt) ? ip_strength(W + H, 90 - ang, is_sm) : 0;
        if (s.up) {
            for (int o = l; o < 2 * (W + H) - 1; o += G) fe[o] = ip_up(tl + 1, o, W + H, -1, W + min(W, H), bdmax);
            s.maxb = 2 * (W + H) - 2;
            s.d1 <<= 1;
        } else if (st) {
            for (int i = l; i < W + H; i += G) fe[i] = ip_smooth(tl + 1, i, 0, W + H, -1, W + min(W, H), st);
            s.maxb = W + H - 1;
        } else {
            for (int i = l; i < W + min(W, H); i += G) fe[i] = tl[1 + i];
            s.maxb = W + min(W, H) - 1;
        }
    } else if (s.mode == DGPU_Z3_PRED) {   // src/ipred_tmpl.c:542-581; fe[maxb - i] == left[-i]
        s.d1 = dspt_dr_deriv[(270 - ang) >> 1];
        s.up = filt ? ip_upsample(W + H, ang - 180, is_sm) : 0;
        const int st = (!s.up && filt) ? ip_strength(W + H, ang - 180, is_sm) : 0;
        if (s.up) {
            for (int o = l; o < 2 * (W + H) - 1; o += G)
                fe[o] = ip_up(tl - (W + H), o, W + H, max(W - H, 0), W + H + 1, bdmax);
            s.maxb = 2 * (W + H) - 2;
            s.d1 <<= 1;
        } else if (st) {
            for (int i = l; i < W + H; i += G) fe[i] = ip_smooth(tl - (W + H), i, 0, W + H, max(W - H, 0), W + H + 1, st);
            s.maxb = W + H - 1;
        } else {
            s.maxb = H + min(W, H) - 1;
            for (int i = l; i <= s.maxb; i += G) fe[i] = tl[-1 - s.maxb + i];
        }
    } else if (s.mode == DGPU_Z2_PRED) {   // src/ipred_tmpl.c:462-513
        s.d2 = dspt_dr_deriv[(ang - 90) >> 1];   // dy
        s.d1 = dspt_dr_deriv[(180 - ang) >> 1];  // dx
        s.upl = filt ? ip_upsample(W + H, 180 - ang, is_sm) : 0;
        s.up = filt ? ip_upsample(W + H, ang - 90, is_sm) : 0;
        int16_t *c = fe + 2 * H;   // corner
        if (s.up) {
            for (int o = l; o < 2 * W + 1; o += G) c[o] = ip_up(tl, o, W + 1, 0, W + 1, bdmax);
        } else {
            const int st = filt ? ip_strength(W + H, ang - 90, is_sm) : 0;
            for (int i = l; i < W; i += G) c[1 + i] = st ? ip_smooth(tl + 1, i, 0, p.p.intra.max_w, -1, W, st) : tl[1 + i];
        }
        if (s.upl) {
            for (int o = l; o < 2 * H + 1; o += G) c[-2 * H + o] = ip_up(tl - H, o, H + 1, 0, H + 1, bdmax);
        } else {
            const int st = filt ? ip_strength(W + H, 180 - ang, is_sm) : 0;
            for (int i = l; i < H; i += G)
                c[-H + i] = st ? ip_smooth(tl - H, i, H - p.p.intra.max_h, H, 0, H + 1, st) : tl[-H + i];
        }
        wave_sync();
        if (l == 0) c[0] = tl[0];
        if (s.up) s.d1 <<= 1;
        if (s.upl) s.d2 <<= 1;
    } else if (s.mode != DGPU_VERT_PRED && s.mode != DGPU_HOR_PRED && s.mode <= DGPU_DC_128_PRED) {
        // DC family: group reduction of the edge sums (src/ipred_tmpl.c:86-166)
        unsigned st = 0, sl = 0;
        for (int i = l; i < W; i += G) st += tl[1 + i];
        for (int i = l; i < H; i += G) sl += tl[-1 - i];
        for (int off = 1; off < G; off <<= 1) {
            st += __shfl_xor(st, off, 64);
            sl += __shfl_xor(sl, off, 64);
        }
        unsigned v;
        if (s.mode == DGPU_DC_128_PRED) v = (bdmax + 1) >> 1;
        else if (s.mode == DGPU_TOP_DC_PRED) v = (st + (W >> 1)) >> __builtin_ctz(W);
        else if (s.mode == DGPU_LEFT_DC_PRED) v = (sl + (H >> 1)) >> __builtin_ctz(H);
        else {
            v = (st + sl + ((W + H) >> 1)) >> __builtin_ctz(W + H);
            if (W != H) {
                const bool r4 = W > 2 * H || H > 2 * W;
                if (BPC == 8) v = (v * (r4 ? 0x3334u : 0x5556u)) >> 16;
                else v = (v * (r4 ? 0x6667u : 0xAAABu)) >> 17;
            }
        }
        s.dc = (int)v;
    }
    return s;
}

// one 4x2 task (x0 = 4q, rows y0, y0 + 1) of every mode but FILTER_PRED
template <typename P>
__device__ __forceinline__ void tintra_task(const IntraState &s, int W, int H, const P *tl, const int16_t *fe, int x0,
                                            int y0, int *pv) {
    switch (s.mode) {
    case DGPU_VERT_PRED:
#pragma unroll
        for (int i = 0; i < 8; i++) pv[i] = tl[1 + x0 + (i & 3)];
        break;
    case DGPU_HOR_PRED:
#pragma unroll
        for (int i = 0; i < 8; i++) pv[i] = tl[-(1 + y0 + (i >> 2))];
        break;
    case DGPU_PAETH_PRED: {   // src/ipred_tmpl.c:244-265
        const int c0 = tl[0];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int top = tl[1 + x0 + (i & 3)], left = tl[-(1 + y0 + (i >> 2))];
            const int base = left + top - c0;
            const int dl = abs(left - base), dt = abs(top - base), dd = abs(c0 - base);
            pv[i] = (dl <= dt && dl <= dd) ? left : dt <= dd ? top : c0;
        }
        break;
    }
    case DGPU_SMOOTH_PRED: {   // src/ipred_tmpl.c:267-325
        const int bl = tl[-H], tr = tl[W];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int x = x0 + (i & 3), y = y0 + (i >> 2);
            const int wv = dspt_sm_weights[H + y], wh = dspt_sm_weights[W + x];
            pv[i] = (wv * tl[1 + x] + (256 - wv) * bl + wh * tl[-(1 + y)] + (256 - wh) * tr + 256) >> 9;
        }
        break;
    }
    case DGPU_SMOOTH_V_PRED: {
        const int bl = tl[-H];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int wv = dspt_sm_weights[H + y0 + (i >> 2)];
            pv[i] = (wv * tl[1 + x0 + (i & 3)] + (256 - wv) * bl + 128) >> 8;
        }
        break;
    }
    case DGPU_SMOOTH_H_PRED: {
        const int tr = tl[W];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int wh = dspt_sm_weights[W + x0 + (i & 3)];
            pv[i] = (wh * tl[-(1 + y0 + (i >> 2))] + (256 - wh) * tr + 128) >> 8;
        }
        break;
    }
    case DGPU_Z1_PRED:
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int x = x0 + (i & 3), y = y0 + (i >> 2);
            const int xpos = (y + 1) * s.d1, frac = xpos & 0x3e;
            const int base = (xpos >> 6) + x * (1 + s.up);
            pv[i] = base < s.maxb ? (fe[base] * (64 - frac) + fe[base + 1] * frac + 32) >> 6 : fe[s.maxb];
        }
        break;
    case DGPU_Z3_PRED:
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int x = x0 + (i & 3), y = y0 + (i >> 2);
            const int ypos = (x + 1) * s.d1, frac = ypos & 0x3e;
            const int base = (ypos >> 6) + y * (1 + s.up);
            pv[i] = base < s.maxb ? (fe[s.maxb - base] * (64 - frac) + fe[s.maxb - base - 1] * frac + 32) >> 6
                                  : fe[0];
        }
        break;
    case DGPU_Z2_PRED: {
        const int16_t *c = fe + 2 * H;
        const int16_t *lft = c - (1 + s.upl);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int x = x0 + (i & 3), y = y0 + (i >> 2);
            const int xpos = ((1 + s.up) << 6) - (y + 1) * s.d1;
            const int bx = (xpos >> 6) + x * (1 + s.up);
            int t;
            if (bx >= 0) {
                const int fx = xpos & 0x3e;
                t = c[bx] * (64 - fx) + c[bx + 1] * fx;
            } else {
                const int ypos = (y << (6 + s.upl)) - (x + 1) * s.d2;
                const int by = ypos >> 6, fy = ypos & 0x3e;
                t = lft[-by] * (64 - fy) + lft[-(by + 1)] * fy;
            }
            pv[i] = (t + 32) >> 6;
        }
        break;
    }
    default:   // DC family
#pragma unroll
        for (int i = 0; i < 8; i++) pv[i] = s.dc;
        break;
    }
}

// Filter intra (src/ipred_tmpl.c:617-655): 4x2 cells == the group's tasks,
// run in anti-diagonal steps.  Each lane first keeps the residual of its
// cells in registers; the cells' predicted values then go into `acc` (the
// recursion reads its neighbours' predictions there), and at the end each
// lane adds its residual back.
template <int BPC, typename P>
__device__ __forceinline__ void tfilter_intra(const Dav1dGpuPred &p, int W, int H, int G, const P *tl,
                                              typename TAcc<BPC>::T *ab, int l, int bdmax) {
    using A = typename TAcc<BPC>::T;
    constexpr int S = TAcc<BPC>::S;
    constexpr int MT = 2;   // tasks per lane: FILTER_PRED blocks are <= 32x32 with G >= NT / 2
    const int QW = W / 4, NT = W * H / 8;
    const signed char *taps = &dspt_filter_intra[(p.p.intra.angle & 511) * 56];
    int res[MT][8];
#pragma unroll
    for (int k = 0; k < MT; k++) {
        const int t = l + k * G;
        if (t < NT) {
            const int x = (t % QW) * 4, y = (t / QW) * 2;
#pragma unroll
            for (int o = 0; o < 8; o++) res[k][o] = ab[(y + (o >> 2)) * S + x + (o & 3)];
        }
    }
    wave_sync();
    for (int step = 0; step < QW + H / 2 - 1; step++) {
#pragma unroll
        for (int k = 0; k < MT; k++) {
            const int t = l + k * G;
            const int cy = t / QW, cx = t % QW;
            if (t < NT && cx + cy == step) {
                const int x = cx * 4, y = cy * 2;
                int p0, p1, p2, p3, p4, p5, p6;
                if (y == 0) {
                    p0 = tl[x];
                    p1 = tl[1 + x]; p2 = tl[2 + x]; p3 = tl[3 + x]; p4 = tl[4 + x];
                } else {
                    const A *upr = ab + (y - 1) * S + x;
                    p0 = x == 0 ? (int)tl[-y] : (int)upr[-1];
                    p1 = upr[0]; p2 = upr[1]; p3 = upr[2]; p4 = upr[3];
                }
                p5 = x == 0 ? (int)tl[-(y + 1)] : (int)ab[y * S + x - 1];
                p6 = x == 0 ? (int)tl[-(y + 2)] : (int)ab[(y + 1) * S + x - 1];
#pragma unroll
                for (int o = 0; o < 8; o++) {
                    const signed char *tk = taps + o * 7;
                    const int acc = tk[0] * p0 + tk[1] * p1 + tk[2] * p2 + tk[3] * p3 + tk[4] * p4 +
                                    tk[5] * p5 + tk[6] * p6;
                    ab[(y + (o >> 2)) * S + x + (o & 3)] = (A)clampi((acc + 8) >> 4, 0, bdmax);
                }
            }
        }
        wave_sync();
    }
#pragma unroll
    for (int k = 0; k < MT; k++) {
        const int t = l + k * G;
        if (t < NT) {
            const int x = (t % QW) * 4, y = (t / QW) * 2;
#pragma unroll
            for (int o = 0; o < 8; o++) {
                A *d = &ab[(y + (o >> 2)) * S + x + (o & 3)];
                *d = (A)clampi((int)*d + res[k][o], 0, bdmax);
            }
        }
    }
}

// one 4x2 task: prediction + residual -> acc
template <int BPC>
__device__ __forceinline__ void acc_put8(typename TAcc<BPC>::T *a, const int *pv, int bdmax) {
    constexpr int S = TAcc<BPC>::S;
    acc_put4<BPC>(a, pv, bdmax);
    acc_put4<BPC>(a + S, pv + 4, bdmax);
}

// A cooperative group: INTRA (edge preparation, the 14 modes) or CFL
// (cfl_ac over the co-located luma + cfl_pred, src/ipred_tmpl.c:657-703,
// :71-84, :103-218).
template <int BPC>
__device__ __forceinline__ void tile_coop(const TileArgs<BPC> &a, const TileCtx<BPC> &c, const Dav1dGpuPred &p,
                                          int l) {
    using P = typename Px<BPC>::pixel;
    using A = typename TAcc<BPC>::T;
    constexpr int S = TAcc<BPC>::S;
    const int W = p.w4 * 4, H = p.h4 * 4, G = 1 << p.lanes_log2;
    const int QW = p.w4, NT = W * H / 8;
    const int bdmax = c.bdmax;
    const P *tl = c.ed + p.p.intra.edge_off;
    int16_t *fe = c.fe + (p.p.intra.edge_off - 2 * H);
    A *ab = c.acc + (p.y4 * 4) * S + p.x4 * 4;
    if (p.kind == DGPU_PRED_INTRA) {
        const IntraState is = tintra_prep<BPC>(p, W, H, G, tl, fe, l, bdmax);
        wave_sync();
        if (is.mode == DGPU_FILTER_PRED) {
            tfilter_intra<BPC>(p, W, H, G, tl, ab, l, bdmax);
        } else {
            for (int t = l; t < NT; t += G) {
                const int j = t / QW, q = t % QW;
                int pv[8];
                tintra_task(is, W, H, tl, fe, 4 * q, 2 * j, pv);
                acc_put8<BPC>(ab + 2 * j * S + 4 * q, pv, bdmax);
            }
        }
    } else {   // CFL: the group's tasks, at most 4 per lane
        constexpr int MT = 4;
        const IntraState dcs = tintra_prep<BPC>(p, W, H, G, tl, fe, l, bdmax);   // DC family reads tl only
        const int ssh = a.cfl_ss & 1, ssv = (a.cfl_ss >> 1) & 1;
        const int wpad = p.p.intra.cfl_pad_wh & 15, hpad = p.p.intra.cfl_pad_wh >> 4;
        const int vw = W - 4 * wpad, vh = H - 4 * hpad;
        const int ys = a.cfl_luma_stride;
        const P *yp = a.cfl_luma + p.p.intra.aux;
        const int acsh = 1 + !ssv + !ssh;
        int ac[MT][8];
        int sum = 0;
#pragma unroll
        for (int k = 0; k < MT; k++) {
            const int t = l + k * G;
#pragma unroll
            for (int i = 0; i < 8; i++) ac[k][i] = 0;
            if (t < NT) {
                const int j = t / QW, q = t % QW;
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int sx = min(4 * q + (i & 3), vw - 1), sy = min(2 * j + (i >> 2), vh - 1);
                    const P *pp = yp + (sy << ssv) * ys + (sx << ssh);
                    int v = gld<P>(pp);
                    if (ssh) v += gld<P>(pp + 1);
                    if (ssv) {
                        v += gld<P>(pp + ys);
                        if (ssh) v += gld<P>(pp + ys + 1);
                    }
                    ac[k][i] = v << acsh;
                    sum += ac[k][i];
                }
            }
        }
        for (int off = 1; off < G; off <<= 1) sum += __shfl_xor(sum, off, 64);
        const int lg = __builtin_ctz(W) + __builtin_ctz(H);
        const int avg = (sum + ((1 << lg) >> 1)) >> lg;
        const int alpha = p.p.intra.alpha;
#pragma unroll
        for (int k = 0; k < MT; k++) {
            const int t = l + k * G;
            if (t < NT) {
                const int j = t / QW, q = t % QW;
                int pv[8];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int d = alpha * (int)(int16_t)(ac[k][i] - avg);   // ac is int16 in the reference
                    const int mag = (abs(d) + 32) >> 6;
                    pv[i] = clampi(dcs.dc + (d < 0 ? -mag : mag), 0, bdmax);
                }
                acc_put8<BPC>(ab + 2 * j * S + 4 * q, pv, bdmax);
            }
        }
    }
}

// --------------------------------------------------------------------- mc --

// Footprint rows of a 4-column task: RR = R + 7 rows starting at (sx, sy)
// (the task's top-left - 3), rows clamped to the plane; row r is loaded only
// when rlo <= r <= rhi (the rows the vertical taps read).  Each row is one
// aligned load from the row's dword: 16 bytes at 8 bpc (realigned by `sh`
// in mc_hrow), 28 bytes at 16 bpc.  When the 11 columns leave the plane
// (emu_edge), the load window is moved inside the plane and every pixel is
// picked at its clamped column with byte permutes (sh = 0 then).
template <int BPC, int RR> struct FootRows {
    static constexpr int ND = BPC == 8 ? 4 : 7;   // dwords loaded per row
    static constexpr int NO = BPC == 8 ? 3 : 6;   // dwords of the 12-pixel window
    uint32_t d[RR][ND];
    unsigned sh;
    // rows r0 .. r0 + RR - 1 of the footprint (rlo / rhi in footprint rows)
    __device__ __forceinline__ void load(const typename Px<BPC>::pixel *base, int stride, int iw, int ih, int sx, int sy,
                                         int rlo, int rhi, int r0 = 0) {
        constexpr int B = BPC / 8;
        constexpr int NP = BPC == 8 ? 2 : 4;   // dword pairs a window byte can come from
        const bool colsafe = sx >= 0 && sx + 11 <= iw;
        const int xa = colsafe ? sx : clampi(sx, 0, max(iw - 12, 0));
        const uintptr_t a0 = reinterpret_cast<uintptr_t>(base + xa);
        const unsigned s0 = (unsigned)(a0 & 3);   // strides and planes are dword multiples (launch check)
        const uint8_t *col = reinterpret_cast<const uint8_t *>(a0 - s0);
        sh = colsafe ? s0 : 0;
        // emu_edge: output byte j of window dword k is raw byte bi, taken as
        // byte (bi & 7) of the dword pair (bi >> 3) -- v_perm per pair, then
        // per-byte masks pick the pair (no register indexing)
        uint32_t sel[NO], msk[NO][NP];
        if (!colsafe) {
#pragma unroll
            for (int k = 0; k < NO; k++) {
                sel[k] = 0;
#pragma unroll
                for (int q = 0; q < NP; q++) msk[k][q] = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int px = BPC == 8 ? 4 * k + j : 2 * k + (j >> 1);
                    const int bi = (int)s0 + B * (clampi(sx + px, 0, iw - 1) - xa) + (BPC == 8 ? 0 : (j & 1));
                    sel[k] |= (uint32_t)(bi & 7) << (8 * j);
#pragma unroll
                    for (int q = 1; q < NP; q++) msk[k][q] |= (bi >> 3) >= q ? 0xffu << (8 * j) : 0u;
                }
            }
        }
        // 1. every row's load, back to back.  A row no vertical tap reads is
        // not loaded (exec-masked); its registers keep an opaque value that
        // only ever meets zero taps -- no select on the loaded value, which
        // would make each load wait for the previous one.
#pragma unroll
        for (int r = 0; r < RR; r++) {
            const int yy = clampi(sy + r0 + r, 0, ih - 1);
            const uint8_t *rp = col + (size_t)yy * stride * B;
#pragma unroll
            for (int k = 0; k < ND; k++) asm volatile("" : "=v"(d[r][k]));
            if (r0 + r >= rlo && r0 + r <= rhi) {
                const u32x4a4 v = gld<u32x4a4>(rp);
                d[r][0] = v.x; d[r][1] = v.y; d[r][2] = v.z; d[r][3] = v.w;
                if constexpr (BPC == 16) {
                    typedef uint32_t u32x3a4 __attribute__((ext_vector_type(3), aligned(4)));
                    const u32x3a4 t = gld<u32x3a4>(rp + 16);
                    d[r][4] = t.x; d[r][5] = t.y; d[r][6] = t.z;
                }
            }
        }
        // 2. emu_edge lanes: pick every window byte at its clamped column
        if (!colsafe) {
#pragma unroll
            for (int r = 0; r < RR; r++) {
                uint32_t w[NO];
#pragma unroll
                for (int k = 0; k < NO; k++) {
                    uint32_t o = __builtin_amdgcn_perm(d[r][1], d[r][0], sel[k]);
#pragma unroll
                    for (int q = 1; q < NP; q++) {
                        const uint32_t hi = 2 * q + 1 < ND ? d[r][2 * q + 1] : 0u;
                        const uint32_t pq = __builtin_amdgcn_perm(hi, d[r][2 * q], sel[k]);
                        o = (pq & msk[k][q]) | (o & ~msk[k][q]);
                    }
                    w[k] = o;
                }
#pragma unroll
                for (int k = 0; k < NO; k++) d[r][k] = w[k];
            }
        }
    }
};

// Horizontal 8-tap of one footprint row -> 4 intermediates (8 bpc: stored as
// mid - 2048, see HPass::compute; 16 bpc: the reference's mid).
template <int BPC>
__device__ __forceinline__ void mc_hrow(const uint32_t *d, unsigned sh, uint4 th, int ib, int *m) {
    if constexpr (BPC == 8) {
        const uint32_t w0 = alb(d[1], d[0], sh) ^ 0x80808080u, w1 = alb(d[2], d[1], sh) ^ 0x80808080u,
                       w2 = alb(d[3], d[2], sh) ^ 0x80808080u;
        const uint32_t lo[4] = {w0, alb(w1, w0, 1), alb(w1, w0, 2), alb(w1, w0, 3)};
        const uint32_t hi[4] = {w1, alb(w2, w1, 1), alb(w2, w1, 2), alb(w2, w1, 3)};
        hdot4x4(lo, hi, th.x, th.y, m);
    } else {
        const int hs = 6 - ib, rnd = (1 << hs) >> 1;
        uint32_t e[6];
#pragma unroll
        for (int i = 0; i < 6; i++) e[i] = alb(d[i + 1], d[i], sh);
        uint32_t o[5];
#pragma unroll
        for (int i = 0; i < 5; i++) o[i] = alb(e[i + 1], e[i], 2);
        m[0] = (dot2(e[3], th.w, dot2(e[2], th.z, dot2(e[1], th.y, dot2(e[0], th.x, 0)))) + rnd) >> hs;
        m[1] = (dot2(o[3], th.w, dot2(o[2], th.z, dot2(o[1], th.y, dot2(o[0], th.x, 0)))) + rnd) >> hs;
        m[2] = (dot2(e[4], th.w, dot2(e[3], th.z, dot2(e[2], th.y, dot2(e[1], th.x, 0)))) + rnd) >> hs;
        m[3] = (dot2(o[4], th.w, dot2(o[3], th.z, dot2(o[2], th.y, dot2(o[1], th.x, 0)))) + rnd) >> hs;
    }
}

// The 4 x R outputs of one reference, row by row: emit(y, t) with t[i] =
// (vertical 8-tap sum of the stored intermediates + kk) >> vsh, kk
// including kMidBias<BPC>.
template <int BPC, int R, typename Emit>
__device__ __forceinline__ void mc_ref(const TileCtx<BPC> &c, const Dav1dGpuPred &p, int k, int x0, int y0, int kk,
                                       int vsh, Emit &&emit) {
    constexpr int RR = R + 7, NP = (RR + 1) / 2;
    const int f2d = p.p.inter.filter2d;
    const bool bil = f2d == DGPU_FILTER_2D_BILINEAR;
    const int ftype = bil ? 0 : (int)((0x951a62840ull >> (4 * f2d)) & 15);
    const int bank_h = mc_bank(ftype & 3, bil, p.bw4 * 4), bank_v = mc_bank(ftype >> 2, bil, p.bh4 * 4);
    const int mx = k ? p.p.inter.mx[1] : p.p.inter.mx[0], my = k ? p.p.inter.my[1] : p.p.inter.my[0];
    const int ri = (k ? p.p.inter.ref[1] : p.p.inter.ref[0]) * 3 + c.plane;
    const int sx = (k ? p.p.inter.src_x[1] : p.p.inter.src_x[0]) + x0 - 3;
    const int sy = (k ? p.p.inter.src_y[1] : p.p.inter.src_y[0]) + y0 - 3;
    // rows the vertical taps read: identity (m == 0) tap 3, bilinear 3..4,
    // the 4-tap banks 2..5, 8-tap 0..7
    const int tf = my == 0 ? 3 : bil ? 3 : bank_v >= 3 ? 2 : 0;
    const int tlst = my == 0 ? 3 : bil ? 4 : bank_v >= 3 ? 5 : 7;
    FootRows<BPC, RR> fr;
    fr.load(c.rt->ref[ri], c.rt->stride[ri], c.rt->w[ri], c.rt->h[ri], sx, sy, tf, R - 1 + tlst);
    uint4 th;
    if constexpr (BPC == 8) {
        const uint2 t2 = reinterpret_cast<const uint2 *>(dspt_mc8)[bank_h * 16 + mx];
        th = make_uint4(t2.x, t2.y, 0, 0);
    } else {
        th = reinterpret_cast<const uint4 *>(dspt_mc16)[bank_h * 16 + mx];
    }
    const uint4 tv = reinterpret_cast<const uint4 *>(dspt_mc16)[bank_v * 16 + my];
    uint32_t E[NP][4];   // (row 2p, row 2p + 1) int16 pairs per column
#pragma unroll
    for (int q = 0; q < NP; q++) {
        int m0[4], m1[4] = {0, 0, 0, 0};
        mc_hrow<BPC>(fr.d[2 * q], fr.sh, th, c.ib, m0);
        if (2 * q + 1 < RR) mc_hrow<BPC>(fr.d[2 * q + 1], fr.sh, th, c.ib, m1);
#pragma unroll
        for (int i = 0; i < 4; i++) E[q][i] = pack16(m0[i], m1[i]);
    }
#pragma unroll
    for (int y = 0; y < R; y++) {
        const int j = y >> 1;
        uint32_t V[4][4];
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int i = 0; i < 4; i++) V[q][i] = (y & 1) ? alb(E[j + q + 1][i], E[j + q][i], 2) : E[j + q][i];
        int t[4];
        vdot4x4(V, tv, kk, vsh, t);
        emit(y, t);
    }
}

// mc put / mct x2 + avg / w_avg / mask for one 4 x R task -> acc.  One
// loop over the references (put: 1, compound: 2), so the filter code exists
// once and a wave mixing put and compound lanes runs it at most twice.
template <int BPC, int R>
__device__ __forceinline__ void tile_mc(const TileArgs<BPC> &a, const TileCtx<BPC> &c, const Dav1dGpuPred &p, int x0,
                                        int y0, typename TAcc<BPC>::T *ab) {
    constexpr int S = TAcc<BPC>::S;
    constexpr int PB = Px<BPC>::PBIAS;
    const int ib = c.ib, bdmax = c.bdmax;
    const bool comp = p.kind != DGPU_PRED_INTER;
    // put: rnd_sh(t, 6 + ib); compound: prep = rnd_sh(t, 6) - PB, kept as
    // p = prep + PREP_BIAS so the reference's bias terms cancel
    // (src/mc_tmpl.c:587-639).  The first reference's values wait as int16
    // pairs of p - PREP_BIAS, the reference's own int16 tmp (src/mc_tmpl.c:252
    // asserts it fits).
    const int vsh = comp ? 6 : 6 + ib;
    const int kk = kMidBias<BPC> + (1 << (vsh - 1));
    const int bw = p.bw4 * 4;
    uint32_t t0[R][2];
#pragma unroll 1
    for (int k = 0; k <= (int)comp; k++) {
        mc_ref<BPC, R>(c, p, k, x0, y0, kk, vsh, [&](int y, const int *t) {
            if (k == 0 && comp) {
                t0[y][0] = pack16(t[0] - PB, t[1] - PB);
                t0[y][1] = pack16(t[2] - PB, t[3] - PB);
                return;
            }
            int pv[4];
            if (!comp) {
#pragma unroll
                for (int i = 0; i < 4; i++) pv[i] = clampi(t[i], 0, bdmax);
            } else {
                const int q0[4] = {(int)(int16_t)(t0[y][0] & 0xffff) + PB, ((int)t0[y][0] >> 16) + PB,
                                   (int)(int16_t)(t0[y][1] & 0xffff) + PB, ((int)t0[y][1] >> 16) + PB};
                if (p.kind == DGPU_PRED_INTER_AVG) {
#pragma unroll
                    for (int i = 0; i < 4; i++) pv[i] = clampi((q0[i] + t[i] + (1 << ib)) >> (ib + 1), 0, bdmax);
                } else if (p.kind == DGPU_PRED_INTER_WAVG) {
                    const int wt = p.p.inter.weight;
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        pv[i] = clampi((q0[i] * wt + t[i] * (16 - wt) + (8 << ib)) >> (ib + 4), 0, bdmax);
                } else {   // INTER_MASK: the block's mask, stride bw
                    const uint32_t mk = gld<uint32_t>(a.aux_pool + p.p.inter.aux + (y0 + y) * bw + x0);
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int m = (int)((mk >> (8 * i)) & 0xff);
                        pv[i] = clampi((q0[i] * m + t[i] * (64 - m) + (32 << ib)) >> (ib + 6), 0, bdmax);
                    }
                }
            }
            acc_put4<BPC>(ab + y * S, pv, bdmax);
        });
    }
}

// inter-intra (src/recon_tmpl.c:1540-1580): put, intra_pred of the
// inter-intra modes (DC / V / H / SMOOTH, computed per lane from the edge
// array in memory), blend_c with the block mask (src/mc_tmpl.c:641-653)
template <int BPC, int R>
__device__ __forceinline__ void tile_ii(const TileArgs<BPC> &a, const TileCtx<BPC> &c, const Dav1dGpuPred &p, int x0,
                                        int y0, typename TAcc<BPC>::T *ab) {
    using P = typename Px<BPC>::pixel;
    constexpr int S = TAcc<BPC>::S;
    const int ib = c.ib, bdmax = c.bdmax;
    const int W = p.w4 * 4, H = p.h4 * 4, bw = p.bw4 * 4;
    int t0[R][4];
    const int sh = 6 + ib;
    mc_ref<BPC, R>(c, p, 0, x0, y0, kMidBias<BPC> + (1 << (sh - 1)), sh, [&](int y, const int *t) {
#pragma unroll
        for (int i = 0; i < 4; i++) t0[y][i] = t[i];
    });
    const u32x4 rec = gld<u32x4>(a.aux_pool + p.p.inter.aux);
    const P *tl = a.edges + (int)rec[0];
    const int mode = (int)(rec[1] & 0xff);
    const uint8_t *mkb = a.aux_pool + rec[2];
    int dc = 0;
    if (mode == DGPU_DC_PRED) {   // src/ipred_tmpl.c:86-166
        unsigned st = 0;
        for (int i = 0; i < W; i++) st += gld<P>(tl + 1 + i);
        for (int i = 0; i < H; i++) st += gld<P>(tl - 1 - i);
        unsigned v = (st + ((W + H) >> 1)) >> __builtin_ctz(W + H);
        if (W != H) {
            const bool r4 = W > 2 * H || H > 2 * W;
            if (BPC == 8) v = (v * (r4 ? 0x3334u : 0x5556u)) >> 16;
            else v = (v * (r4 ? 0x6667u : 0xAAABu)) >> 17;
        }
        dc = (int)v;
    }
    const int bl = gld<P>(tl - H), tr = gld<P>(tl + W);
#pragma unroll
    for (int y = 0; y < R; y++) {
        const int yy = y0 + y;
        const int left = gld<P>(tl - 1 - yy);
        const uint32_t mk = gld<uint32_t>(mkb + yy * bw + x0);
        int pv[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int xx = x0 + i;
            int ip;
            if (mode == DGPU_DC_PRED) ip = dc;
            else if (mode == DGPU_VERT_PRED) ip = gld<P>(tl + 1 + xx);
            else if (mode == DGPU_HOR_PRED) ip = left;
            else {   // SMOOTH
                const int wv = dspt_sm_weights[H + yy], wh = dspt_sm_weights[W + xx];
                ip = (wv * gld<P>(tl + 1 + xx) + (256 - wv) * bl + wh * left + (256 - wh) * tr + 256) >> 9;
            }
            const int m = (int)((mk >> (8 * i)) & 0xff);
            const int ipv = clampi(t0[y][i], 0, bdmax);
            pv[i] = (ipv * (64 - m) + ip * m + 32) >> 6;
        }
        acc_put4<BPC>(ab + y * S, pv, bdmax);
    }
}

// warp8x8 (src/mc_tmpl.c:758-791) for one 4 x R task inside an 8x8 of a
// WARP pred.  Record: int16 abcd[4], 8 pad bytes, then per 8x8 (row-major)
// int16 x, int16 y (the 8x8's source position, dx / dy of
// recon_tmpl.c:1162-1167), int16 mx >> 6, int16 my >> 6.  The 15 x 15
// footprint is clamped to the plane (the emu_edge of recon_tmpl.c:1172).
template <int BPC, int R>
__device__ __forceinline__ void tile_warp(const TileArgs<BPC> &a, const TileCtx<BPC> &c, const Dav1dGpuPred &p, int x0,
                                          int y0, typename TAcc<BPC>::T *ab) {
    constexpr int RR = R + 7, S = TAcc<BPC>::S;
    const int ib = c.ib, bdmax = c.bdmax;
    const uint8_t *rec = a.aux_pool + p.p.inter.aux;
    const u32x2 abcd = gld<u32x2>(rec);
    const int a0 = (int16_t)(abcd[0] & 0xffff), a1 = (int)abcd[0] >> 16;
    const int a2 = (int16_t)(abcd[1] & 0xffff), a3 = (int)abcd[1] >> 16;
    const int nbx = p.w4 / 2;
    const int xs = x0 & 7, ys = y0 & 7;   // task position inside its 8x8
    const u32x2 sb = gld<u32x2>(rec + 16 + 8 * ((y0 >> 3) * nbx + (x0 >> 3)));
    const int bx = (int16_t)(sb[0] & 0xffff), by = (int)sb[0] >> 16;
    const int mx = (int)(int16_t)(sb[1] & 0xffff) * 64, my = ((int)sb[1] >> 16) * 64;
    const int ri = p.p.inter.ref[0] * 3 + c.plane;
    FootRows<BPC, RR> fr;   // rows ys - 3 .. ys + R + 3, columns xs - 3 .. xs + 7 of the 8x8
    fr.load(c.rt->ref[ri], c.rt->stride[ri], c.rt->w[ri], c.rt->h[ri], bx + xs - 3, by + ys - 3, 0, RR - 1);
    const int hsh = 7 - ib, hrnd = (1 << hsh) >> 1;
    int mid[RR][4];
#pragma unroll
    for (int r = 0; r < RR; r++) {
        const int row = ys + r;   // row of the reference's 15-row mid (0 = footprint row -3)
        const uint32_t *d = fr.d[r];
        if constexpr (BPC == 8) {
            const uint32_t w0 = alb(d[1], d[0], fr.sh) ^ 0x80808080u, w1 = alb(d[2], d[1], fr.sh) ^ 0x80808080u,
                           w2 = alb(d[3], d[2], fr.sh) ^ 0x80808080u;
            const uint32_t lo[4] = {w0, alb(w1, w0, 1), alb(w1, w0, 2), alb(w1, w0, 3)};
            const uint32_t hi[4] = {w1, alb(w2, w1, 1), alb(w2, w1, 2), alb(w2, w1, 3)};
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int pos = mx + row * a1 + (xs + i) * a0;
                const uint2 kt = c.wtab[64 + ((pos + 512) >> 10)];
                // taps sum to 128 and p ^ 0x80 == p - 128: sum = acc + 128 * 128
                mid[r][i] = (dot4(hi[i], kt.y, dot4(lo[i], kt.x, 16384 + hrnd))) >> hsh;
            }
        } else {
            uint32_t e[6];
#pragma unroll
            for (int i = 0; i < 6; i++) e[i] = alb(d[i + 1], d[i], fr.sh);
            uint32_t o[5];
#pragma unroll
            for (int i = 0; i < 5; i++) o[i] = alb(e[i + 1], e[i], 2);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int pos = mx + row * a1 + (xs + i) * a0;
                const uint2 kt = c.wtab[64 + ((pos + 512) >> 10)];
                uint32_t tp[4];   // int8 taps -> int16 pairs
#pragma unroll
                for (int m = 0; m < 4; m++) {
                    const uint32_t src = m < 2 ? kt.x : kt.y;
                    tp[m] = pack16(__builtin_amdgcn_sbfe((int)src, 16 * (m & 1), 8),
                                   __builtin_amdgcn_sbfe((int)src, 16 * (m & 1) + 8, 8));
                }
                const uint32_t *pp = (i & 1) ? o + (i >> 1) : e + (i >> 1);
                mid[r][i] = (dot2(pp[3], tp[3], dot2(pp[2], tp[2], dot2(pp[1], tp[1], dot2(pp[0], tp[0], 0)))) + hrnd) >> hsh;
            }
        }
    }
    const int vsh = 7 + ib, vrnd = (1 << vsh) >> 1;
#pragma unroll
    for (int y = 0; y < R; y++) {
        int pv[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int pos = my + (ys + y) * a3 + (xs + i) * a2;
            const uint2 kt = c.wtab[64 + ((pos + 512) >> 10)];
            int s = vrnd;
#pragma unroll
            for (int kk = 0; kk < 8; kk++)
                s += __builtin_amdgcn_sbfe((int)(kk < 4 ? kt.x : kt.y), 8 * (kk & 3), 8) * mid[y + kk][i];
            pv[i] = clampi(s >> vsh, 0, bdmax);
        }
        acc_put4<BPC>(ab + y * S, pv, bdmax);
    }
}

// one independent task of a pred (4 columns x R rows at (x0, y0) of the pred)
template <int BPC, int R>
__device__ __forceinline__ void tile_task(const TileArgs<BPC> &a, const TileCtx<BPC> &c, const Dav1dGpuPred &p,
                                          int x0, int y0, int plane_x, int plane_y) {
    using P = typename Px<BPC>::pixel;
    constexpr int S = TAcc<BPC>::S;
    auto *ab = c.acc + (p.y4 * 4 + y0) * S + p.x4 * 4 + x0;
    switch (p.kind) {
    case DGPU_PRED_INTER:
    case DGPU_PRED_INTER_AVG:
    case DGPU_PRED_INTER_WAVG:
    case DGPU_PRED_INTER_MASK:
        tile_mc<BPC, R>(a, c, p, x0, y0, ab);
        break;
    case DGPU_PRED_INTER_INTRA:
        tile_ii<BPC, R>(a, c, p, x0, y0, ab);
        break;
    case DGPU_PRED_WARP:
        tile_warp<BPC, R>(a, c, p, x0, y0, ab);
        break;
    case DGPU_PRED_PAL: {   // pal_pred (src/ipred_tmpl.c:717-730): record = 8 entries, then
                            // the packed index map (stride w / 2)
        const uint8_t *rec = a.aux_pool + p.p.intra.aux;
        const u32x4 pal = gld<u32x4>(rec);
        const int W = p.w4 * 4;
#pragma unroll
        for (int y = 0; y < R; y++) {
            const uint32_t ix = gld<uint16_t>(rec + 16 + (y0 + y) * (W / 2) + x0 / 2);
            int pv[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int e = (int)((ix >> (4 * i)) & 7);
                if constexpr (BPC == 8)
                    pv[i] = (int)(((e < 4 ? pal[0] : pal[1]) >> (8 * (e & 3))) & 0xff);
                else
                    pv[i] = (int)(((e < 2 ? pal[0] : e < 4 ? pal[1] : e < 6 ? pal[2] : pal[3]) >> (16 * (e & 1))) &
                                  0xffff);
            }
            acc_put4<BPC>(ab + y * S, pv, c.bdmax);
        }
        break;
    }
    default: {   // NONE: the residual goes onto the existing picture
        const P *dp = a.dst[c.plane] + (size_t)plane_y * a.dst_stride[c.plane] + plane_x;
#pragma unroll
        for (int y = 0; y < R; y++) {
            int pv[4];
            if constexpr (BPC == 8) {
                const uint32_t v = gld<uint32_t>(dp + (size_t)y * a.dst_stride[c.plane]);
#pragma unroll
                for (int i = 0; i < 4; i++) pv[i] = (int)((v >> (8 * i)) & 0xff);
            } else {
                const u32x2 v = gld<u32x2>(dp + (size_t)y * a.dst_stride[c.plane]);
                pv[0] = (int)(v[0] & 0xffff); pv[1] = (int)(v[0] >> 16);
                pv[2] = (int)(v[1] & 0xffff); pv[3] = (int)(v[1] >> 16);
            }
            acc_put4<BPC>(ab + y * S, pv, c.bdmax);
        }
        break;
    }
    }
}

// ----------------------------------------------------------------- kernel --

// HUGE: the launch over the tiles with 64-point transforms (the 64-point
// row / column code is compiled only there: its registers would otherwise
// set the occupancy of every tile)
// (3 waves per SIMD the register allocator must allow; 4 spilled: 165 us)
template <int BPC, bool HUGE>
__global__ __launch_bounds__(kTileThreads) __attribute__((amdgpu_waves_per_eu(3))) void k_tiles(
    TileArgs<BPC> a) {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    using A = typename TAcc<BPC>::T;
    using L = TileLds<BPC>;
    constexpr int S = TAcc<BPC>::S;
    __shared__ __attribute__((aligned(16))) uint8_t lds[L::BYTES];
    __shared__ TileRefTab<BPC> rt;
    const int tid = threadIdx.x;
    // XCD-contiguous order: blocks are dealt round-robin over the 8 XCDs, so
    // XCD x takes the x-th contiguous eighth of the tiles (a band of the
    // picture, all planes): its L2 sees whole picture lines written and the
    // neighbouring tiles' reference footprints
    const int nb = gridDim.x, b = blockIdx.x;
    const int lb = (b & 7) * (nb >> 3) + (b >> 3);
    if (lb >= a.n_tiles) return;
    auto mark = [&](int i) {
        if constexpr (DGPU_TILE_TRACE) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if ((tid & 63) == 0) a.trace[((size_t)(a.tile0 + lb) * 4 + (tid >> 6)) * 8 + i] = t;
        }
    };
    mark(0);
    const Dav1dGpuTile T = bld(a.tiles + a.tile0 + lb);
    const int plane = T.plane;
    const int TW = T.w4 * 4, TH = T.h4 * 4;

    A *acc = reinterpret_cast<A *>(lds + L::O_ACC);
    uint8_t *cfb = lds + L::O_CF;
    uint8_t *edb = lds + L::O_EDGE;
    uint8_t *txmap = lds + L::O_TXMAP;
    uint8_t *pmap = lds + L::O_PMAP;
    uint2 *wtab = reinterpret_cast<uint2 *>(lds + L::O_WARP);

    // ---- P0: staging ----
    if (tid < DGPU_MAX_REFS * 3) {
        rt.ref[tid] = a.ref[tid];
        rt.stride[tid] = a.ref_stride[tid];
        rt.w[tid] = a.ref_w[tid];
        rt.h[tid] = a.ref_h[tid];
    }
    // coefficients and edges: 16-byte chunks from the 16-byte block holding
    // the first byte (skew), all loads in flight before the LDS writes
    const uint8_t *cg = reinterpret_cast<const uint8_t *>(a.coef + T.coef0);
    const int csk = (int)(reinterpret_cast<uintptr_t>(cg) & 15);
    const int cnch = T.n_coef ? (csk + T.n_coef * (int)sizeof(C) + 15) >> 4 : 0;
    const uint8_t *eg = reinterpret_cast<const uint8_t *>(a.edges + T.edge0);
    const int esk = (int)(reinterpret_cast<uintptr_t>(eg) & 15);
    const int ench = T.n_edge ? (esk + T.n_edge * (int)sizeof(P) + 15) >> 4 : 0;
    constexpr int CIT = (4096 * (int)sizeof(C) + 31) / 16 / kTileThreads + 1;
    constexpr int EIT = (DGPU_TILE_MAX_EDGE * (int)sizeof(P) + 31) / 16 / kTileThreads + 1;
    u32x4 cv[CIT], ev[EIT];
#pragma unroll
    for (int k = 0; k < CIT; k++) {
        const int i = tid + k * kTileThreads;
        if (i < cnch) cv[k] = gld<u32x4>(cg - csk + 16 * i);
    }
#pragma unroll
    for (int k = 0; k < EIT; k++) {
        const int i = tid + k * kTileThreads;
        if (i < ench) ev[k] = gld<u32x4>(eg - esk + 16 * i);
    }
    uint2 wv = make_uint2(0, 0);
    const bool haswarp = T.flags & 1;
    if (haswarp && tid < 193) wv = reinterpret_cast<const uint2 *>(dspt_warp)[tid];
    // lane maps: each record writes its index over its lanes
    if (tid < T.n_tx) {
        const Dav1dGpuTx tx = bld(a.txs + T.tx0 + tid);
        const int n = tile_tx_lanes((tx.w0 >> 8) & 31), l0 = tx.w1 >> 16;   // n >= 4, l0 a multiple of n
        for (int i = 0; i < n; i += 4) *reinterpret_cast<uint32_t *>(txmap + l0 + i) = 0x01010101u * (uint32_t)tid;
    }
    if (tid < T.n_pred) {
        const uint4 ph = bld(reinterpret_cast<const uint4 *>(a.preds + T.pred0 + tid));   // kind .. lane0
        const int kind = ph.x & 0xff, w4 = (ph.x >> 24) & 0xff, h4 = ph.y & 0xff, lg = (ph.y >> 24) & 0xff;
        const int l0 = ph.z & 0xffff;
        int n, base;
        if (kind == DGPU_PRED_INTRA || kind == DGPU_PRED_CFL) {
            n = 1 << lg;
            base = l0;
        } else {
            const int R = (BPC == 8 && h4 >= 2) ? 8 : 4;
            n = w4 * (h4 * 4 / R);
            base = T.lanes_coop + l0;
        }
        for (int i = 0; i < n; i++) pmap[base + i] = (uint8_t)tid;
    }
    // the cooperative section's padding lanes [lanes_coop_used, lanes_coop)
    // belong to no prediction but still read one below (P2): give them
    // record 0, so no lane indexes the record array with stale LDS (an
    // index up to 255 past the tile's records read past the array's end:
    // the intermittent illegal-address faults of the round-3 / round-4
    // GPU runs)
#if DGPU_BOUNDS
    if (!a.bnd_noclamp)
#endif
    for (int i = T.lanes_coop_used + tid; i < T.lanes_coop; i += kTileThreads) pmap[i] = 0;
    // zero the residual tile
    for (int i = tid; i < L::ACC / 16; i += kTileThreads) reinterpret_cast<u32x4 *>(acc)[i] = u32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < CIT; k++) {
        const int i = tid + k * kTileThreads;
        if (i < cnch) reinterpret_cast<u32x4 *>(cfb)[i] = cv[k];
    }
#pragma unroll
    for (int k = 0; k < EIT; k++) {
        const int i = tid + k * kTileThreads;
        if (i < ench) reinterpret_cast<u32x4 *>(edb)[i] = ev[k];
    }
    if (haswarp && tid < 193) wtab[tid] = wv;
    mark(1);
    __syncthreads();
    mark(2);
    // the coefficient-zeroing contract (src/itx_tmpl.c:55/89): every load of
    // the range completed before the barrier
    if (a.zero_coefs)
        for (int i = tid; i < T.n_coef; i += kTileThreads) bst<C>(a.coef + T.coef0 + i, 0);

    TileCtx<BPC> c;
    c.acc = acc;
    c.cf = reinterpret_cast<const C *>(cfb + csk);
    c.ed = reinterpret_cast<const P *>(edb + esk);
    c.fe = reinterpret_cast<int16_t *>(cfb + 16);   // P2 only (aliases the coefficients)
    c.wtab = wtab;
    c.rt = &rt;
    c.plane = plane;
    c.bdmax = a.bdmax;
    c.ib = Px<BPC>::ibits(a.bdmax);

    // ---- P1: inverse transforms into acc ----
    const Clip rc = ItxClip<BPC>::row(a.bdmax), cc = ItxClip<BPC>::col(a.bdmax);
    for (int base = 0; base < T.lanes_tx; base += kTileThreads) {
        const int lane = base + tid;
        const bool act = lane < T.lanes_tx;
        Dav1dGpuTx tx = {0, 0};
        if (act) tx = bld(a.txs + T.tx0 + DGPU_TILE_INDEX((int)txmap[lane], T.n_tx, 0));
        const int txs = (tx.w0 >> 8) & 31, txtp = (tx.w0 >> 13) & 31;
        const int nzw = (tx.w0 >> 18) & 63, nzh = (tx.w0 >> 24) & 63;
        const int l = lane - (int)(tx.w1 >> 16);
        const TxInfo ti = tx_info(txs);
        const int W = ti.w, H = ti.h;
        A *ab = acc + (((tx.w0 >> 4) & 15) * 4) * S + (tx.w0 & 15) * 4;
        const C *cs = c.cf + (tx.w1 & 0xffff);
        const bool wht = txtp == DGPU_WHT_WHT;   // lossless 4x4: one lane, both passes, int32
        if (act && wht && l == 0) {
            int t[16];
            wht4x4(cs, nzw, nzh, t);
#pragma unroll
            for (int y = 0; y < 4; y++)
#pragma unroll
                for (int x = 0; x < 4; x++)
                    ab[y * S + x] = (A)(BPC == 8 ? clampi(t[4 * y + x], -32768, 32767) : t[4 * y + x]);
        }
        if (act && !wht && nzw && l < nzh) {   // row pass
            const bool rect2 = W * 2 == H || H * 2 == W;
            A *arow = ab + l * S;
            const int kh = kind_h(txtp);
            switch (W) {
            case 4: tile_row<BPC, 4>(cs, nzw, nzh, l, kh, ti.shift, rect2, rc, cc, arow); break;
            case 8: tile_row<BPC, 8>(cs, nzw, nzh, l, kh, ti.shift, rect2, rc, cc, arow); break;
            case 16: tile_row<BPC, 16>(cs, nzw, nzh, l, kh, ti.shift, rect2, rc, cc, arow); break;
            case 32: tile_row<BPC, 32>(cs, nzw, nzh, l, kh, ti.shift, rect2, rc, cc, arow); break;
            default:
                if constexpr (HUGE) tile_row<BPC, 64>(cs, nzw, nzh, l, kh, ti.shift, rect2, rc, cc, arow);
                break;
            }
        }
        wave_sync();
        if (act && !wht && l < W) {   // column pass, in place
            A *acol = ab + l;
            if (!nzw) {   // DC-only (src/itx_tmpl.c:53-65)
                int dc = cs[0];
                if (W * 2 == H || H * 2 == W) dc = r8s(dc);
                dc = r8s(dc);
                dc = (dc + ((1 << ti.shift) >> 1)) >> ti.shift;
                const int dcres = (dc * 181 + 128 + 2048) >> 12;
                for (int y = 0; y < H; y++) acol[y * S] = (A)dcres;
            } else {
                const int kv = kind_v(txtp);
                switch (H) {
                case 4: tile_col<BPC, 4>(acol, nzh, kv, cc); break;
                case 8: tile_col<BPC, 8>(acol, nzh, kv, cc); break;
                case 16: tile_col<BPC, 16>(acol, nzh, kv, cc); break;
                case 32: tile_col<BPC, 32>(acol, nzh, kv, cc); break;
                default:
                    if constexpr (HUGE) tile_col<BPC, 64>(acol, nzh, kv, cc);
                    break;
                }
            }
        }
        wave_sync();
    }
    mark(3);
    __syncthreads();
    mark(4);

    // ---- P2: predictions (+ residual, clip) into acc ----
    const int lanes_pred = T.lanes_coop + T.lanes_task;
    for (int base = 0; base < lanes_pred; base += kTileThreads) {
        const int lane = base + tid;
        const int wlane = base + (tid & ~63);   // wave-uniform: its section
        if (lane < lanes_pred) {
            const Dav1dGpuPred p = bld(a.preds + T.pred0 + DGPU_TILE_INDEX((int)pmap[lane], T.n_pred, 1));
            if (wlane < T.lanes_coop) {
                if (lane < T.lanes_coop_used) tile_coop<BPC>(a, c, p, lane - p.lane0);
            } else {
                const int t = lane - T.lanes_coop - p.lane0;
                const int R = (BPC == 8 && p.h4 >= 2) ? 8 : 4;
                const int x0 = (t % p.w4) * 4, y0 = (t / p.w4) * R;
                const int px = T.x + p.x4 * 4 + x0, py = T.y + p.y4 * 4 + y0;
                if constexpr (BPC == 8) {
                    if (R == 8) tile_task<BPC, 8>(a, c, p, x0, y0, px, py);
                    else tile_task<BPC, 4>(a, c, p, x0, y0, px, py);
                } else {
                    tile_task<BPC, 4>(a, c, p, x0, y0, px, py);
                }
            }
        }
    }
    mark(5);
    __syncthreads();
    mark(6);

    // ---- P3: store the tile, whole rows ----
    P *dp = a.dst[plane] + (size_t)T.y * a.dst_stride[plane] + T.x;
    const int ds = a.dst_stride[plane];
    if constexpr (BPC == 8) {
        if ((TW & 15) == 0) {   // 16 pixels per lane
            const int cpr = TW >> 4;
            for (int i = tid; i < TH * cpr; i += kTileThreads) {
                const int y = i / cpr, x = (i - y * cpr) * 16;
                const uint32_t *s = reinterpret_cast<const uint32_t *>(acc + y * S + x);
                u32x4 o;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t lo = s[2 * k], hi = s[2 * k + 1];
                    o[k] = __builtin_amdgcn_perm(hi, lo, 0x06040200u);   // low bytes of the 4 int16
                }
                gst<u32x4>(dp + (size_t)y * ds + x, o);
            }
        } else {
            const int cpr = TW >> 2;
            for (int i = tid; i < TH * cpr; i += kTileThreads) {
                const int y = i / cpr, x = (i - y * cpr) * 4;
                const uint32_t *s = reinterpret_cast<const uint32_t *>(acc + y * S + x);
                gst<uint32_t>(dp + (size_t)y * ds + x, __builtin_amdgcn_perm(s[1], s[0], 0x06040200u));
            }
        }
    } else {
        const int cpr = TW >> 2;   // 4 pixels (8 bytes) per lane
        for (int i = tid; i < TH * cpr; i += kTileThreads) {
            const int y = i / cpr, x = (i - y * cpr) * 4;
            const A *s = acc + y * S + x;
            gst<u32x2>(dp + (size_t)y * ds + x,
                       u32x2{(uint32_t)s[0] | (uint32_t)s[1] << 16, (uint32_t)s[2] | (uint32_t)s[3] << 16});
        }
        mark(7);
}
}

}  // namespace dgpu
