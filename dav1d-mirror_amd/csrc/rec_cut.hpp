// rec_cut.hpp -- the batch recorder's cut, run per recorded block on the
// device (csrc/recorder.hip).
//
// What recon_b_inter / recon_b_intra (src/recon_tmpl.c:1598, :1195) iterate
// per block -- its transform grid (:1258-1262), mc() per prediction unit with
// its emu_edge decision (:986-999, scaled :1036-1046, warp :1168-1177), the
// intra edge record of every transform block (:1248-1294) -- is derived here
// from the recording by one function per block, cut_block<W>.  It runs twice
// per flush: W = false counts what the block needs (cells, aux-pool bytes,
// clamped footprint copies and their scratch rows, launch-ahead units, edge
// pixels, producer lookups), an exclusive scan over blocks turns the counts
// into the block's bases, and W = true writes the block's records at them.
// Offsets are therefore exactly those of a sequential cut in decode order.
// The same functions run serially on the host for DAV1D_GPU_REC_HOSTONLY
// (diagnostics: the upload image without a device).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "dav1d_gpu.h"

namespace rec {

constexpr int NC = DGPU_N_RECT_TX_SIZES;
constexpr int kEmuStride = 128;   // pixels per row of the clamped-footprint scratch plane
constexpr int kMapPad4 = 32;      // 4x4 cells past the grid a transform block can reach (128 px)

// transform sizes: log2(w / 4), log2(h / 4), 3 bits per size (Dav1dGpuTxfmSize order)
constexpr int kTxLw[NC] = {0, 1, 2, 3, 4, 0, 1, 1, 2, 2, 3, 3, 4, 0, 2, 1, 3, 2, 4};
constexpr int kTxLh[NC] = {0, 1, 2, 3, 4, 1, 0, 2, 1, 3, 2, 4, 3, 2, 0, 3, 1, 4, 2};
constexpr uint64_t pack3(const int (&a)[NC]) {
    uint64_t v = 0;
    for (int i = 0; i < NC; i++) v |= (uint64_t)a[i] << (3 * i);
    return v;
}
constexpr uint64_t kTxWp = pack3(kTxLw), kTxHp = pack3(kTxLh);
__host__ __device__ inline int tx_w(int t) { return 4 << (int)((kTxWp >> (3 * t)) & 7); }
__host__ __device__ inline int tx_h(int t) { return 4 << (int)((kTxHp >> (3 * t)) & 7); }
__host__ __device__ inline int tx_of(int w, int h) {
    for (int t = 0; t < NC; t++)
        if (tx_w(t) == w && tx_h(t) == h) return t;
    return -1;
}

// av1_intra_prediction_edges needs (src/ipred_prepare_tmpl.c:50-75):
// bit0 left, 1 top, 2 top-left, 3 top-right, 4 bottom-left
__host__ __device__ inline int needs(int m) {
    // 5 bits per mode: {3, 2, 1, 1, 2, 0, 14, 7, 21, 3, 3, 3, 7, 7}
    constexpr uint64_t lo = 3ull | 2ull << 5 | 1ull << 10 | 1ull << 15 | 2ull << 20 | 0ull << 25 | 14ull << 30 |
                            7ull << 35 | 21ull << 40 | 3ull << 45 | 3ull << 50 | 3ull << 55;
    return m < 12 ? (int)((lo >> (5 * m)) & 31) : 7;
}

// the mode remap of dav1d_prepare_intra_edges (src/ipred_prepare_tmpl.c:83-104)
__host__ __device__ inline int remap_mode(int mode, int angle, bool hl, bool ht) {
    if (mode >= 1 && mode <= 8) {
        // the directional modes' base angles: 90, 180, 45, 135, 113, 157, 203, 67
        constexpr uint64_t dir = 90ull | 180ull << 8 | 45ull << 16 | 135ull << 24 | 113ull << 32 | 157ull << 40 |
                                 203ull << 48 | 67ull << 56;
        const int a = (int)((dir >> (8 * (mode - 1))) & 255) + 3 * angle;
        if (a <= 90) return a < 90 && ht ? DGPU_Z1_PRED : DGPU_VERT_PRED;
        if (a < 180) return DGPU_Z2_PRED;
        return a > 180 && hl ? DGPU_Z3_PRED : DGPU_HOR_PRED;
    }
    if (mode == 0) return hl ? (ht ? DGPU_DC_PRED : DGPU_LEFT_DC_PRED) : (ht ? DGPU_TOP_DC_PRED : DGPU_DC_128_PRED);
    if (mode == 12) return hl ? (ht ? DGPU_PAETH_PRED : DGPU_HOR_PRED) : (ht ? DGPU_VERT_PRED : DGPU_DC_128_PRED);
    return mode;
}

// kinds recorded with block data (dav1d_gpu_rec_block_aux); the last four
// are predicted by the launch ahead of the wavefront
__host__ __device__ inline bool is_ext_kind(int k) {
    return k == DGPU_PRED_INTER_MASK || k == DGPU_PRED_PAL || k == DGPU_PRED_WARP || k == DGPU_PRED_INTER_WMASK ||
           k == DGPU_PRED_INTER_OBMC || k == DGPU_PRED_INTER_SCALED || k == DGPU_PRED_INTER_INTRA;
}
__host__ __device__ inline bool is_prelaunch_kind(int k) {
    return k == DGPU_PRED_WARP || k == DGPU_PRED_INTER_WMASK || k == DGPU_PRED_INTER_OBMC ||
           k == DGPU_PRED_INTER_SCALED;
}
__host__ __device__ inline bool is_mc_kind(int k) {   // the flow kinds that read references through src_off
    return k == DGPU_PRED_INTER || k == DGPU_PRED_INTER_AVG || k == DGPU_PRED_INTER_WAVG ||
           k == DGPU_PRED_INTER_MASK;
}

struct RecRes {   // one recorded residual (32 B)
    int32_t plane, x, y, tx, txtp, nzw, nzh;
    int32_t coef;   // element offset into the coefficient pool
};

// emu_edge per transform / prediction unit: a footprint that leaves its
// reference picture is copied, every read clamped, into a scratch plane of
// kEmuStride pixels per row (a band of rows per copy; warp 8x8s side by side)
struct EmuJob {
    int32_t x0, y0;   // the footprint's top-left in the reference (may be outside)
    int32_t o0;       // its top-left in the scratch plane (pixels)
    uint8_t w, h, slot, plane;
};
static_assert(sizeof(EmuJob) == 16, "EmuJob layout");

// what the level pass needs of a cell (its geometry in 4x4 units, the edge
// needs of its remapped mode, the tile end)
struct LvJob {
    int16_t x4, y4, W4, H4;
    uint8_t p, cw4, ch4, nd, fl, pad_[3];
    int32_t link;   // IIRES: its block's inter-intra prediction cell
    enum { HL = 1, HT = 2, TR = 4, BL = 8, CFL = 16, IIRES = 32, IIC = 64 };
};

struct ObmcBlockLap {   // dav1d_gpu_rec_block_aux INTER_OBMC entry (24 B)
    int32_t mvx, mvy;
    uint8_t filter2d, ref, x0, y0, x1, y1, lap_w4, lap_h4, dir, mask_off, pad_[6];
};
struct ObmcUnitLap {    // Dav1dGpuPredKind INTER_OBMC unit entry (16 B)
    int32_t src_off;
    uint8_t mx, my, filter2d, ref, x0, y0, x1, y1, lap_w4, lap_h4, dir, mask_off;
};
struct ScaledBlockRef {   // INTER_SCALED block record, per ref
    int32_t x, y;
    uint16_t mx, my, dx, dy;
};
struct ScaledUnitRef {
    int32_t src_off;
    uint16_t mx, my, dx, dy;
    uint32_t pad_;
};
static_assert(sizeof(ObmcBlockLap) == 24 && sizeof(ObmcUnitLap) == 16 && sizeof(ScaledBlockRef) == 16 &&
              sizeof(ScaledUnitRef) == 16 && sizeof(LvJob) == 20, "record layouts");

// per block: what it needs (count pass), scanned into its bases
enum { C_CELLS, C_AUX, C_EJOBS, C_EROWS, C_XU, C_EDGE, C_RES, C_RAW, C_N };
struct BlockCnt {
    long long v[C_N];
};
struct BlockCntSum {
    __host__ __device__ BlockCnt operator()(const BlockCnt &a, const BlockCnt &b) const {
        BlockCnt r;
        for (int i = 0; i < C_N; i++) r.v[i] = a.v[i] + b.v[i];
        return r;
    }
};

enum { E_BAD = 1, E_OVERLAP = 2, E_STALL = 4 };
struct Hdr {   // the flush's device-side header (read back by the host)
    int32_t err, last_aux, max_level, ticket;
    int32_t n_bk, pad_[3];
    long long aux_end;
    BlockCnt tot;
};

struct RefInfo {   // ref[slot][plane] as the flush gives it
    long long stride_b;   // bytes
    int32_t stride_px;    // stride / bpp whenever ref[] is given (the plane may be NULL)
    int32_t w, h, ok;     // ok: a plane to read
};

__host__ __device__ inline void amax(int32_t *p, int32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    if (v > *p) *p = v;   // (host-only flushes run the steps serially)
#endif
}
__host__ __device__ inline void aor(int32_t *p, int32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    *p |= v;
#endif
}
__host__ __device__ inline void bcopy(uint8_t *d, const uint8_t *s, int n) {
    for (int i = 0; i < n; i++) d[i] = s[i];
}

struct CutCtx {
    // the recording
    const Dav1dGpuRecBlock *blocks;
    const int32_t *baux_off;   // per block: offset into baux, -1 none; a COMPOUND_SEG chroma
                               // INTER_MASK block: -2 - the last INTER_WMASK block's index
    const uint8_t *baux;       // (16-byte aligned entries)
    const RecRes *res;
    int32_t *res_at[3];        // per 4x4: the residual recorded there (res_base + index)
    int32_t mw[3], pw[3], ph[3], ds_px[3];
    int32_t res_base, bpp, top_on, sbl[3];
    RefInfo ref[DGPU_MAX_REFS][3];
    Hdr *hdr;
    // count pass
    BlockCnt *cnt;
    int32_t *auxend;   // per block: its aux-pool bytes, unrounded
    // write pass
    const BlockCnt *base;
    Dav1dGpuUnit *cu;          // cells in decode order
    Dav1dGpuIntraEdge *crec;
    int32_t *caux, *csort, *rawc;
    LvJob *jobs;
    uint8_t *auxp;
    EmuJob *emu;
    Dav1dGpuUnit *xu;          // launch-ahead units, decode order
    int32_t *xa;
};

// the producer lookups of a cell (the level rule): the 4x4s its edges (or CfL
// luma, or an inter-intra residual's prediction) read.  W = false counts
// them; W = true passes each writer (or -1) to put
template <bool W, class F>
__host__ __device__ inline int lookups(const LvJob &j, const int32_t *own_p, int w4p, const int32_t *own0, int w40,
                                       F &&put) {
    int n = 0;
    auto cell = [&](int cx, int cy) {
        n++;
        if constexpr (W) put(own_p[(size_t)cy * w4p + cx]);
    };
    const int x4 = j.x4, y4 = j.y4, cw4 = j.cw4, ch4 = j.ch4, W4 = j.W4, H4 = j.H4, nd = j.nd;
    const bool hl = j.fl & LvJob::HL, ht = j.fl & LvJob::HT;
    if (nd & 1) {
        if (hl) {
            for (int q = y4; q < min(y4 + ch4, H4); q++) cell(x4 - 1, q);
            if ((nd & 16) && y4 + ch4 < H4 && (j.fl & LvJob::BL))
                for (int q = y4 + ch4; q < min(y4 + 2 * ch4, H4); q++) cell(x4 - 1, q);
        } else if (ht) {
            cell(x4, y4 - 1);
        }
    }
    if (nd & 2) {
        if (ht) {
            for (int q = x4; q < min(x4 + cw4, W4); q++) cell(q, y4 - 1);
            if ((nd & 8) && x4 + cw4 < W4 && (j.fl & LvJob::TR))
                for (int q = x4 + cw4; q < min(x4 + 2 * cw4, W4); q++) cell(q, y4 - 1);
        } else if (hl) {
            cell(x4 - 1, y4);
        }
    }
    if (j.fl & LvJob::IIRES) {   // the block's inter-intra prediction cell (given as -2 - link)
        n++;
        if constexpr (W) put(-2 - j.link);
    }
    if (nd & 4) {
        if (hl && ht) cell(x4 - 1, y4 - 1);
        else if (hl) cell(x4 - 1, y4);
        else if (ht) cell(x4, y4 - 1);
    }
    if (j.fl & LvJob::CFL) {
        for (int cy = 2 * y4; cy < 2 * (y4 + ch4); cy++)
            for (int cx = 2 * x4; cx < 2 * (x4 + cw4); cx++) {
                n++;
                if constexpr (W) put(own0[(size_t)cy * w40 + cx]);
            }
    }
    return n;
}

// One block: W = false counts into c.cnt[bi], W = true writes at c.base[bi].
// Returns 0 or E_BAD (a recording the flush rejects).
template <bool W>
__host__ __device__ inline int cut_block(const CutCtx &c, int bi) {
    const Dav1dGpuRecBlock b = c.blocks[bi];
    const int tw = tx_w(b.tx), th = tx_h(b.tx);
    const int p = b.plane, w4p = c.mw[p];
    const int bpp = c.bpp;
    const bool inter = is_mc_kind(b.kind);
    const bool cfl = b.kind == DGPU_PRED_CFL, pal = b.kind == DGPU_PRED_PAL;
    const bool pre = is_prelaunch_kind(b.kind);
    const int32_t bo = c.baux_off[bi];
    const uint8_t *bdata = bo >= 0 ? c.baux + bo : nullptr;
    const int bw4 = b.w / 4, bh4 = b.h / 4, tw4 = tw / 4, th4 = th / 4;
    const int bwc = min(b.w, c.pw[p] - b.x), bhc = min(b.h, c.ph[p] - b.y);
    const int bw4c = bwc / 4, bh4c = bhc / 4;
    const int ds_px = c.ds_px[p];
    // the block's bases (write pass; scalars, so nothing of them goes to
    // scratch) and its running counts
    int32_t b_aux = 0, b_erows = 0, b_edge = 0, b_cells = 0;
    long long b_ejobs = 0, b_xu = 0;
    if constexpr (W) {
        const BlockCnt &q = c.base[bi];
        b_cells = (int32_t)q.v[C_CELLS];
        b_aux = (int32_t)q.v[C_AUX];
        b_ejobs = q.v[C_EJOBS];
        b_erows = (int32_t)q.v[C_EROWS];
        b_xu = q.v[C_XU];
        b_edge = (int32_t)q.v[C_EDGE];
    }
    int n_cells = 0, n_ejobs = 0, n_xu = 0, n_res = 0;
    int32_t aux_end = 0, erows = 0, edge = 0;
    long long n_raw = 0;
    auto aux_alloc = [&](int nbytes) -> int32_t {   // 16-byte aligned records
        const int32_t o = (aux_end + 15) & ~15;
        aux_end = o + nbytes;
        return b_aux + o;
    };
    // a clamped copy of the fw x fh footprint at (x0, y0) of ref slot / plane
    // in a band of new scratch rows; returns its scratch offset
    auto emu_band = [&](int x0, int y0, int fw, int fh, int slot, int plane) -> int32_t {
        const int32_t o = (b_erows + erows) * kEmuStride;
        if constexpr (W)
            c.emu[b_ejobs + n_ejobs] = EmuJob{x0, y0, o, (uint8_t)fw, (uint8_t)fh, (uint8_t)slot, (uint8_t)plane};
        n_ejobs++;
        erows += fh;
        return o;
    };
    auto refok = [&](int rr) { return rr < DGPU_MAX_REFS && c.ref[rr][p].ok; };
    // every reference an inter block reads must be given
    if (inter || pre) {
        const int nref = b.kind == DGPU_PRED_INTER || b.kind == DGPU_PRED_WARP || b.kind == DGPU_PRED_INTER_OBMC ? 1
                         : b.kind == DGPU_PRED_INTER_SCALED ? *(const int32_t *)bdata : 2;
        for (int k = 0; k < nref; k++)
            if (!refok(b.ref[k])) return E_BAD;
    }
    int32_t wm_off = -1, wm_w = 0, wm_h = 0;   // INTER_WMASK: its seg mask (4:2:0)
    int32_t mask_base = 0, mask_stride = 0;    // INTER_MASK: the block's mask
    if (b.kind == DGPU_PRED_INTER_MASK) {
        if (bdata) {
            mask_base = aux_alloc(b.w * b.h);
            if constexpr (W) bcopy(c.auxp + mask_base, bdata, b.w * b.h);
            mask_stride = b.w;
        } else {   // COMPOUND_SEG chroma: the luma block's w_mask output (its first aux record)
            if (bo > -2) return E_BAD;
            const int lk = -2 - bo;
            const int lw = c.blocks[lk].w >> 1, lh = c.blocks[lk].h >> 1;
            if (b.w != lw || b.h != lh) return E_BAD;
            if constexpr (W) mask_base = (int32_t)c.base[lk].v[C_AUX];
            mask_stride = lw;
        }
    }
    if (pre) {   // prediction units of at most 32 x 32, no residual
        const int uw = min(b.w, 32), uh = min(b.h, 32), utx = tx_of(uw, uh);
        if (utx < 0) return E_BAD;
        if (b.kind == DGPU_PRED_INTER_WMASK) {   // its seg mask at the 4:2:0 chroma resolution
            wm_w = b.w >> 1;
            wm_h = b.h >> 1;
            wm_off = aux_alloc(wm_w * wm_h);
        }
        // mc()'s emu_edge decision per prediction unit and reference
        // (src/recon_tmpl.c:986-999): the unit kernel reads a W+7 x H+7
        // footprint with aligned 16-byte row loads (up to 16 bytes past
        // it), so a direct read needs all of that inside the reference
        // picture, else the footprint is read from a clamped copy
        auto mc_inside = [&](int rr, int ix, int iy) {
            const RefInfo &ri = c.ref[rr][p];
            return ix - 3 >= 0 && iy - 3 >= 0 && ix + uw + 4 <= ri.w && iy + uh + 4 <= ri.h &&
                   (iy + uh + 4 < ri.h || (long long)(ix + uw + 4) * bpp + 16 <= ri.stride_b);
        };
        auto mc_emu = [&](int rr, int ix, int iy) {   // the copy's (0, 0) pixel offset
            return emu_band(ix - 3, iy - 3, uw + 7, uh + 7, rr, p) + 3 * kEmuStride + 3;
        };
        for (int oy = 0; oy < bhc; oy += uh)
            for (int ox = 0; ox < bwc; ox += uw) {
                const int ux = b.x + ox, uy = b.y + oy;
                Dav1dGpuUnit u;
                memset(&u, 0, sizeof(u));
                u.dst_off = uy * ds_px + ux;
                u.tx = (uint8_t)utx;
                u.plane = (uint8_t)p;
                u.pred = (uint8_t)b.kind;
                u.txtp = DGPU_NO_RESIDUAL;
                u.bw4 = (uint8_t)bw4;
                u.bh4 = (uint8_t)bh4;
                for (int k = 0; k < 2; k++) {
                    const int rr = b.ref[k];
                    const int rs = refok(rr) ? c.ref[rr][p].stride_px : 0;
                    u.p.inter.src_off[k] = (uy + (b.mvy[k] >> 4)) * rs + ux + (b.mvx[k] >> 4);
                    u.p.inter.mx[k] = (uint8_t)(b.mvx[k] & 15);
                    u.p.inter.my[k] = (uint8_t)(b.mvy[k] & 15);
                    u.p.inter.ref[k] = (uint8_t)rr;
                }
                u.p.inter.filter2d = b.filter2d;
                u.p.inter.weight = b.weight;
                // WMASK: both refs' footprints; OBMC: the block's own put
                const int nmc = b.kind == DGPU_PRED_INTER_WMASK ? 2 : b.kind == DGPU_PRED_INTER_OBMC ? 1 : 0;
                for (int k = 0; k < nmc; k++) {
                    const int rr = b.ref[k], ix = ux + (b.mvx[k] >> 4), iy = uy + (b.mvy[k] >> 4);
                    if (!mc_inside(rr, ix, iy)) {
                        u.p.inter.src_off[k] = mc_emu(rr, ix, iy);
                        u.p.inter.ref[k] = (uint8_t)DGPU_REC_EMU_SLOT;
                    }
                }
                int32_t ao = 0;
                if (b.kind == DGPU_PRED_INTER_WMASK) {
                    ao = wm_off + (oy >> 1) * wm_w + (ox >> 1);
                } else if (b.kind == DGPU_PRED_WARP) {   // abcd, then the unit's 8x8s
                    const int gw = b.w / 8, nx = uw / 8, ny = uh / 8;
                    ao = aux_alloc(16 + 8 * nx * ny);
                    // warp_affine's emu_edge (src/recon_tmpl.c:1168-1177): an
                    // 8x8 reads 15 x 15 pixels at (x - 3, y - 3); the kernel's
                    // aligned loads reach 16 bytes past column x + 11.  When
                    // any 8x8 of the unit leaves the picture, every 8x8 of it
                    // is read from a clamped copy (exact for the ones inside):
                    // 15-row strips, 8x8s 16 px apart, positions rewritten to
                    // the copy and the strip base in src_off[0] (the kernel
                    // adds it); otherwise src_off[0] = 0
                    const int rr = b.ref[0];
                    const RefInfo &ri = c.ref[rr][p];
                    bool all_in = true;
                    for (int i = 0; i < nx * ny && all_in; i++) {
                        const int sy = i / nx, sx = i % nx;
                        const int16_t *xy = (const int16_t *)(bdata + 16 + 8 * ((oy / 8 + sy) * gw + ox / 8 + sx));
                        all_in = xy[0] - 3 >= 0 && xy[1] - 3 >= 0 && xy[0] + 12 <= ri.w && xy[1] + 12 <= ri.h &&
                                 (xy[1] + 12 < ri.h || (long long)(xy[0] + 12) * bpp + 16 <= ri.stride_b);
                    }
                    if constexpr (W) {
                        bcopy(c.auxp + ao, bdata, 8);
                        for (int sy = 0; sy < ny; sy++)
                            bcopy(c.auxp + ao + 16 + 8 * sy * nx, bdata + 16 + 8 * ((oy / 8 + sy) * gw + ox / 8), 8 * nx);
                    }
                    u.p.inter.src_off[0] = 0;
                    if (!all_in) {
                        const int32_t band = (b_erows + erows) * kEmuStride;
                        for (int sy = 0; sy < ny; sy++)
                            for (int sx = 0; sx < nx; sx++) {
                                const int16_t *xy = (const int16_t *)(bdata + 16 + 8 * ((oy / 8 + sy) * gw + ox / 8 + sx));
                                if constexpr (W) {
                                    c.emu[b_ejobs + n_ejobs] =
                                        EmuJob{xy[0] - 3, xy[1] - 3, band + 15 * sy * kEmuStride + 16 * sx, 15, 15,
                                               (uint8_t)rr, (uint8_t)p};
                                    int16_t *e8 = (int16_t *)(c.auxp + ao + 16 + 8 * (sy * nx + sx));
                                    e8[0] = (int16_t)(16 * sx + 3);
                                    e8[1] = (int16_t)(15 * sy + 3);
                                }
                                n_ejobs++;
                            }
                        erows += 15 * ny;
                        u.p.inter.src_off[0] = band;
                        u.p.inter.ref[0] = (uint8_t)DGPU_REC_EMU_SLOT;
                    }
                } else if (b.kind == DGPU_PRED_INTER_OBMC) {   // the laps overlapping the unit
                    const int n = *(const int32_t *)bdata;
                    const ObmcBlockLap *lb = (const ObmcBlockLap *)(bdata + 16);
                    int ne = 0;
                    for (int k = 0; k < n; k++) {
                        const ObmcBlockLap &e = lb[k];
                        const int x0 = max((int)e.x0 - ox, 0), x1 = min((int)e.x1 - ox, uw);
                        const int y0 = max((int)e.y0 - oy, 0), y1 = min((int)e.y1 - oy, uh);
                        if (x0 >= x1 || y0 >= y1) continue;
                        if (e.ref >= DGPU_REC_EMU_SLOT || !refok(e.ref) || e.filter2d > 9) return E_BAD;
                        ne++;
                    }
                    ao = aux_alloc(16 + 16 * ne);
                    if constexpr (W) *(int32_t *)(c.auxp + ao) = ne;
                    int ie = 0;
                    for (int k = 0; k < n; k++) {
                        const ObmcBlockLap &e = lb[k];
                        const int x0 = max((int)e.x0 - ox, 0), x1 = min((int)e.x1 - ox, uw);
                        const int y0 = max((int)e.y0 - oy, 0), y1 = min((int)e.y1 - oy, uh);
                        if (x0 >= x1 || y0 >= y1) continue;
                        const int rs = c.ref[e.ref][p].stride_px;
                        ObmcUnitLap q;
                        q.src_off = (uy + (e.mvy >> 4)) * rs + ux + (e.mvx >> 4);
                        q.mx = (uint8_t)(e.mvx & 15);
                        q.my = (uint8_t)(e.mvy & 15);
                        q.filter2d = e.filter2d;
                        q.ref = e.ref;
                        q.x0 = (uint8_t)x0, q.y0 = (uint8_t)y0, q.x1 = (uint8_t)x1, q.y1 = (uint8_t)y1;
                        q.lap_w4 = e.lap_w4, q.lap_h4 = e.lap_h4, q.dir = e.dir;
                        q.mask_off = (uint8_t)(e.mask_off + (e.dir ? ox : oy));
                        const int ix = ux + (e.mvx >> 4), iy = uy + (e.mvy >> 4);
                        if (!mc_inside(e.ref, ix, iy)) {   // the lap's prediction reads the unit's whole footprint
                            q.src_off = mc_emu(e.ref, ix, iy);
                            q.ref = (uint8_t)DGPU_REC_EMU_SLOT;
                        }
                        if constexpr (W) memcpy(c.auxp + ao + 16 + 16 * ie, &q, 16);
                        ie++;
                    }
                } else {   // INTER_SCALED: the unit's integer position and phase (running sums)
                    const int n = *(const int32_t *)bdata;
                    const ScaledBlockRef *sb = (const ScaledBlockRef *)(bdata + 16);
                    ao = aux_alloc(16 + 16 * n);
                    if constexpr (W) *(int32_t *)(c.auxp + ao) = n;
                    for (int k = 0; k < n; k++) {
                        const int rr = b.ref[k];
                        const RefInfo &ri = c.ref[rr][p];
                        const int px_ = sb[k].mx + ox * sb[k].dx, py_ = sb[k].my + oy * sb[k].dy;
                        const int ix = sb[k].x + (px_ >> 10), iy = sb[k].y + (py_ >> 10);
                        ScaledUnitRef q;
                        q.src_off = iy * ri.stride_px + ix;
                        q.mx = (uint16_t)(px_ & 1023), q.my = (uint16_t)(py_ & 1023);
                        q.dx = sb[k].dx, q.dy = sb[k].dy;
                        q.pad_ = 0;
                        // the scaled mc()'s emu_edge (src/recon_tmpl.c:1036-1046): the
                        // kernel reads columns ix - 3 .. ((mx + (W - 1) dx) >> 10) + 4
                        // past ix and rows iy - 3 .. ((my + (H - 1) dy) >> 10) + 4 past iy
                        // (its row count capped at 2H + 8), pixel by pixel
                        const int fw = ((q.mx + (uw - 1) * q.dx) >> 10) + 8;
                        const int fh = min(((q.my + (uh - 1) * q.dy) >> 10) + 8, 2 * uh + 8);
                        if (ix - 3 < 0 || iy - 3 < 0 || ix - 3 + fw > ri.w || iy - 3 + fh > ri.h) {
                            q.src_off = emu_band(ix - 3, iy - 3, fw, fh, rr, p) + 3 * kEmuStride + 3;
                            u.p.inter.ref[k] = (uint8_t)DGPU_REC_EMU_SLOT;
                        }
                        if constexpr (W) memcpy(c.auxp + ao + 16 + 16 * k, &q, 16);
                    }
                    if (n == 1) u.p.inter.weight = 0;
                }
                if constexpr (W) {
                    memcpy(&c.xu[b_xu + n_xu], &u, sizeof(u));
                    c.xa[b_xu + n_xu] = ao;
                }
                n_xu++;
            }
    }
    // the transform cells; an INTER_INTRA block first gets one cell for
    // the whole block's prediction (recon_b_inter predicts the block,
    // :1540-1580, then adds the residuals), its transform cells become
    // residual-only cells that read it
    const bool iib = b.kind == DGPU_PRED_INTER_INTRA;
    const int ncx = (bwc + tw - 1) / tw, ncy = (bhc + th - 1) / th;
    const int32_t iic_at = b_cells;   // the inter-intra block's prediction cell (its first)
    for (int k = iib ? -1 : 0; k < ncx * ncy; k++) {
        const bool iic = k < 0;
        const int ox = iic ? 0 : (k % ncx) * tw, oy = iic ? 0 : (k / ncx) * th;
        const int ctw = iic ? b.w : tw, cth = iic ? b.h : th, ctw4 = ctw / 4, cth4 = cth / 4;
        const int ux = b.x + ox, uy = b.y + oy, x4 = ux / 4, y4 = uy / 4;
        Dav1dGpuUnit u;
        memset(&u, 0, sizeof(u));
        Dav1dGpuIntraEdge e;
        memset(&e, 0, sizeof(e));
        int32_t caux = 0, sortmode = 0;
        u.dst_off = uy * ds_px + ux;
        u.tx = (uint8_t)(iic ? tx_of(b.w, b.h) : b.tx);
        u.plane = (uint8_t)p;
        u.pred = (uint8_t)((pre || (iib && !iic)) ? DGPU_PRED_NONE : b.kind);
        u.txtp = DGPU_NO_RESIDUAL;
        const int32_t rs_ = iic ? -1 : c.res_at[p][(size_t)y4 * w4p + x4];
        const int ri = rs_ >= c.res_base ? rs_ - c.res_base : -1;   // (an earlier flush's: none)
        if (ri >= 0 && c.res[ri].tx == b.tx) {
            const RecRes q = c.res[ri];
            u.txtp = (uint8_t)q.txtp;
            u.nzw = (uint8_t)q.nzw;
            u.nzh = (uint8_t)q.nzh;
            u.coef_off = q.coef;
            n_res++;
        } else if (ri >= 0) {
            return E_BAD;   // a residual whose size differs from its block's transforms
        } else if (pre || (iib && !iic)) {
            continue;   // predicted elsewhere, nothing to add
        }
        e.unit = -1;
        e.x4 = (int16_t)x4;
        e.y4 = (int16_t)y4;
        e.w4 = (int16_t)(b.tile_x1 / 4);
        e.h4 = (int16_t)(b.tile_y1 / 4);
        int nd = 0;
        const bool hl = ux > b.tile_x0, ht = uy > b.tile_y0;
        // the TOP_SB_EDGE flag of an edge record whose top row is a
        // superblock's top (per transform block, recon_tmpl.c:1276 / :1395;
        // inter-intra per block, :1665 / :1794)
        const int top_sb = c.top_on && ht && (uy & ((1 << c.sbl[p]) - 1)) == 0 ? DGPU_IE_TOP_SB_EDGE : 0;
        if (pre || (iib && !iic)) {   // PRED_NONE: the residual onto the prediction
            sortmode = 0;
        } else if (pal) {   // pal_pred: palette, then the unit's rows of the index map
            const int bw2 = b.w / 2;
            caux = aux_alloc(16 + (tw / 2) * th);
            if constexpr (W) {
                bcopy(c.auxp + caux, bdata, 8 * bpp);
                for (int yy = 0; yy < th; yy++)
                    bcopy(c.auxp + caux + 16 + yy * (tw / 2), bdata + 8 * bpp + (oy + yy) * bw2 + ox / 2, tw / 2);
            }
            sortmode = 15;
        } else if (inter || iic) {
            u.bw4 = (uint8_t)bw4;
            u.bh4 = (uint8_t)bh4;
            for (int k2 = 0; k2 < 2; k2++) {
                const int rr = b.ref[k2];
                // every reference an inter block reads must be given
                const bool used = k2 == 0 || (b.kind != DGPU_PRED_INTER && !iic);
                if (used && !refok(rr)) return E_BAD;
                const int rs = c.ref[rr][p].stride_px;   // (given with a NULL plane too)
                const int ix = ux + (b.mvx[k2] >> 4), iy = uy + (b.mvy[k2] >> 4);
                u.p.inter.src_off[k2] = iy * rs + ix;
                u.p.inter.mx[k2] = (uint8_t)(b.mvx[k2] & 15);
                u.p.inter.my[k2] = (uint8_t)(b.mvy[k2] & 15);
                u.p.inter.ref[k2] = (uint8_t)rr;
                if (used) {
                    // the unit kernel reads the footprint with both 8-tap
                    // margins whatever the fraction, and its aligned row loads
                    // may run up to 16 bytes past the last pixel: direct only
                    // when all of that stays inside the picture, else a
                    // clamped copy
                    const RefInfo &rf = c.ref[rr][p];
                    const bool inside = ix - 3 >= 0 && iy - 3 >= 0 && ix + ctw + 4 <= rf.w && iy + cth + 4 <= rf.h &&
                                        (iy + cth + 4 < rf.h || (ix + ctw + 4) * bpp + 16 <= rs * bpp);
                    if (!inside) {
                        u.p.inter.src_off[k2] = emu_band(ix - 3, iy - 3, ctw + 7, cth + 7, rr, p) + 3 * kEmuStride + 3;
                        u.p.inter.ref[k2] = (uint8_t)DGPU_REC_EMU_SLOT;
                    }
                }
            }
            u.p.inter.filter2d = b.filter2d;
            u.p.inter.weight = b.kind == DGPU_PRED_INTER_WAVG ? b.weight : 0;
            if (b.kind == DGPU_PRED_INTER_MASK) caux = mask_base + oy * mask_stride + ox;
            sortmode = b.filter2d;
            if (iic) {   // the intra half: edges gathered by the wavefront like an INTRA unit's
                // record: edge_off (unused when gathered), mode, angle, then the mask offset
                caux = aux_alloc(16 + b.w * b.h);
                const int32_t moff = caux + 16;
                if constexpr (W) {
                    c.auxp[caux + 4] = b.mode;
                    memcpy(c.auxp + caux + 8, &moff, 4);
                    bcopy(c.auxp + moff, bdata, b.w * b.h);
                }
                // prepare_intra_edges with no edge flags, no edge filter, angle 0 (:1551-1566)
                e.mode = b.mode;
                e.angle = 0;
                e.flags = (uint8_t)((hl ? DGPU_IE_HAVE_LEFT : 0) | (ht ? DGPU_IE_HAVE_TOP : 0) | top_sb);
                const int m = remap_mode(e.mode, 0, hl, ht);
                nd = needs(m);
                sortmode = 16 + m;
            }
        } else {
            int fl = (hl ? DGPU_IE_HAVE_LEFT : 0) | (ht ? DGPU_IE_HAVE_TOP : 0) | top_sb;
            if (!cfl) {   // recon_tmpl.c:1252-1266 (blocks up to 64 wide: one 64x64 step)
                const int x = ox / 4, y = oy / 4;
                const bool sb_tr = b.flags & DGPU_IE_TOP_HAS_RIGHT, sb_bl = b.flags & DGPU_IE_LEFT_HAS_BOTTOM;
                if (!((y > 0 || !sb_tr) && x + tw4 >= bw4c)) fl |= DGPU_IE_TOP_HAS_RIGHT;
                if (!(x > 0 || (!sb_bl && y + th4 >= bh4c))) fl |= DGPU_IE_LEFT_HAS_BOTTOM;
                fl |= b.flags & (DGPU_IE_FILTER_EDGE | DGPU_IE_SMOOTH);
                e.mode = b.mode;
                e.angle = b.angle;
                u.p.intra.max_w = (uint16_t)(c.pw[p] - ux);
                u.p.intra.max_h = (uint16_t)(c.ph[p] - uy);
            } else {
                e.mode = DGPU_DC_PRED;   // cfl_pred's DC source (:1395-1410)
                e.angle = 0;
                u.p.cfl.alpha = b.cfl_alpha;
                u.p.cfl.pad_wh = b.mode;   // cfl_ac's w_pad | h_pad << 4 (:1372-1380)
                u.p.cfl.luma_off = (2 * uy) * c.ds_px[0] + 2 * ux;
            }
            e.flags = (uint8_t)fl;
            u.p.intra.edge_off = b_edge + edge + 2 * th;   // CFL: the same field
            edge += 2 * th + 2 * tw + 1;
            const int m = remap_mode(e.mode, e.angle, hl, ht);
            nd = needs(m);
            sortmode = 16 + m;
        }
        // the level pass reads the cell's geometry and edge needs
        LvJob j;
        memset(&j, 0, sizeof(j));
        j.x4 = (int16_t)x4;
        j.y4 = (int16_t)y4;
        j.W4 = e.w4;
        j.H4 = e.h4;
        j.p = (uint8_t)p;
        j.cw4 = (uint8_t)ctw4;
        j.ch4 = (uint8_t)cth4;
        j.nd = (uint8_t)nd;
        j.fl = (uint8_t)((hl ? LvJob::HL : 0) | (ht ? LvJob::HT : 0) | ((e.flags & DGPU_IE_TOP_HAS_RIGHT) ? LvJob::TR : 0) |
                         ((e.flags & DGPU_IE_LEFT_HAS_BOTTOM) ? LvJob::BL : 0) | (cfl ? LvJob::CFL : 0) |
                         ((iib && !iic) ? LvJob::IIRES : 0) | (iic ? LvJob::IIC : 0));
        j.link = iib && !iic ? iic_at : -1;
        const int nl = lookups<false>(j, nullptr, 0, nullptr, 0, [](int32_t) {});
        if constexpr (W) {
            const long long ci = (long long)b_cells + n_cells;
            memcpy(&c.cu[ci], &u, sizeof(u));
            memcpy(&c.crec[ci], &e, sizeof(e));
            c.caux[ci] = caux;
            c.csort[ci] = sortmode;
            memcpy(&c.jobs[ci], &j, sizeof(j));
            c.rawc[ci] = nl;
        }
        n_raw += nl;
        n_cells++;
    }
    if constexpr (!W) {
        BlockCnt &o = c.cnt[bi];
        o.v[C_CELLS] = n_cells;
        o.v[C_AUX] = (aux_end + 15) & ~15;
        o.v[C_EJOBS] = n_ejobs;
        o.v[C_EROWS] = erows;
        o.v[C_XU] = n_xu;
        o.v[C_EDGE] = edge;
        o.v[C_RES] = n_res;
        o.v[C_RAW] = n_raw;
        c.auxend[bi] = aux_end;
        if (aux_end) amax(&c.hdr->last_aux, bi);
    }
    return 0;
}

}  // namespace rec
