// itx.hip -- Dav1dInvTxfmDSPContext (src/itx.h:42-44) on gfx950.
//
// Per-call kernel: one 64-lane workgroup per transform.  Pass 1: lane y
// owns row y (min(h,32) rows) as a register array and runs the horizontal
// 1-D transform; rounding/clipping to the column range, transpose through
// LDS; pass 2: lane x owns column x and runs the vertical transform, then
// adds to the prediction (src/itx_tmpl.c:40-100).
#include "dav1d_gpu.h"
#include "dsp_common.hpp"
#include "runtime.hpp"

#include <string.h>
#include <utility>

namespace dgpu {

// The reference's 156 instantiations per bitdepth (src/itx_tmpl.c:142-160,
// 201-268): all 16 types up to 16 px per side except 16x16 (12 types),
// DCT_DCT + IDTX with a 32 side, DCT_DCT only with a 64 side; WHT 4x4.
__host__ __device__ constexpr bool itx_supported(int tx, int tp) {
    if (tp == DGPU_WHT_WHT) return tx == DGPU_TX_4X4;
    const int w = tx_info(tx).w, h = tx_info(tx).h, m = w > h ? w : h;
    if (m == 64) return tp == DGPU_DCT_DCT;
    if (m == 32) return tp == DGPU_DCT_DCT || tp == DGPU_IDTX;
    if (w == 16 && h == 16) return tp <= DGPU_H_DCT;
    return true;
}

template <int BPC, int TX>
__global__ __launch_bounds__(64) void k_itx(typename Px<BPC>::pixel *dst, ptrdiff_t ds,
                                            typename Px<BPC>::coef *coef, int eob, int txtp,
                                            int bdmax) {
    constexpr int W = tx_info(TX).w, H = tx_info(TX).h, SHIFT = tx_info(TX).shift;
    constexpr int SW = W < 32 ? W : 32, SH = H < 32 ? H : 32;
    constexpr bool RECT2 = W * 2 == H || H * 2 == W;
    constexpr int RND = (1 << SHIFT) >> 1;
    __shared__ int t[H][W + 1];
    const int lane = threadIdx.x;
    using pixel = typename Px<BPC>::pixel;

    if (TX == DGPU_TX_4X4 && txtp == DGPU_WHT_WHT) {  // src/itx_tmpl.c:166-185
        if (lane < 4) {
            int c[4];
#pragma unroll
            for (int x = 0; x < 4; x++) c[x] = coef[lane + x * 4] >> 2;
            wht4<1>(c);
#pragma unroll
            for (int x = 0; x < 4; x++) t[lane][x] = c[x];
        }
        __syncthreads();
        if (lane < 16) coef[lane] = 0;
        if (lane < 4) {
            int c[4];
#pragma unroll
            for (int y = 0; y < 4; y++) c[y] = t[y][lane];
            wht4<1>(c);
#pragma unroll
            for (int y = 0; y < 4; y++) {
                pixel &d = dst[y * ds + lane];
                d = (pixel)clampi(d + c[y], 0, bdmax);
            }
        }
        return;
    }

    if (txtp == DGPU_DCT_DCT && eob < 1) {  // DC-only, src/itx_tmpl.c:53-65
        int dc = coef[0];
        if (RECT2) dc = r8s(dc);
        dc = r8s(dc);
        dc = (dc + RND) >> SHIFT;
        dc = (dc * 181 + 128 + 2048) >> 12;
        for (int i = lane; i < W * H; i += 64) {
            pixel &d = dst[(i / W) * ds + (i % W)];
            d = (pixel)clampi(d + dc, 0, bdmax);
        }
        __syncthreads();
        if (lane == 0) coef[0] = 0;
        return;
    }

    const Clip rc = ItxClip<BPC>::row(bdmax), cc = ItxClip<BPC>::col(bdmax);
    if (lane < SH) {
        int c[W];
#pragma unroll
        for (int x = 0; x < W; x++) {
            int v = x < SW ? (int)coef[lane + x * SH] : 0;
            c[x] = RECT2 ? r8s(v) : v;
        }
        tx1d<W, 1, BPC == 8>(kind_h(txtp), c, rc);
#pragma unroll
        for (int x = 0; x < W; x++) t[lane][x] = cc((c[x] + RND) >> SHIFT);
    }
    __syncthreads();
    for (int i = lane; i < SW * SH; i += 64) coef[i] = 0;
    if (lane < W) {
        int c[H];
#pragma unroll
        for (int y = 0; y < H; y++) c[y] = y < SH ? t[y][lane] : 0;
        tx1d<H, 1, BPC == 8>(kind_v(txtp), c, cc);
#pragma unroll
        for (int y = 0; y < H; y++) {
            pixel &d = dst[y * ds + lane];
            d = (pixel)clampi(d + ((c[y] + 8) >> 4), 0, bdmax);
        }
    }
}

template <int BPC, int TX, int TP>
static bool itx_entry(typename Px<BPC>::pixel *dst, ptrdiff_t stride,
                      typename Px<BPC>::coef *coef, int eob, int bdmax) {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    constexpr long B = sizeof(P);
    constexpr int W = tx_info(TX).w, H = tx_info(TX).h;
    constexpr int SW = W < 32 ? W : 32, SH = H < 32 ? H : 32;
    Stager st;
    const int ic = st.inout1(coef, (long)SW * SH * sizeof(C));
    const int od = st.inout(dst, stride, 0, W * B, 0, H);
    if (!st.upload()) return false;
    k_itx<BPC, TX><<<1, 64, 0, st.stream()>>>(st.origin<P>(od), st.pitch(od) / B, st.origin<C>(ic),
                                              eob, TP, bdmax);
    return st.finish();
}

// The caller's entries before dav1d_itx_dsp_init_gpu_* overwrote them (run
// when the GPU path fails: runtime.hpp's error contract).
static Dav1dInvTxfmDSPContext_8bpc g_fb8;
static Dav1dInvTxfmDSPContext_16bpc g_fb16[2];   // 10 bit, 12 bit (fb16_slot)

template <int TX, int TP>
static void itx8(uint8_t *d, ptrdiff_t s, int16_t *c, int eob) {
    DGPU_OR_FALLBACK((itx_entry<8, TX, TP>(d, s, c, eob, 255)), g_fb8.itxfm_add[TX][TP], d, s, c, eob);
}
template <int TX, int TP>
static void itx16(uint16_t *d, ptrdiff_t s, int32_t *c, int eob, int bdmax) {
    DGPU_OR_FALLBACK((itx_entry<16, TX, TP>(d, s, c, eob, bdmax)), g_fb16[fb16_slot_bdmax(bdmax)].itxfm_add[TX][TP], d, s, c, eob,
                     bdmax);
}

template <typename Ctx, int TX, int TP>
static void fill_one(Ctx *c, bool hbd) {
    if constexpr (itx_supported(TX, TP)) {
        if (hbd) ((Dav1dInvTxfmDSPContext_16bpc *)c)->itxfm_add[TX][TP] = itx16<TX, TP>;
        else ((Dav1dInvTxfmDSPContext_8bpc *)c)->itxfm_add[TX][TP] = itx8<TX, TP>;
    }
}

template <typename Ctx, int TX, int... TP>
static void fill_types(Ctx *c, bool hbd, std::integer_sequence<int, TP...>) {
    (fill_one<Ctx, TX, TP>(c, hbd), ...);
}

template <typename Ctx, int... TX>
static void fill_all(Ctx *c, bool hbd, std::integer_sequence<int, TX...>) {
    (fill_types<Ctx, TX>(c, hbd, std::make_integer_sequence<int, DGPU_N_TX_TYPES_PLUS_LL>()), ...);
}

}  // namespace dgpu

using namespace dgpu;

// bitfn(dav1d_itx_dsp_init) replacement, src/itx_tmpl.c:200-284.  Entries
// the reference leaves unset stay NULL; `bpc` selects nothing here (one
// kernel set covers 10 and 12 bit through bitdepth_max).  The _gpu_ hooks
// keep the caller's previous entries as fallbacks, per bit depth for 16bpc
// (the caller's 10- and 12-bit entries differ).
extern "C" void dav1d_itx_dsp_init_gpu_8bpc(Dav1dInvTxfmDSPContext_8bpc *c, int bpc) {
    (void)bpc;
    Dav1dInvTxfmDSPContext_8bpc g{};
    fill_all(&g, false, std::make_integer_sequence<int, DGPU_N_RECT_TX_SIZES>());
    save_fallback(&g_fb8, c, &g);
    fill_all(c, false, std::make_integer_sequence<int, DGPU_N_RECT_TX_SIZES>());
}
extern "C" void dav1d_itx_dsp_init_gpu_16bpc(Dav1dInvTxfmDSPContext_16bpc *c, int bpc) {
    Dav1dInvTxfmDSPContext_16bpc g{};
    fill_all(&g, true, std::make_integer_sequence<int, DGPU_N_RECT_TX_SIZES>());
    save_fallback(&g_fb16[fb16_slot(bpc)], c, &g);
    fill_all(c, true, std::make_integer_sequence<int, DGPU_N_RECT_TX_SIZES>());
}
extern "C" void dav1d_itx_dsp_init_8bpc(Dav1dInvTxfmDSPContext_8bpc *c, int bpc) {
    (void)bpc;
    memset(c, 0, sizeof(*c));
    fill_all(c, false, std::make_integer_sequence<int, DGPU_N_RECT_TX_SIZES>());
}
extern "C" void dav1d_itx_dsp_init_16bpc(Dav1dInvTxfmDSPContext_16bpc *c, int bpc) {
    (void)bpc;
    memset(c, 0, sizeof(*c));
    fill_all(c, true, std::make_integer_sequence<int, DGPU_N_RECT_TX_SIZES>());
}
