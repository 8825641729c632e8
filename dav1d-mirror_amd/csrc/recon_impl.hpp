// recon_impl.hpp -- batch-tier launch logic (instantiated per bitdepth in
// recon8.hip / recon16.hip so the two heavy TUs compile in parallel).
//
// Two launches at most per frame batch: one over the transform classes with
// both sides <= 32 (the only ones in 4:2:0 content up to 32x32 transforms),
// one over the classes with a 64-point side (their 64-entry register arrays
// would otherwise set the VGPR budget, and hence occupancy, of every wave).
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <utility>

#include "recon_kernel.hpp"

namespace dgpu {

template <bool BIG> struct ClassSet;
template <> struct ClassSet<false> {
    template <int BPC> static constexpr int wave_lds() {
        return MaxWave<BPC, DGPU_TX_4X4, DGPU_TX_8X8, DGPU_TX_16X16, DGPU_TX_32X32, DGPU_RTX_4X8,
                       DGPU_RTX_8X4, DGPU_RTX_8X16, DGPU_RTX_16X8, DGPU_RTX_16X32, DGPU_RTX_32X16,
                       DGPU_RTX_4X16, DGPU_RTX_16X4, DGPU_RTX_8X32, DGPU_RTX_32X8>::v;
    }
};
template <> struct ClassSet<true> {
    template <int BPC> static constexpr int wave_lds() {
        return MaxWave<BPC, DGPU_TX_64X64, DGPU_RTX_32X64, DGPU_RTX_64X32, DGPU_RTX_16X64,
                       DGPU_RTX_64X16>::v;
    }
};

template <int BPC, int TX, bool BIG>
__device__ __forceinline__ void dispatch_one(const ReconArgs<BPC> &a, int cls, int wic, uint8_t *lds) {
    if constexpr (Cls<TX>::BIG == BIG) {
        if (cls == TX) {
            constexpr int U = Cls<TX>::U;
            const int first = a.class_start[TX] + wic * U;
            const int count = min(U, a.class_start[TX + 1] - first);
            recon_units<BPC, TX>(a, first, count, lds);
        }
    }
}

template <int BPC, bool BIG, int... TX>
__device__ __forceinline__ void dispatch(const ReconArgs<BPC> &a, int cls, int wic, uint8_t *lds,
                                         std::integer_sequence<int, TX...>) {
    (dispatch_one<BPC, TX, BIG>(a, cls, wic, lds), ...);
}

template <int BPC, bool BIG>
__global__ __launch_bounds__(256) void k_recon(ReconArgs<BPC> a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int WL = ClassSet<BIG>::template wave_lds<BPC>();
    const int wave = threadIdx.x >> 6;
    const int gw = blockIdx.x * 4 + wave;
    int cls = -1;
#pragma unroll
    for (int c = 0; c < DGPU_N_RECT_TX_SIZES; c++)
        if (gw >= a.wave_start[c] && gw < a.wave_start[c + 1]) cls = c;
    if (cls < 0) return;
    dispatch<BPC, BIG>(a, cls, gw - a.wave_start[cls], lds + wave * WL,
                       std::make_integer_sequence<int, DGPU_N_RECT_TX_SIZES>());
}

static constexpr int units_per_wave(int tx) {
    const int w = tx_info(tx).w, h = tx_info(tx).h;
    const int sh = h < 32 ? h : 32;
    return 64 / (w > sh ? w : sh);
}
static constexpr bool is_big(int tx) { return tx_info(tx).w == 64 || tx_info(tx).h == 64; }

template <int BPC>
static int launch(const Dav1dGpuFrameBatch *b, hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    constexpr int B = BPC / 8;
    if (!b || !b->units || b->n_units < 0) return -1;
    for (int c = 0; c < DGPU_N_RECT_TX_SIZES; c++)
        if (b->class_start[c + 1] < b->class_start[c]) return -2;
    if (b->class_start[0] != 0 || b->class_start[DGPU_N_RECT_TX_SIZES] != b->n_units) return -2;
    if (b->n_units == 0) return 0;

    ReconArgs<BPC> a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) {
        a.dst[p] = (P *)b->dst[p].data;
        a.dst_stride[p] = (int)(b->dst[p].stride / B);
        for (int r = 0; r < DGPU_MAX_REFS; r++) {
            a.ref[r][p] = (const P *)b->ref[r][p].data;
            a.ref_stride[r][p] = (int)(b->ref[r][p].stride / B);
        }
    }
    a.units = b->units;
    a.coef = (C *)b->coef;
    a.edges = (const P *)b->edges;
    memcpy(a.class_start, b->class_start, sizeof(a.class_start));
    a.bdmax = BPC == 8 ? 255 : b->bitdepth_max;
    a.zero_coefs = b->zero_coefs;
    {   // debug-only phase ablation for profiling (never set in production)
        const char *ev = getenv("DAV1D_GPU_ABLATE");
        a.ablate = ev ? atoi(ev) : 0;
    }

    for (int big = 0; big < 2; big++) {
        int acc = 0;
        for (int c = 0; c < DGPU_N_RECT_TX_SIZES; c++) {
            a.wave_start[c] = acc;
            if (is_big(c) == (bool)big) {
                const int n = b->class_start[c + 1] - b->class_start[c];
                acc += (n + units_per_wave(c) - 1) / units_per_wave(c);
            }
        }
        a.wave_start[DGPU_N_RECT_TX_SIZES] = acc;
        if (!acc) continue;
        const dim3 grid((acc + 3) / 4);
        if (big) {
            constexpr int lds = 4 * ClassSet<true>::wave_lds<BPC>();
            static bool attr = false;
            if (!attr) {
                hipFuncSetAttribute((const void *)k_recon<BPC, true>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds);
                attr = true;
            }
            k_recon<BPC, true><<<grid, 256, lds, stream>>>(a);
        } else {
            constexpr int lds = 4 * ClassSet<false>::wave_lds<BPC>();
            static bool attr = false;
            if (!attr) {
                hipFuncSetAttribute((const void *)k_recon<BPC, false>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds);
                attr = true;
            }
            k_recon<BPC, false><<<grid, 256, lds, stream>>>(a);
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            fprintf(stderr, "dav1d-gpu: recon launch failed: %s\n", hipGetErrorString(e));
            return -3;
        }
    }
    return 0;
}

}  // namespace dgpu

