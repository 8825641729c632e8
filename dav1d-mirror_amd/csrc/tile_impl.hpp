// tile_impl.hpp -- launch of the superblock-tile batch kernel (instantiated
// per bitdepth in tile8.hip / tile16.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tile_kernel.hpp"

namespace dgpu {

template <int BPC>
static int launch_tiles(const Dav1dGpuTileBatch *b, hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    constexpr int B = BPC / 8;
    if (!b || b->n_tiles < 0 || b->n_tiles_huge < 0 || b->n_tiles_huge > b->n_tiles ||
        (b->n_tiles && (!b->tiles || !b->preds))) return -1;
    for (int p = 0; p < 3; p++) {
        // output rows are stored 16 / 8 bytes at a time at tile positions
        if (((uintptr_t)b->dst[p].data & 15) || (b->dst[p].stride & 15)) return -4;
        for (int r = 0; r < DGPU_MAX_REFS; r++)   // footprint rows: aligned dword loads
            if (b->ref[r][p].data && (((uintptr_t)b->ref[r][p].data & 3) || (b->ref[r][p].stride & 3))) return -4;
    }
    if (b->n_tiles == 0) return 0;
    TileArgs<BPC> a;
    memset(&a, 0, sizeof(a));
#if DGPU_BOUNDS
    {   // diagnostics: the planes and the buffers the caller registered
        // (dav1d_gpu_debug_register_buffer, exact sizes); strict when any
        DgpuBndTab t{};
        for (int p = 0; p < 3; p++) {
            bnd_add(t, b->dst[p], BND_DST);
            for (int r = 0; r < DGPU_MAX_REFS; r++) bnd_add(t, b->ref[r][p], BND_REF);
        }
        bnd_add(t, b->cfl_luma, BND_CFL);
        bnd_add_extra(t);
        bnd_print<P>(t, "tiles");
        if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_dgpu_bnd), &t, sizeof(t), 0, hipMemcpyHostToDevice, stream) != hipSuccess ||
            hipStreamSynchronize(stream) != hipSuccess)
            return -3;
        a.bnd_noclamp = getenv("DAV1D_GPU_BND_NOCLAMP") != nullptr;
    }
#endif
    for (int p = 0; p < 3; p++) {
        a.dst[p] = (P *)b->dst[p].data;
        a.dst_stride[p] = (int)(b->dst[p].stride / B);
        for (int r = 0; r < DGPU_MAX_REFS; r++) {
            a.ref[r * 3 + p] = (const P *)b->ref[r][p].data;
            a.ref_stride[r * 3 + p] = (int)(b->ref[r][p].stride / B);
            a.ref_w[r * 3 + p] = b->ref[r][p].w;
            a.ref_h[r * 3 + p] = b->ref[r][p].h;
        }
    }
    a.tiles = b->tiles;
    a.preds = b->preds;
    a.txs = b->txs;
    a.coef = (C *)b->coef;
    a.edges = (const P *)b->edges;
    a.aux_pool = (const uint8_t *)b->aux_pool;
    a.cfl_luma = (const P *)b->cfl_luma.data;
    a.cfl_luma_stride = (int)(b->cfl_luma.stride / B);
    a.cfl_ss = b->cfl_ss;
    a.bdmax = BPC == 8 ? 255 : b->bitdepth_max;
    a.zero_coefs = b->zero_coefs;
    static unsigned long long *trace_buf = nullptr;   // DGPU_TILE_TRACE builds only
    if (DGPU_TILE_TRACE) {
        const size_t n = (size_t)b->n_tiles * 32;
        static size_t cap = 0;
        if (n > cap) {
            if (trace_buf) (void)hipFree(trace_buf);
            if (hipMalloc(&trace_buf, n * 8) != hipSuccess) return -3;
            cap = n;
        }
        a.trace = trace_buf;
    }
    // the 64-point tiles (if any) first: their longer workgroups start early
    const int nh = b->n_tiles_huge, nn = b->n_tiles - nh;
    if (nh) {
        a.tile0 = nn;
        a.n_tiles = nh;
        k_tiles<BPC, true><<<dim3((nh + 7) & ~7), kTileThreads, 0, stream>>>(a);
    }
    if (nn) {
        a.tile0 = 0;
        a.n_tiles = nn;   // grid: a multiple of 8 (XCD-contiguous block order)
        k_tiles<BPC, false><<<dim3((nn + 7) & ~7), kTileThreads, 0, stream>>>(a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "dav1d-gpu: tile launch failed: %s\n", hipGetErrorString(e));
        return -3;
    }
    if (DGPU_TILE_TRACE) {   // debug: synchronous dump of the phase timestamps
        const char *f = getenv("DAV1D_GPU_TRACE_FILE");
        if (f && hipStreamSynchronize(stream) == hipSuccess) {
            const size_t n = (size_t)b->n_tiles * 32;
            unsigned long long *h = (unsigned long long *)malloc(n * 8);
            FILE *fp = fopen(f, "wb");
            if (h && fp && hipMemcpy(h, trace_buf, n * 8, hipMemcpyDeviceToHost) == hipSuccess) fwrite(h, 8, n, fp);
            if (fp) fclose(fp);
            free(h);
        }
    }
    return 0;
}

}  // namespace dgpu
