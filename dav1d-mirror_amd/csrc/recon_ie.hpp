// recon_ie.hpp -- the intra wavefront's reconstruction launch: the unit
// batch's SMALL / HUGE groups compiled with GATHER (recon_kernel.hpp), so
// one launch per dependency level does edge preparation
// (dav1d_prepare_intra_edges), prediction, residual and the top_edge backup
// of superblock-bottom rows.  Instantiated in recon_ie8.hip / recon_ie16.hip.
#pragma once
#include "recon_impl.hpp"
#include "flow_impl.hpp"

namespace dgpu {

template <int BPC>
static int launch_ie(const Dav1dGpuFrameBatch *b, const Dav1dGpuIntraEdgeBatch *e, hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    constexpr int B = BPC / 8;
    if (!b || !e || !b->units || b->n_units < 0 || (b->n_units && !e->recs)) return -1;
    for (int c = 0; c < DGPU_N_RECT_TX_SIZES; c++)
        if (b->class_start[c + 1] < b->class_start[c] || b->class_warp[c]) return -2;
    if (b->class_start[0] != 0 || b->class_start[DGPU_N_RECT_TX_SIZES] != b->n_units) return -2;
    for (int p = 0; p < 3; p++) {
        if (((uintptr_t)b->dst[p].data & 15) || (b->dst[p].stride & 15)) return -4;
        // row offsets are 24-bit multiplies in the kernels (__mul24): strides in [0, 2^23) bytes
        if (!stride24(b->dst[p].stride)) return -4;
        for (int r = 0; r < DGPU_MAX_REFS; r++)
            if (b->ref[r][p].data && !stride24(b->ref[r][p].stride)) return -4;
    }
    if (b->n_units == 0) return 0;
    ReconArgs<BPC> a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) {
        a.dst[p] = (P *)b->dst[p].data;
        a.dst_stride[p] = (int)(b->dst[p].stride / B);
        for (int r = 0; r < DGPU_MAX_REFS; r++) {   // inter units of a mixed frame
            a.ref[r][p] = (const P *)b->ref[r][p].data;
            a.ref_stride[r][p] = (int)(b->ref[r][p].stride / B);
        }
        a.top[p] = (P *)e->top_edge[p].data;
        a.top_stride[p] = (int)(e->top_edge[p].stride / B);
        a.top_rows[p] = e->top_edge[p].h;
        a.sb_log2[p] = e->sb_log2[p];
    }
    a.units = b->units;
    a.units_rw = e->units;
    a.recs = e->recs;
    a.coef = (C *)b->coef;
    a.edges = (const P *)b->edges;
    a.cfl_luma = (const P *)b->cfl_luma.data;
    if (b->cfl_luma.data && !stride24(b->cfl_luma.stride)) return -4;
    a.cfl_luma_stride = (int)(b->cfl_luma.stride / B);
    a.cfl_ss = b->cfl_ss;
    a.aux = b->aux;   // INTER_MASK masks / PAL records (recorder flushes)
    a.aux_pool = (const uint8_t *)b->aux_pool;
    a.bdmax = BPC == 8 ? 255 : b->bitdepth_max;
    a.zero_coefs = b->zero_coefs;
    int rc = launch_group<BPC, GROUP_HUGE_IE>(a, b, ~0u, stream);
    if (!rc) rc = launch_group<BPC, GROUP_SMALL_IE>(a, b, ~0u, stream);
    return rc;
}

}  // namespace dgpu
