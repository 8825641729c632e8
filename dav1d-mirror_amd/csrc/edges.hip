// edges.hip -- device intra edge preparation (include/dav1d_gpu.h,
// Dav1dGpuIntraEdgeBatch): bytefn(dav1d_prepare_intra_edges)
// (src/ipred_prepare_tmpl.c:76-204) for a batch of intra transform blocks.
//
// 16 lanes per record, 16 records per 256-thread workgroup.  Every lane
// derives the record's implementation mode (the remap of :83-104) and then
// fills its share of the edge array topleft[-2*4*th .. 2*4*tw], each entry
// computed directly from the picture with the reference's extension rules
// (no lane waits for another: the Z2 top-left filter of :197-200 recomputes
// topleft[-1] and topleft[1] itself).  Edges the remapped mode does not need
// are left untouched, as in the reference.  HBM-bound gather: per block the
// edge pixels read (strided for the left column) and written.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "dav1d_gpu.h"
#include "dsp_common.hpp"
#include "intra_edge_dev.hpp"
#include "lead_levels.hpp"

// the fused reconstruction launch (recon_ie.hpp, recon_ie8/16.hip)
int dgpu_recon_ie_8bpc(const Dav1dGpuFrameBatch *b, const Dav1dGpuIntraEdgeBatch *e, void *stream);
int dgpu_recon_ie_16bpc(const Dav1dGpuFrameBatch *b, const Dav1dGpuIntraEdgeBatch *e, void *stream);
int dgpu_recon_flow_8bpc(const Dav1dGpuFrameBatch *b, const Dav1dGpuIntraEdgeBatch *e, const Dav1dGpuIntraSchedule *s,
                         void *stream);
int dgpu_recon_flow_16bpc(const Dav1dGpuFrameBatch *b, const Dav1dGpuIntraEdgeBatch *e, const Dav1dGpuIntraSchedule *s,
                          void *stream);
int64_t dgpu_flow_workspace_bytes_8bpc(const Dav1dGpuIntraSchedule *s, int n_units);

namespace dgpu {

constexpr int kEdgeLanes = 16;

template <int BPC> struct EdgeArgs {
    using P = typename Px<BPC>::pixel;
    const P *pic[3];
    int ps[3];                 // pixels
    const P *top[3];
    int ts[3];                 // pixels
    int sb_log2[3];
    Dav1dGpuUnit *units;
    P *edges;
    const Dav1dGpuIntraEdge *recs;
    int n;
    int bdmax;
};

template <int BPC>
__global__ __launch_bounds__(256) void k_intra_edges(EdgeArgs<BPC> a) {
    using P = typename Px<BPC>::pixel;
    const int ri = blockIdx.x * (256 / kEdgeLanes) + threadIdx.x / kEdgeLanes;
    const int l = threadIdx.x % kEdgeLanes;
    if (ri >= a.n) return;
    const Dav1dGpuIntraEdge r = a.recs[ri];
    Dav1dGpuUnit *u = a.units + r.unit;
    if (u->pred != DGPU_PRED_INTRA && u->pred != DGPU_PRED_CFL) return;   // not an edge consumer
    const int pl = u->plane, txs = u->tx;
    const IeCtx<P> c = ie_setup<P>(r, a.pic[pl], a.ps[pl], a.top[pl], a.ts[pl], a.sb_log2[pl], tx_info(txs).w >> 2,
                                   tx_info(txs).h >> 2, a.bdmax);
    P *tl = a.edges + u->p.intra.edge_off;
    for (int i = -2 * c.szl + l; i <= 2 * c.szt; i += kEdgeLanes) {
        bool need;
        const int v = ie_value(c, i, need);
        if (need) tl[i] = (P)v;
    }
    if (l == 0) {
        u->p.intra.mode = (uint8_t)c.mode;   // CFL: its DC source (the same byte)
        if (u->pred != DGPU_PRED_CFL) u->p.intra.angle = ie_angle_field(r, c.angle);
    }
}

template <int BPC>
static int launch_edges(const Dav1dGpuIntraEdgeBatch *b, hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    constexpr int B = BPC / 8;
    if (!b || b->n_recs < 0 || (b->n_recs && (!b->recs || !b->units || !b->edges))) return -1;
    if (!b->n_recs) return 0;
    EdgeArgs<BPC> a;
    for (int p = 0; p < 3; p++) {
        a.pic[p] = (const P *)b->pic[p].data;
        a.ps[p] = (int)(b->pic[p].stride / B);
        a.top[p] = (const P *)b->top_edge[p].data;
        a.ts[p] = (int)(b->top_edge[p].stride / B);
        a.sb_log2[p] = b->sb_log2[p];
    }
    a.units = b->units;
    a.edges = (P *)b->edges;
    a.recs = b->recs;
    a.n = b->n_recs;
    a.bdmax = BPC == 8 ? 255 : b->bitdepth_max;
    constexpr int RPB = 256 / kEdgeLanes;
    k_intra_edges<BPC><<<dim3((b->n_recs + RPB - 1) / RPB), 256, 0, stream>>>(a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "dav1d-gpu: intra edge launch failed: %s\n", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

// bytefn(dav1d_backup_ipred_edge) for runs of columns: one 64-lane
// workgroup per run.
template <int BPC> struct BackupArgs {
    using P = typename Px<BPC>::pixel;
    const P *pic[3];
    int ps[3];
    P *top[3];
    int ts[3];
    int sb_log2[3];
    const Dav1dGpuEdgeBackup *runs;
};

template <int BPC>
__global__ __launch_bounds__(64) void k_backup_edge(BackupArgs<BPC> a) {
    const Dav1dGpuEdgeBackup r = a.runs[blockIdx.x];
    const int y = ((r.sby + 1) << a.sb_log2[r.plane]) - 1;
    const auto *src = a.pic[r.plane] + (size_t)y * a.ps[r.plane] + r.x0;
    auto *dst = a.top[r.plane] + (size_t)r.sby * a.ts[r.plane] + r.x0;
    for (int i = threadIdx.x; i < r.w; i += 64) dst[i] = src[i];
}

template <int BPC>
static int launch_backup(const Dav1dGpuIntraEdgeBatch *b, const Dav1dGpuEdgeBackup *runs, int n,
                         hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    constexpr int B = BPC / 8;
    if (!b || n < 0 || (n && !runs)) return -1;
    if (!n) return 0;
    BackupArgs<BPC> a;
    for (int p = 0; p < 3; p++) {
        a.pic[p] = (const P *)b->pic[p].data;
        a.ps[p] = (int)(b->pic[p].stride / B);
        a.top[p] = (P *)b->top_edge[p].data;
        a.ts[p] = (int)(b->top_edge[p].stride / B);
        a.sb_log2[p] = b->sb_log2[p];
    }
    a.runs = runs;
    k_backup_edge<BPC><<<dim3(n), 64, 0, stream>>>(a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "dav1d-gpu: edge backup launch failed: %s\n", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

// The level loop of the intra wavefront: edges -> recon -> backups per level.
template <int BPC>
static int launch_intra_frame(const Dav1dGpuFrameBatch *rb, const Dav1dGpuIntraEdgeBatch *eb,
                              const Dav1dGpuIntraSchedule *s, hipStream_t stream) {
    constexpr int NC = DGPU_N_RECT_TX_SIZES;
    if (!rb || !eb || !s || s->n_levels < 0) return -1;
    if (s->n_levels && (!s->unit_start || !s->class_start || !s->rec_start || !s->run_start)) return -1;
    for (int l = 0; l < s->n_levels; l++) {
        if (s->unit_start[l + 1] < s->unit_start[l] || s->rec_start[l + 1] < s->rec_start[l] ||
            s->run_start[l + 1] < s->run_start[l])
            return -2;
        const int32_t *cs = s->class_start + (size_t)l * (NC + 1);
        if (cs[0] != 0 || cs[NC] != s->unit_start[l + 1] - s->unit_start[l]) return -2;
    }
    if (s->n_levels && (s->unit_start[0] < 0 || s->unit_start[s->n_levels] > rb->n_units ||
                        s->rec_start[0] < 0 || s->rec_start[s->n_levels] > eb->n_recs || s->run_start[0] < 0))
        return -2;
    if (s->flags & DGPU_IS_PERSISTENT) {   // one launch: the level loop runs on the device
        if (s->n_levels && s->rec_start[0] != s->unit_start[0]) return -2;
        for (int l = 0; l <= s->n_levels; l++)
            if (s->rec_start[l] != s->unit_start[l]) return -2;
        // DGPU_IS_LEVEL0_BATCH: the leading levels (lead_levels.hpp) in fused
        // launches first, one per level; the persistent kernel takes the rest
        for (int l = 0, nl = lead_levels(s); l < nl; l++) {
            const int u0 = s->unit_start[l];
            Dav1dGpuFrameBatch lb = *rb;
            memset(lb.class_warp, 0, sizeof(lb.class_warp));
            lb.units = rb->units + u0;
            lb.n_units = s->unit_start[l + 1] - u0;
            if (rb->aux) lb.aux = rb->aux + u0;   // (per unit, like the units)
            memcpy(lb.class_start, s->class_start + (size_t)l * (NC + 1), sizeof(lb.class_start));
            Dav1dGpuIntraEdgeBatch le = *eb;
            le.units = eb->units + u0;
            le.recs = eb->recs + u0;
            le.n_recs = lb.n_units;
            const int rc = BPC == 8 ? dgpu_recon_ie_8bpc(&lb, &le, stream) : dgpu_recon_ie_16bpc(&lb, &le, stream);
            if (rc) return rc;
        }
        return BPC == 8 ? dgpu_recon_flow_8bpc(rb, eb, s, stream) : dgpu_recon_flow_16bpc(rb, eb, s, stream);
    }
    const bool fused = s->flags & DGPU_IS_FUSED;
    if (fused)
        for (int l = 0; l <= s->n_levels; l++)
            if (s->rec_start[l] != s->unit_start[l]) return -2;
    Dav1dGpuFrameBatch lb = *rb;
    memset(lb.class_warp, 0, sizeof(lb.class_warp));
    Dav1dGpuIntraEdgeBatch le = *eb;
    for (int l = 0; l < s->n_levels; l++) {
        if (fused) {   // edges, prediction, residual and backups in one launch per level
            lb.units = rb->units + s->unit_start[l];
            if (rb->aux) lb.aux = rb->aux + s->unit_start[l];   // (per unit, like the units)
            lb.n_units = s->unit_start[l + 1] - s->unit_start[l];
            memcpy(lb.class_start, s->class_start + (size_t)l * (NC + 1), sizeof(lb.class_start));
            le.units = eb->units + s->unit_start[l];
            le.recs = eb->recs + s->unit_start[l];
            le.n_recs = lb.n_units;
            const int rc = BPC == 8 ? dgpu_recon_ie_8bpc(&lb, &le, stream) : dgpu_recon_ie_16bpc(&lb, &le, stream);
            if (rc) return rc;
            continue;
        }
        le.recs = eb->recs + s->rec_start[l];
        le.n_recs = s->rec_start[l + 1] - s->rec_start[l];
        int rc = le.n_recs ? launch_edges<BPC>(&le, stream) : 0;
        if (rc) return rc;
        lb.units = rb->units + s->unit_start[l];
        lb.n_units = s->unit_start[l + 1] - s->unit_start[l];
        memcpy(lb.class_start, s->class_start + (size_t)l * (NC + 1), sizeof(lb.class_start));
        rc = BPC == 8 ? dav1d_gpu_recon_8bpc(&lb, stream) : dav1d_gpu_recon_16bpc(&lb, stream);
        if (rc) return rc;
        rc = launch_backup<BPC>(eb, s->runs + s->run_start[l], s->run_start[l + 1] - s->run_start[l], stream);
        if (rc) return rc;
    }
    return 0;
}

}  // namespace dgpu

extern "C" int dav1d_gpu_prepare_intra_edges_8bpc(const Dav1dGpuIntraEdgeBatch *b, void *stream) {
    return dgpu::launch_edges<8>(b, (hipStream_t)stream);
}
extern "C" int dav1d_gpu_prepare_intra_edges_16bpc(const Dav1dGpuIntraEdgeBatch *b, void *stream) {
    return dgpu::launch_edges<16>(b, (hipStream_t)stream);
}
extern "C" int dav1d_gpu_backup_ipred_edge_8bpc(const Dav1dGpuIntraEdgeBatch *b, const Dav1dGpuEdgeBackup *runs,
                                                int n_runs, void *stream) {
    return dgpu::launch_backup<8>(b, runs, n_runs, (hipStream_t)stream);
}
extern "C" int dav1d_gpu_backup_ipred_edge_16bpc(const Dav1dGpuIntraEdgeBatch *b, const Dav1dGpuEdgeBackup *runs,
                                                 int n_runs, void *stream) {
    return dgpu::launch_backup<16>(b, runs, n_runs, (hipStream_t)stream);
}
extern "C" int dav1d_gpu_recon_intra_frame_8bpc(const Dav1dGpuFrameBatch *recon, const Dav1dGpuIntraEdgeBatch *edges,
                                                const Dav1dGpuIntraSchedule *s, void *stream) {
    return dgpu::launch_intra_frame<8>(recon, edges, s, (hipStream_t)stream);
}
extern "C" int dav1d_gpu_recon_intra_frame_16bpc(const Dav1dGpuFrameBatch *recon, const Dav1dGpuIntraEdgeBatch *edges,
                                                 const Dav1dGpuIntraSchedule *s, void *stream) {
    return dgpu::launch_intra_frame<16>(recon, edges, s, (hipStream_t)stream);
}
extern "C" int64_t dav1d_gpu_intra_workspace_bytes(const Dav1dGpuIntraSchedule *s, int n_units) {
    if (!s || s->n_levels < 0 || (s->n_levels && (!s->unit_start || !s->class_start))) return -2;
    return dgpu_flow_workspace_bytes_8bpc(s, n_units);
}
