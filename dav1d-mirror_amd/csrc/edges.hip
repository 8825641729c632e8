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

// needs per implementation mode: bit0 left, 1 top, 2 top-left, 3 top-right,
// 4 bottom-left (av1_intra_prediction_edges, src/ipred_prepare_tmpl.c:50-75)
__device__ __forceinline__ int ie_needs(int m) {
    constexpr uint64_t t = (3ull << 0) | (2ull << 5) | (1ull << 10) | (1ull << 15) | (2ull << 20) | (0ull << 25) |
                           (14ull << 30) | (7ull << 35) | (21ull << 40) | (3ull << 45) | (3ull << 50) |
                           (3ull << 55) | (7ull << 60);
    return m == DGPU_FILTER_PRED ? 7 : (int)((t >> (5 * m)) & 31);
}

template <int BPC>
__global__ __launch_bounds__(256) void k_intra_edges(EdgeArgs<BPC> a) {
    using P = typename Px<BPC>::pixel;
    const int ri = blockIdx.x * (256 / kEdgeLanes) + threadIdx.x / kEdgeLanes;
    const int l = threadIdx.x % kEdgeLanes;
    if (ri >= a.n) return;
    const Dav1dGpuIntraEdge r = a.recs[ri];
    Dav1dGpuUnit *u = a.units + r.unit;
    const int pl = u->plane, txs = u->tx;
    const int tw = tx_info(txs).w >> 2, th = tx_info(txs).h >> 2;
    const int ps = a.ps[pl];
    const P *dst = a.pic[pl] + (size_t)(r.y4 * 4) * ps + r.x4 * 4;
    const int hl = r.flags & DGPU_IE_HAVE_LEFT, ht = r.flags & DGPU_IE_HAVE_TOP;
    // mode remap (:83-104)
    int angle = r.angle, mode = r.mode;
    if (mode >= 1 && mode <= 8) {
        // base angles of modes 1..8: 90 180 45 135 113 157 203 67
        angle = (int)((0x43cb9d71872db45aull >> (8 * (mode - 1))) & 0xff) + 3 * angle;
        mode = angle <= 90 ? (angle < 90 && ht ? DGPU_Z1_PRED : DGPU_VERT_PRED)
             : angle < 180 ? DGPU_Z2_PRED
                           : (angle > 180 && hl ? DGPU_Z3_PRED : DGPU_HOR_PRED);
    } else if (mode == 0) {
        mode = hl ? (ht ? DGPU_DC_PRED : DGPU_LEFT_DC_PRED) : (ht ? DGPU_TOP_DC_PRED : DGPU_DC_128_PRED);
    } else if (mode == 12) {
        mode = hl ? (ht ? DGPU_PAETH_PRED : DGPU_HOR_PRED) : (ht ? DGPU_VERT_PRED : DGPU_DC_128_PRED);
    }
    const int nd = ie_needs(mode);
    const int half = (a.bdmax + 1) >> 1;
    const P *top = dst - ps;
    if (r.flags & DGPU_IE_TOP_SB_EDGE)
        top = a.top[pl] + (size_t)(((r.y4 * 4) >> a.sb_log2[pl]) - 1) * a.ts[pl] + r.x4 * 4;
    const int szl = th * 4, szt = tw * 4;
    const int nl = min(szl, (r.h4 - r.y4) * 4), nt = min(szt, (r.w4 - r.x4) * 4);
    const bool hbl = hl && r.y4 + th < r.h4 && (r.flags & DGPU_IE_LEFT_HAS_BOTTOM);
    const bool htr = ht && r.x4 + tw < r.w4 && (r.flags & DGPU_IE_TOP_HAS_RIGHT);
    const int nbl = hbl ? min(szl, (r.h4 - r.y4 - th) * 4) : 1;
    const int ntr = htr ? min(szt, (r.w4 - r.x4 - tw) * 4) : 1;
    auto leftv = [&](int k) -> int {
        return hl ? (int)dst[(size_t)min(k, nl - 1) * ps - 1] : ht ? (int)top[0] : half + 1;
    };
    auto topv = [&](int k) -> int {
        return ht ? (int)top[min(k, nt - 1)] : hl ? (int)dst[-1] : half - 1;
    };
    P *tl = a.edges + u->p.intra.edge_off;
    for (int i = -2 * szl + l; i <= 2 * szt; i += kEdgeLanes) {
        int v;
        if (i < -szl) {           // bottom-left (:135-154)
            if (!(nd & 16)) continue;
            const int k = -i - szl - 1;
            v = hbl ? (int)dst[(size_t)(szl + min(k, nbl - 1)) * ps - 1] : leftv(szl - 1);
        } else if (i < 0) {       // left (:124-133)
            if (!(nd & 1)) continue;
            v = leftv(-i - 1);
        } else if (i == 0) {      // top-left (:187-201)
            if (!(nd & 4)) continue;
            v = hl ? (ht ? (int)top[-1] : (int)dst[-1]) : (ht ? (int)top[0] : half);
            if (mode == DGPU_Z2_PRED && tw + th >= 6 && (r.flags & DGPU_IE_FILTER_EDGE))
                v = ((leftv(0) + topv(0)) * 5 + v * 6 + 8) >> 4;
        } else if (i <= szt) {    // top (:156-166)
            if (!(nd & 2)) continue;
            v = topv(i - 1);
        } else {                  // top-right (:168-185)
            if (!(nd & 8)) continue;
            const int k = i - szt - 1;
            v = htr ? (int)top[szt + min(k, ntr - 1)] : topv(szt - 1);
        }
        tl[i] = (P)v;
    }
    if (l == 0) {
        u->p.intra.mode = (uint8_t)mode;   // CFL: its DC source (the same byte)
        if (u->pred != DGPU_PRED_CFL)
            u->p.intra.angle = (uint16_t)((angle & 511) | ((r.flags & DGPU_IE_SMOOTH) ? 512 : 0) |
                                      ((r.flags & DGPU_IE_FILTER_EDGE) ? 1024 : 0));
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
    Dav1dGpuFrameBatch lb = *rb;
    memset(lb.class_warp, 0, sizeof(lb.class_warp));
    Dav1dGpuIntraEdgeBatch le = *eb;
    for (int l = 0; l < s->n_levels; l++) {
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
