// recorder.hip -- the batch recorder at the reconstruction seam (SURVEY 8(f)
// row 2; include/dav1d_gpu.h, Dav1dGpuRecorder).
//
// A decoder's recon_b_inter / recon_b_intra (src/recon_tmpl.c:1598, :1195)
// hand over, per block and plane, what they would have passed to the DSP
// (one Dav1dGpuRecBlock) and, per coded transform block, what they would
// have passed to inv_txfm_add (dav1d_gpu_rec_residual).  The recording goes
// straight into page-locked staging; a flush uploads it as recorded and
// builds the device's work on the device, on the recorder's own stream:
//   1. the cut (rec_cut.hpp): every transform cell of every block
//      (recon_b_* iterate the block's transform grid, :1258-1262), carrying
//      the block's prediction and the cell's residual if one was recorded,
//      the dav1d_prepare_intra_edges record of each intra / CfL cell, the
//      clamped footprint copies (emu_edge) and the launch-ahead units -- a
//      count pass per block, an exclusive scan, a write pass per block;
//   2. dependency levels at 4x4 granularity: every cell stamps its 4x4s in a
//      writer map, looks up the writers of the pixels its edges (CfL: the
//      co-located luma; an inter-intra residual: its block's prediction)
//      read, and takes one level above the highest of them (a dataflow
//      kernel in decode order, which is a topological order);
//   3. one radix sort of (level, size class, kind, mode, type, decode
//      index), the cells and their producer lists scattered to their ranks;
//   4. the launch-ahead units in class order, and their superblock-bottom
//      backup runs.
// The host reads back three small results (the totals after the count, the
// level count and class ranges at the end) and launches the persistent
// wavefront (dav1d_gpu_recon_intra_frame_*) on the caller's stream, behind
// the prep.  With DAV1D_GPU_REC_HOSTONLY (diagnostics, no device) the same
// step functions run serially on the host.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "bounds.hpp"
#include "dav1d_gpu.h"
#include "rec_cut.hpp"

#ifndef DGPU_BOUNDS
#define DGPU_BOUNDS 0
#endif

using namespace rec;

namespace {

static bool host_only() {   // DAV1D_GPU_REC_HOSTONLY=1 (diagnostics, no device needed)
    static const bool v = getenv("DAV1D_GPU_REC_HOSTONLY") != nullptr;
    return v;
}

// device buffers (host memory for host-only flushes), grown as needed
struct Mem {
    void *p = nullptr;
    size_t cap = 0;
    template <typename T> T *as() const { return (T *)p; }
    int grow(size_t n) {
        if (n <= cap && p) return 0;
        release();
        // rounded up to 256 bytes: the one read past a buffer's last element
        // the kernels make by design is Stage's (the 16-byte block holding a
        // region's last byte, at most 15 bytes further)
        const size_t sz = (std::max<size_t>(n, 16) + 255) & ~(size_t)255;
        if (host_only()) {
            p = malloc(sz);
            if (!p) return -1;
        } else if (hipMalloc(&p, sz) != hipSuccess) {
            p = nullptr;
            return -1;
        }
        cap = sz;
        return 0;
    }
    void release() {
        if (p) {
            if (host_only()) free(p);
            else (void)hipFree(p);
        }
        p = nullptr;
        cap = 0;
    }
};

// The recording: page-locked (portable, CPU-cached unless
// DAV1D_GPU_REC_PIN=default) so the flush's uploads are asynchronous copies
// of it, or ordinary memory for host-only flushes.  Nothing in the library
// registers ordinary host memory.
struct Stage {
    uint8_t *p = nullptr;
    size_t n = 0, cap = 0;
    size_t up = 0;   // bytes already copied to the device mirror (streamed while recording)
    bool pinned = false;
    void *append(size_t m) {
        if (n + m > cap && reserve(n + m)) return nullptr;
        void *q = p + n;
        n += m;
        return q;
    }
    int reserve(size_t m) {
        const size_t nc = std::max(m, std::max<size_t>(2 * cap, 1 << 16));
        void *q = nullptr;
        bool pin = !host_only();
        if (pin) {
            static const bool coherent = [] {
                const char *e = getenv("DAV1D_GPU_REC_PIN");
                return e && !strcmp(e, "default");
            }();
            // (no device in this process yet, or none at all: ordinary
            // memory, uploaded through the runtime's staging)
            if (hipHostMalloc(&q, nc, hipHostMallocPortable | (coherent ? 0 : hipHostMallocNonCoherent)) != hipSuccess) {
                q = nullptr;
                pin = false;
            }
        }
        if (!q && !(q = malloc(nc))) return -1;
        if (n) memcpy(q, p, n);
        release_mem();
        p = (uint8_t *)q;
        cap = nc;
        pinned = pin;
        return 0;
    }
    void release_mem() {
        if (p) {
            if (pinned) (void)hipHostFree(p);
            else free(p);
        }
        p = nullptr;
        cap = 0;
    }
    void release() {
        release_mem();
        n = 0;
    }
};

// one 64-lane workgroup per footprint: lanes along the row, clamped reads
struct EmuArgs {
    const void *ref[DGPU_MAX_REFS - 1][3];
    int32_t stride[DGPU_MAX_REFS - 1][3];   // pixels
    int32_t w[DGPU_MAX_REFS - 1][3], h[DGPU_MAX_REFS - 1][3];
    void *out;
    const EmuJob *jobs;
    int32_t n, rows;   // rows: the scratch plane's (diagnostics)
};
template <typename P>
__global__ __launch_bounds__(64) void k_emu_footprints(EmuArgs a) {
    const int j = blockIdx.x;
    if (j >= a.n) return;
    const EmuJob jb = a.jobs[j];
    const P *ref = static_cast<const P *>(a.ref[jb.slot][jb.plane]);
    const int rs = a.stride[jb.slot][jb.plane], rw = a.w[jb.slot][jb.plane], rh = a.h[jb.slot][jb.plane];
    P *out = static_cast<P *>(a.out) + jb.o0;
#if DGPU_BOUNDS   // diagnostics: the job's scratch rows and the clamped reads stay inside their buffers
    if (threadIdx.x == 0 && (jb.o0 < 0 || jb.o0 + (jb.h - 1) * kEmuStride + jb.w > a.rows * kEmuStride ||
                             (jb.o0 % kEmuStride) + jb.w > kEmuStride || rw <= 0 || rh <= 0 || !ref))
        printf("DGPU_BOUNDS emu job %d: at %d, %dx%d of %d rows, ref %dx%d\n", j, jb.o0, jb.w, jb.h, a.rows, rw, rh);
#endif
    for (int c = threadIdx.x; c < jb.w; c += 64) {
        const int x = min(max(jb.x0 + c, 0), rw - 1);
        for (int i = 0; i < jb.h; i++) {
            const int y = min(max(jb.y0 + i, 0), rh - 1);
            out[(size_t)i * kEmuStride + c] = ref[(size_t)y * rs + x];
        }
    }
}

template <typename F>
__global__ __launch_bounds__(256) void k_each(int n, F f) {
    const int i = (int)(blockIdx.x * 256 + threadIdx.x);
    if (i < n) f(i);
}

// the sort key of a cell: level | tx (5) | pred (4) | mode (6) | type (5,
// NO_RESIDUAL last), then the decode index in the low 21 bits (the sort is
// then a stable one by the key)
__host__ __device__ inline uint64_t level_key(const Dav1dGpuUnit &u, int sortmode, int level, int ci) {
    const uint64_t key = (uint64_t)level << 20 | (uint64_t)u.tx << 15 | (uint64_t)u.pred << 11 |
                         (uint64_t)(sortmode & 63) << 5 | (uint64_t)(u.txtp == DGPU_NO_RESIDUAL ? 31 : u.txtp);
    return key << 21 | (uint64_t)ci;
}

struct LevelArgs {
    const int32_t *pstart, *prod, *csort;
    const Dav1dGpuUnit *cu;
    int32_t *lv;
    uint64_t *keys;
    Hdr *hdr;
    int n, spin_limit;
};
constexpr int kLevelSpinLimit = 1 << 22;
// The levels in decode order: one wave per 64 consecutive cells, taken by
// ticket, so every cell a wave waits for is held by a wave that already
// runs (producers come earlier in decode order).  A cell's level is one above
// its producers' highest; producers inside the wave are read from LDS, the
// others from the level array at agent scope (the level is the datum, no
// fence needed).  The loop is wave-uniform: a lane whose producers are not
// all known yet tries again on the next pass.
__global__ __launch_bounds__(64) void k_levels(LevelArgs a) {
    __shared__ int32_t slv[64];
    const int lane = threadIdx.x;
    int t = 0;
    if (lane == 0) t = __hip_atomic_fetch_add(&a.hdr->ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __shfl(t, 0);
    const int c0 = t * 64, ci = c0 + lane;
    const bool live = ci < a.n;
    slv[lane] = -1;
    __syncthreads();
    int k = live ? a.pstart[ci] : 0;
    const int k1 = live ? a.pstart[ci + 1] : 0;
    int d = -1, level = 0;
    bool done = !live;
    for (int it = 0;; it++) {
        if (!done) {
            for (; k < k1; k++) {
                const int q = a.prod[k];
                const int v = q >= c0 ? slv[q - c0]
                                      : __hip_atomic_load(&a.lv[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v < 0) break;
                d = max(d, v);
            }
            if (k >= k1) {
                level = d + 1;
                done = true;
                slv[lane] = level;
                __hip_atomic_store(&a.lv[ci], level, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (__all(done)) break;
        if (it >= a.spin_limit) {   // never expected: the flush fails instead of hanging
            if (lane == 0) aor(&a.hdr->err, E_STALL);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    int m = 0;
    if (live) {
        const Dav1dGpuUnit u = a.cu[ci];
        a.keys[ci] = level_key(u, a.csort[ci], level, ci);
        m = level;
    }
    for (int o = 32; o; o >>= 1) m = max(m, __shfl_xor(m, o));
    if (lane == 0) amax(&a.hdr->max_level, m);
}

// The flush's steps on the device (the recorder's stream) or serially on the
// host (host-only flushes)
struct Exec {
    bool host;
    hipStream_t st;
    Mem *tmp;   // hipcub temporary storage
    int err = 0;
    template <typename F> void each(long long n, F f) {
        if (n <= 0 || err) return;
        if (host) {
            for (long long i = 0; i < n; i++) f((int)i);
            return;
        }
        k_each<<<dim3((unsigned)((n + 255) / 256)), 256, 0, st>>>((int)n, f);
        if (hipGetLastError() != hipSuccess) err = -3;
    }
    void memset(void *p, int v, size_t n) {
        if (!n || err) return;
        if (host) ::memset(p, v, n);
        else if (hipMemsetAsync(p, v, n, st) != hipSuccess) err = -3;
    }
    void upload(void *d, const void *h, size_t n) {
        if (!n || err) return;
        if (host) memcpy(d, h, n);
        else if (hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st) != hipSuccess) err = -3;
    }
    void fetch(void *h, const void *d, size_t n) {   // queued; complete after sync()
        if (!n || err) return;
        if (host) {
            if (h != d) memcpy(h, d, n);   // (host-only: the "device" buffer is often read in place)
        } else if (hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, st) != hipSuccess) {
            err = -3;
        }
    }
    void sync() {
        if (!host && !err && hipStreamSynchronize(st) != hipSuccess) err = -3;
    }
    // exclusive sum of n1 int32 (in[n1 - 1] = 0 gives the total in out[n1 - 1])
    void scan(const int32_t *in, int32_t *out, int n1) {
        if (n1 <= 0 || err) return;
        if (host) {
            int32_t acc = 0;
            for (int i = 0; i < n1; i++) {
                const int32_t v = in[i];
                out[i] = acc;
                acc += v;
            }
            return;
        }
        size_t b = 0;
        if (hipcub::DeviceScan::ExclusiveSum(nullptr, b, in, out, n1, st) != hipSuccess || tmp->grow(b) ||
            hipcub::DeviceScan::ExclusiveSum(tmp->p, b, in, out, n1, st) != hipSuccess)
            err = -3;
    }
    void scan_blocks(const BlockCnt *in, BlockCnt *out, int n) {
        if (n <= 0 || err) return;
        if (host) {
            BlockCnt acc{};
            for (int i = 0; i < n; i++) {
                const BlockCnt v = in[i];
                out[i] = acc;
                acc = BlockCntSum()(acc, v);
            }
            return;
        }
        size_t b = 0;
        const BlockCnt z{};
        if (hipcub::DeviceScan::ExclusiveScan(nullptr, b, in, out, BlockCntSum(), z, n, st) != hipSuccess ||
            tmp->grow(b) || hipcub::DeviceScan::ExclusiveScan(tmp->p, b, in, out, BlockCntSum(), z, n, st) != hipSuccess)
            err = -3;
    }
    void sort(const uint64_t *in, uint64_t *out, int n, int lo, int hi) {   // keys are distinct
        if (n <= 0 || err) return;
        if (host) {
            memcpy(out, in, (size_t)n * 8);
            std::sort(out, out + n);
            return;
        }
        size_t b = 0;
        if (hipcub::DeviceRadixSort::SortKeys(nullptr, b, in, out, n, lo, hi, st) != hipSuccess || tmp->grow(b) ||
            hipcub::DeviceRadixSort::SortKeys(tmp->p, b, in, out, n, lo, hi, st) != hipSuccess)
            err = -3;
    }
};

}  // namespace

struct Dav1dGpuRecorder {
    int bpc, bdmax, width, height, device;
    // the recording
    Stage blocks, baux_off, baux, res, coefb;
    int32_t last_wmask = -1;   // the last INTER_WMASK block (COMPOUND_SEG chroma masks read it)
    int64_t cell_bound = 0;    // an upper bound of the recording's cells
    // per-4x4 maps kept across flushes (generation-stamped): the residual
    // recorded at each cell (index + res_base) and its writer (cell_base + cell)
    Mem res_at, own;
    size_t map_off[3] = {0, 0, 0};
    int32_t map_w4[3] = {0, 0, 0}, map_h4[3] = {0, 0, 0};
    int32_t res_base = 0, cell_base = 0;
    // the flush's buffers
    Mem d_blocks, d_baux_off, d_baux, d_res, d_coef;
    Mem d_hdr, d_cnt, d_base, d_auxend;
    Mem d_cu, d_crec, d_caux, d_csort, d_jobs, d_rawc, d_raws, d_raw, d_pcnt, d_pstart, d_prod, d_lv;
    Mem d_keys, d_keys2, d_rank, d_ends, d_lend, d_dcnt, d_dstart, d_deps;
    Mem d_units, d_recs, d_aux, d_auxp, d_emu_jobs, d_xu0, d_xa0, d_xk, d_xk2, d_xunits, d_xaux, d_xends;
    Mem d_bkf, d_bks, d_bk, d_edges, d_work, d_emu, d_tmp;
    std::vector<int32_t> unit_start, class_start, rec_start, run_start;
    hipStream_t pst = nullptr;    // the recorder's stream (the prep)
    hipStream_t cst = nullptr;    // the coefficient pool's upload, beside the prep
    hipEvent_t coef_ev = nullptr;
    hipEvent_t prep = nullptr;    // the prep done, for the caller's stream
    hipEvent_t pt0 = nullptr, pt1 = nullptr;   // the prep's span (timing events)
    float prep_ms = 0;
    void *rb = nullptr;           // page-locked readback
    size_t rb_cap = 0;
    void *flag = nullptr;         // the last flush's wavefront error word, copied back on its stream
    // dav1d_gpu_recorder_set_top_edge: the caller's f->ipred_edge planes
    // (superblock-top rows read from and backed up to them), luma superblock log2
    Dav1dGpuPlane top[3] = {};
    bool top_on = false;
    int sb_log2 = 6;
    hipEvent_t done = nullptr;
    bool pending_check = false;   // the last flush's error word not read yet
    int32_t last_units = 0, last_levels = 0;
    bool streaming = false;   // the recording goes up while it is made (after a first flush)
    void drop_recording() {
        blocks.n = baux_off.n = baux.n = res.n = coefb.n = 0;
        blocks.up = baux_off.up = baux.up = res.up = 0;
        last_wmask = -1;
        cell_bound = 0;
    }
    size_t nblocks() const { return blocks.n / sizeof(Dav1dGpuRecBlock); }
    size_t nres() const { return res.n / sizeof(RecRes); }
};

extern "C" Dav1dGpuRecorder *dav1d_gpu_recorder_new(int bpc, int bitdepth_max, int width, int height, int device) {
    if ((bpc != 8 && bpc != 16) || width <= 0 || height <= 0) return nullptr;
    Dav1dGpuRecorder *r = new Dav1dGpuRecorder();
    r->bpc = bpc;
    r->bdmax = bpc == 8 ? 255 : bitdepth_max;
    r->width = width;
    r->height = height;
    r->device = device;
    return r;
}

extern "C" void dav1d_gpu_recorder_free(Dav1dGpuRecorder *r) {
    if (!r) return;
    if (host_only() || hipSetDevice(r->device) == hipSuccess) {
        if (r->done) {
            (void)hipEventSynchronize(r->done);
            (void)hipEventDestroy(r->done);
        }
        for (hipStream_t q : {r->pst, r->cst})
            if (q) {
                (void)hipStreamSynchronize(q);
                (void)hipStreamDestroy(q);
            }
        for (hipEvent_t e : {r->prep, r->pt0, r->pt1, r->coef_ev})
            if (e) (void)hipEventDestroy(e);
        if (r->rb) (void)hipHostFree(r->rb);
        if (r->flag) (void)hipHostFree(r->flag);
        for (Stage *s : {&r->blocks, &r->baux_off, &r->baux, &r->res, &r->coefb}) s->release();
        for (Mem *m : {&r->res_at, &r->own, &r->d_blocks, &r->d_baux_off, &r->d_baux, &r->d_res, &r->d_coef, &r->d_hdr,
                       &r->d_cnt, &r->d_base, &r->d_auxend, &r->d_cu, &r->d_crec, &r->d_caux, &r->d_csort, &r->d_jobs,
                       &r->d_rawc, &r->d_raws, &r->d_raw, &r->d_pcnt, &r->d_pstart, &r->d_prod, &r->d_lv, &r->d_keys,
                       &r->d_keys2, &r->d_rank, &r->d_ends, &r->d_lend, &r->d_dcnt, &r->d_dstart, &r->d_deps,
                       &r->d_units, &r->d_recs, &r->d_aux, &r->d_auxp, &r->d_emu_jobs, &r->d_xu0, &r->d_xa0, &r->d_xk,
                       &r->d_xk2, &r->d_xunits, &r->d_xaux, &r->d_xends, &r->d_bkf, &r->d_bks, &r->d_bk, &r->d_edges,
                       &r->d_work, &r->d_emu, &r->d_tmp})
            m->release();
    }
    delete r;
}

// the plane's part of the decoder's block grid: 4 * f->bw x 4 * f->bh, the
// picture size rounded up to 8 (src/decode.c), >> 1 for 4:2:0 chroma.
// Blocks start inside it and may run past it into the picture's padding;
// transform blocks start inside it (recon_tmpl.c:1208 w4 / h4 clip)
static bool plane_dims(const Dav1dGpuRecorder *r, int plane, int &w, int &h) {
    if (plane < 0 || plane > 2) return false;
    const int gw = (r->width + 7) & ~7, gh = (r->height + 7) & ~7;
    w = plane ? gw >> 1 : gw;
    h = plane ? gh >> 1 : gh;
    return true;
}

// The decoder's superblock-top edge rows (f->ipred_edge, backed up by
// dav1d_backup_ipred_edge, src/recon_tmpl.c:2162-2186, and read by
// prepare_intra_edges as prefilter_toplevel_sb_edge, :1275-1279, :1394-1398,
// :1664-1668, src/ipred_prepare_tmpl.c:117-126).  Rows must cover the plane's
// grid rounded up to whole superblocks (transform blocks past the grid write
// their bottom rows there too, as in dav1d's sb128w * 128 rows) and one row
// per superblock row but the last.
extern "C" int dav1d_gpu_recorder_set_top_edge(Dav1dGpuRecorder *r, const Dav1dGpuPlane top_edge[3], int sb128) {
    if (!r) return -1;
    if (!top_edge) {
        r->top_on = false;
        return 0;
    }
    const int bpp = r->bpc / 8, l2 = sb128 ? 7 : 6;
    for (int p = 0; p < 3; p++) {
        int pw, ph;
        plane_dims(r, p, pw, ph);
        const int sl = p ? l2 - 1 : l2, sb = 1 << sl;
        const int64_t need_w = ((int64_t)pw + sb - 1) / sb * sb, need_h = ((int64_t)ph + sb - 1) / sb - 1;
        const Dav1dGpuPlane &t = top_edge[p];
        if (!t.data || t.w < need_w || t.h < need_h || t.stride < (int64_t)t.w * bpp) return -1;
    }
    for (int p = 0; p < 3; p++) r->top[p] = top_edge[p];
    r->sb_log2 = l2;
    r->top_on = true;
    return 0;
}

static int check_block(const Dav1dGpuRecorder *r, const Dav1dGpuRecBlock *b, bool ext) {
    int pw, ph;
    if (!r || !b || !plane_dims(r, b->plane, pw, ph)) return -1;
    if (b->tx < 0 || b->tx >= DGPU_N_RECT_TX_SIZES) return -1;
    const int tw = tx_w(b->tx), th = tx_h(b->tx);
    if (b->x < 0 || b->y < 0 || b->w <= 0 || b->h <= 0 || b->x >= pw || b->y >= ph || b->w > 128 || b->h > 128)
        return -1;
    if ((b->x & 3) || (b->y & 3) || b->w % tw || b->h % th) return -1;
    if (ext != is_ext_kind(b->kind)) return -1;
    const bool inter = b->kind == DGPU_PRED_INTER || b->kind == DGPU_PRED_INTER_AVG ||
                       b->kind == DGPU_PRED_INTER_WAVG || (ext && b->kind != DGPU_PRED_PAL);
    if (!inter && b->kind != DGPU_PRED_INTRA && b->kind != DGPU_PRED_CFL && b->kind != DGPU_PRED_PAL) return -1;
    if (b->kind == DGPU_PRED_CFL && (b->plane == 0 || b->w != tw || b->h != th || tw != th || tw > 32))
        return -1;   // CfL: one unit per chroma block (cfl_ac + cfl_pred, :1372-1414)
    if (b->kind == DGPU_PRED_CFL ? ((b->mode & 15) >= b->w / 4 || (b->mode >> 4) >= b->h / 4)
                                 : (!inter && b->mode > 13))
        return -1;   // CFL: mode = cfl_ac's w_pad | h_pad << 4
    if (inter && (b->ref[0] >= DGPU_REC_EMU_SLOT || b->ref[1] >= DGPU_REC_EMU_SLOT || b->filter2d > 9)) return -1;
    if (b->tile_x0 < 0 || b->tile_y0 < 0 || b->tile_x1 > pw || b->tile_y1 > ph || b->x < b->tile_x0 ||
        b->y < b->tile_y0 || b->x >= b->tile_x1 || b->y >= b->tile_y1 ||
        (b->x + b->w > b->tile_x1 && b->tile_x1 != pw) || (b->y + b->h > b->tile_y1 && b->tile_y1 != ph))
        return -1;   // inside its tile; only the grid's last tiles' blocks overhang
    return 0;
}

// The recording streamed to the device while the decoder makes it: once a
// first flush has made the recorder's stream and device buffers, every
// kStreamChunk of new block / residual records is queued for upload on the
// recorder's stream right away (the pinned staging is read in place), so a
// flush uploads only the tail.  Only the prep reads these buffers, and every
// flush has finished its prep before it returns.
constexpr size_t kStreamChunk = 1 << 20;
static void stream_up(Dav1dGpuRecorder *r, Stage &s, Mem &d) {
    if (!r->streaming || s.n - s.up < kStreamChunk || s.n > d.cap || !s.pinned) return;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) return;
    if (prev != r->device && hipSetDevice(r->device) != hipSuccess) return;
    if (hipMemcpyAsync((uint8_t *)d.p + s.up, s.p + s.up, s.n - s.up, hipMemcpyHostToDevice, r->pst) == hipSuccess)
        s.up = s.n;
    if (prev != r->device) (void)hipSetDevice(prev);
}
// appends m bytes to a streamed stage: a copy may still be reading the old
// staging when it has to grow, so the recorder's stream is drained first
static void *stage_append(Dav1dGpuRecorder *r, Stage &s, size_t m) {
    if (s.n + m > s.cap && s.up && r->pst) {
        int prev = -1;
        if (hipGetDevice(&prev) == hipSuccess) {
            if (prev != r->device) (void)hipSetDevice(r->device);
            (void)hipStreamSynchronize(r->pst);
            if (prev != r->device) (void)hipSetDevice(prev);
        }
    }
    return s.append(m);
}

// appends the block with its data offset (or -1, or -2 - the INTER_WMASK
// block a COMPOUND_SEG chroma mask reads)
static int push_block(Dav1dGpuRecorder *r, const Dav1dGpuRecBlock *b, int32_t aux_off) {
    if (r->nblocks() >= (size_t)INT32_MAX / 2) return -1;
    void *q = stage_append(r, r->blocks, sizeof(*b));
    int32_t *o = (int32_t *)stage_append(r, r->baux_off, 4);
    if (!q || !o) return -1;
    memcpy(q, b, sizeof(*b));
    *o = aux_off;
    r->cell_bound += (int64_t)(b->w / tx_w(b->tx)) * (b->h / tx_h(b->tx)) + 1;   // (an inter-intra block adds one)
    stream_up(r, r->blocks, r->d_blocks);
    stream_up(r, r->baux_off, r->d_baux_off);
    return 0;
}

extern "C" int dav1d_gpu_rec_block(Dav1dGpuRecorder *r, const Dav1dGpuRecBlock *b) {
    if (check_block(r, b, false)) return -1;
    return push_block(r, b, -1);
}

extern "C" int dav1d_gpu_rec_block_aux(Dav1dGpuRecorder *r, const Dav1dGpuRecBlock *b, const void *aux,
                                       size_t aux_bytes) {
    if (check_block(r, b, true)) return -1;
    const size_t bpp = r->bpc / 8, w = b->w, h = b->h;
    size_t need = 0;
    switch (b->kind) {
    case DGPU_PRED_INTER_MASK:
        if (!aux) {   // a COMPOUND_SEG chroma block: the last INTER_WMASK block's mask
            if (b->plane == 0) return -1;
            return push_block(r, b, r->last_wmask >= 0 ? -2 - r->last_wmask : -1);
        }
        need = w * h;
        break;
    case DGPU_PRED_PAL: need = 8 * bpp + (w / 2) * h; break;
    case DGPU_PRED_INTER_INTRA:   // the block's ii / wedge mask; the intra mode DC / V / H / SMOOTH in `mode`
        if (w > 32 || h > 32 || tx_of(b->w, b->h) < 0 ||
            (b->mode != DGPU_DC_PRED && b->mode != DGPU_VERT_PRED && b->mode != DGPU_HOR_PRED && b->mode != DGPU_SMOOTH_PRED))
            return -1;
        need = w * h;
        break;
    case DGPU_PRED_WARP:
        if ((w & 7) || (h & 7) || (b->x & 7) || (b->y & 7)) return -1;
        need = 16 + (w / 8) * (h / 8) * 8;
        break;
    case DGPU_PRED_INTER_WMASK: {
        if (b->plane != 0 || b->weight > 1) return -1;
        const int32_t bi = (int32_t)r->nblocks();
        if (push_block(r, b, -1)) return -1;
        r->last_wmask = bi;
        return 0;
    }
    case DGPU_PRED_INTER_OBMC: {
        if (!aux || aux_bytes < 16) return -1;
        const int32_t n = *(const int32_t *)aux;
        if (n < 0 || n > 64) return -1;
        need = 16 + sizeof(ObmcBlockLap) * (size_t)n;
        break;
    }
    case DGPU_PRED_INTER_SCALED: {
        if (!aux || aux_bytes < 16) return -1;
        const int32_t n = *(const int32_t *)aux;
        if (n != 1 && n != 2) return -1;
        need = 16 + 16 * (size_t)n;
        if (aux_bytes != need) return -1;
        // steps of a valid reference scale (1/16x .. 2x: dav1d's svc step,
        // src/decode.c:3365-3369): up to 2048 per pixel; phases below 1024
        for (int k = 0; k < n; k++) {
            const ScaledBlockRef *q = (const ScaledBlockRef *)((const uint8_t *)aux + 16) + k;
            if (q->dx < 1 || q->dx > 2048 || q->dy < 1 || q->dy > 2048 || q->mx > 1023 || q->my > 1023) return -1;
        }
        break;
    }
    default: return -1;
    }
    if (!aux || aux_bytes != need) return -1;
    const size_t o = r->baux.n, pad = (16 - (aux_bytes & 15)) & 15;   // entries 16-byte aligned
    if (o + aux_bytes + pad > (size_t)INT32_MAX) return -1;
    uint8_t *q = (uint8_t *)stage_append(r, r->baux, aux_bytes + pad);
    if (!q) return -1;
    memcpy(q, aux, aux_bytes);
    memset(q + aux_bytes, 0, pad);
    if (push_block(r, b, (int32_t)o)) {
        r->baux.n = o;
        r->baux.up = std::min(r->baux.up, o);
        return -1;
    }
    stream_up(r, r->baux, r->d_baux);
    return 0;
}

extern "C" int dav1d_gpu_rec_residual(Dav1dGpuRecorder *r, int plane, int x, int y, int tx, int txtp, int eob,
                                      const void *coef) {
    int pw, ph;
    if (!r || !coef || !plane_dims(r, plane, pw, ph) || tx < 0 || tx >= DGPU_N_RECT_TX_SIZES) return -1;
    if (txtp < 0 || txtp >= DGPU_N_TX_TYPES_PLUS_LL || eob < 0) return -1;
    if (x < 0 || y < 0 || x >= pw || y >= ph || (x & 3) || (y & 3)) return -1;   // starts inside the grid
    const int sw = std::min(tx_w(tx), 32), sh = std::min(tx_h(tx), 32);
    const size_t cb = r->bpc == 8 ? 2 : 4;
    if (r->coefb.n / cb + (size_t)sw * sh > (size_t)INT32_MAX || r->nres() >= (size_t)INT32_MAX / 2) return -1;
    RecRes q{plane, x, y, tx, txtp, 0, 0, (int32_t)(r->coefb.n / cb)};
    auto at = [&](int cx, int cy) -> int32_t {   // the reference's layout: coef[cy + cx * sh]
        return r->bpc == 8 ? ((const int16_t *)coef)[cy + cx * sh] : ((const int32_t *)coef)[cy + cx * sh];
    };
    int nzw = 1, nzh = 1;
    if (!(eob == 0 && txtp == DGPU_DCT_DCT)) {   // the stored region: the bounding box of the non-zero coefficients
        for (int cx = 0; cx < sw; cx++)
            for (int cy = 0; cy < sh; cy++)
                if (at(cx, cy)) {
                    nzw = std::max(nzw, cx + 1);
                    nzh = std::max(nzh, cy + 1);
                }
        q.nzw = nzw;
        q.nzh = nzh;
    }   // else the DC-only call (src/itx_tmpl.c:53): one coefficient, nzw = nzh = 0
    uint8_t *d = (uint8_t *)r->coefb.append((size_t)nzw * nzh * cb);
    void *qq = stage_append(r, r->res, sizeof(q));
    if (!d || !qq) return -1;
    for (int cx = 0; cx < nzw; cx++)   // appended in the ABI's coefficient type, column by column
        memcpy(d + (size_t)cx * nzh * cb, (const uint8_t *)coef + (size_t)cx * sh * cb, (size_t)nzh * cb);
    memcpy(qq, &q, sizeof(q));
    stream_up(r, r->res, r->d_res);
    return 0;
}

// The last flush's outcome, once it has finished: its persistent
// wavefront's error word (workspace int32 [1], set by a wave that gave up
// waiting for its producers) is read back and cleared.  -6: the picture of
// that flush is incomplete; -3: HIP error.
static int recorder_poll(Dav1dGpuRecorder *r) {
    if (!r->pending_check) return 0;
    r->pending_check = false;
    // the flush copied its error word to page-locked memory before `done`
    if (hipEventSynchronize(r->done) != hipSuccess) return -3;
    return *(volatile int32_t *)r->flag ? -6 : 0;
}

extern "C" int dav1d_gpu_recorder_status(Dav1dGpuRecorder *r) {
    if (!r) return -1;
    if (hipSetDevice(r->device) != hipSuccess) return -3;
    return recorder_poll(r);
}

extern "C" int dav1d_gpu_recorder_stats(const Dav1dGpuRecorder *r, int32_t *n_units, int32_t *n_levels) {
    if (!r) return -1;
    if (n_units) *n_units = r->last_units;
    if (n_levels) *n_levels = r->last_levels;
    return 0;
}

extern "C" int dav1d_gpu_recorder_prep_ms(const Dav1dGpuRecorder *r, float *ms) {
    if (!r || !ms) return -1;
    *ms = r->prep_ms;
    return 0;
}

extern "C" int dav1d_gpu_recorder_flush(Dav1dGpuRecorder *r, const Dav1dGpuPlane dst[3],
                                        const Dav1dGpuPlane ref[DGPU_MAX_REFS][3], void *stream) {
    if (!r || !dst) return -1;
    const bool host = host_only();
    if (!host) {
        if (hipSetDevice(r->device) != hipSuccess) return -3;
        if (r->done && hipEventSynchronize(r->done) != hipSuccess) return -3;   // buffers free for reuse
    }
    // a previous flush whose wavefront gave up waiting is reported once,
    // here if dav1d_gpu_recorder_status did not report it: nothing is
    // launched and the recording is kept for a retry
    {
        const int st = recorder_poll(r);
        if (st) return st;
    }
    // DAV1D_GPU_REC_TIMING=1: host phase times on stderr (diagnostics)
    static const bool timing = getenv("DAV1D_GPU_REC_TIMING") != nullptr;
    // DAV1D_GPU_REC_DUMP=<file> (diagnostics): the upload image and the
    // schedule, appended, to compare builds; nothing is launched on the picture
    static const char *dump = getenv("DAV1D_GPU_REC_DUMP");
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto t_0 = now();
    auto lap = [&](const char *what) {
        if (!timing) return;
        const auto t = now();
        fprintf(stderr, "recorder %-8s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t_0).count());
        t_0 = t;
    };
    if (!host && !r->pst) {
        // the prep's streams at the device's greatest priority: the flush
        // waits for the prep, which must not queue behind other work that
        // shares its hardware queue (a process has GPU_MAX_HW_QUEUES of them,
        // 4 by default, for all its streams)
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
        if (hipStreamCreateWithPriority(&r->pst, hipStreamNonBlocking, hi) != hipSuccess) return -3;
        if (hipStreamCreateWithPriority(&r->cst, hipStreamNonBlocking, hi) != hipSuccess ||
            hipEventCreateWithFlags(&r->prep, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&r->coef_ev, hipEventDisableTiming) != hipSuccess || hipEventCreate(&r->pt0) != hipSuccess ||
            hipEventCreate(&r->pt1) != hipSuccess)
            return -3;
    }
    Exec X{host, r->pst, &r->d_tmp};
    // once a step may be queued, a failure drains the recorder's stream
    // before returning: a retry regrows buffers the queued steps still use
    auto fail = [&](int rc) {
        if (!host && r->pst) (void)hipStreamSynchronize(r->pst);
        if (!host && r->cst) (void)hipStreamSynchronize(r->cst);
        return rc;
    };
    const int bpp = r->bpc / 8;
    const size_t cb = r->bpc == 8 ? 2 : 4;
    int pw[3], ph[3], mw[3], mh[3];
    for (int p = 0; p < 3; p++) {
        plane_dims(r, p, pw[p], ph[p]);
        mw[p] = pw[p] / 4 + kMapPad4;   // per-4x4 maps over the grid plus the overhang transform blocks reach
        mh[p] = ph[p] / 4 + kMapPad4;
    }
    const int nb = (int)r->nblocks(), nres = (int)r->nres();
    // the maps, kept across flushes; cleared only when their size changes or
    // the stamps would overflow
    bool reset = (int64_t)r->res_base + nres >= INT32_MAX || (int64_t)r->cell_base + r->cell_bound >= INT32_MAX;
    for (int p = 0; p < 3; p++) reset |= r->map_w4[p] != mw[p] || r->map_h4[p] != mh[p];
    if (reset) {
        size_t tot = 0;
        for (int p = 0; p < 3; p++) {
            r->map_off[p] = tot;
            tot += (size_t)mw[p] * mh[p];
            r->map_w4[p] = mw[p];
            r->map_h4[p] = mh[p];
        }
        if (r->res_at.grow(tot * 4) || r->own.grow(tot * 4)) return -3;
        X.memset(r->res_at.p, 0xff, tot * 4);
        X.memset(r->own.p, 0xff, tot * 4);
        r->res_base = r->cell_base = 0;
    }
    const int32_t res_base = r->res_base, cell_base = r->cell_base;
    // the stamps of this flush, whatever its outcome, are below the next one's
    r->res_base += nres;
    r->cell_base += (int32_t)r->cell_bound;
    int32_t *res_at[3], *own[3];
    for (int p = 0; p < 3; p++) {
        res_at[p] = r->res_at.as<int32_t>() + r->map_off[p];
        own[p] = r->own.as<int32_t>() + r->map_off[p];
    }

    // 0. the recording, as recorded
    // the streamed records' mirrors sized for their staging's capacity (the
    // next recording's chunks then fit); a reallocated mirror is refilled
    auto mirror = [&](Mem &d, Stage &st) {
        const void *old = d.p;
        if (d.grow(host ? st.n : std::max(st.n, st.cap))) return -1;
        if (d.p != old) st.up = 0;
        return 0;
    };
    if (mirror(r->d_blocks, r->blocks) || mirror(r->d_baux_off, r->baux_off) || mirror(r->d_baux, r->baux) ||
        mirror(r->d_res, r->res) || r->d_coef.grow(r->coefb.n) || r->d_hdr.grow(sizeof(Hdr)) ||
        r->d_cnt.grow((size_t)nb * sizeof(BlockCnt)) || r->d_base.grow((size_t)nb * sizeof(BlockCnt)) ||
        r->d_auxend.grow((size_t)nb * 4))
        return fail(-3);
    if (!host && !r->rb) {
        if (hipHostMalloc(&r->rb, 1 << 16, 0) != hipSuccess) return fail(-3);
        r->rb_cap = 1 << 16;
    }
    if (!host && hipEventRecord(r->pt0, r->pst) != hipSuccess) return fail(-3);
    for (auto &m : {std::make_pair(&r->d_blocks, &r->blocks), std::make_pair(&r->d_baux_off, &r->baux_off),
                    std::make_pair(&r->d_baux, &r->baux), std::make_pair(&r->d_res, &r->res)}) {
        Stage &st = *m.second;   // the part not streamed yet
        if (host) st.up = 0;
        X.upload((uint8_t *)m.first->p + st.up, st.p + st.up, st.n - st.up);
        if (!X.err) st.up = st.n;
    }
    r->streaming = !host && !X.err;   // from now on the recording streams up as it is made
    Hdr *hdr = r->d_hdr.as<Hdr>();
    X.memset(hdr, 0, sizeof(Hdr));
    {   // residual lookup: per plane, the top-left 4x4 cell of each residual
        const RecRes *rs = r->d_res.as<RecRes>();
        struct { int32_t *m[3]; int32_t w[3]; } ra = {{res_at[0], res_at[1], res_at[2]}, {mw[0], mw[1], mw[2]}};
        X.each(nres, [=] __host__ __device__(int i) {
            const RecRes q = rs[i];
            ra.m[q.plane][(size_t)(q.y / 4) * ra.w[q.plane] + q.x / 4] = res_base + i;
        });
    }
    // 1. the cut: count, scan, totals
    CutCtx c;
    memset(&c, 0, sizeof(c));
    c.blocks = r->d_blocks.as<Dav1dGpuRecBlock>();
    c.baux_off = r->d_baux_off.as<int32_t>();
    c.baux = r->d_baux.as<uint8_t>();
    c.res = r->d_res.as<RecRes>();
    for (int p = 0; p < 3; p++) {
        c.res_at[p] = res_at[p];
        c.mw[p] = mw[p];
        c.pw[p] = pw[p];
        c.ph[p] = ph[p];
        c.ds_px[p] = (int32_t)(dst[p].stride / bpp);
        c.sbl[p] = p ? r->sb_log2 - 1 : r->sb_log2;
        for (int k = 0; k < DGPU_MAX_REFS; k++) {
            RefInfo &ri = c.ref[k][p];
            if (!ref) continue;
            ri.stride_b = ref[k][p].stride;
            ri.stride_px = (int32_t)(ref[k][p].stride / bpp);
            ri.w = ref[k][p].w;
            ri.h = ref[k][p].h;
            ri.ok = ref[k][p].data != nullptr;
        }
    }
    c.res_base = res_base;
    c.bpp = bpp;
    c.top_on = r->top_on;
    c.hdr = hdr;
    c.cnt = r->d_cnt.as<BlockCnt>();
    c.auxend = r->d_auxend.as<int32_t>();
    c.base = r->d_base.as<BlockCnt>();
    X.each(1, [=] __host__ __device__(int) { hdr->last_aux = -1; });
    X.each(nb, [=] __host__ __device__(int i) {
        const int e = cut_block<false>(c, i);
        if (e) aor(&hdr->err, e);
    });
    X.scan_blocks(c.cnt, r->d_base.as<BlockCnt>(), nb);
    {
        const BlockCnt *cnt = c.cnt, *base = c.base;
        const int32_t *auxend = c.auxend;
        X.each(1, [=] __host__ __device__(int) {
            if (nb) hdr->tot = BlockCntSum()(base[nb - 1], cnt[nb - 1]);
            hdr->aux_end = hdr->last_aux >= 0 ? base[hdr->last_aux].v[C_AUX] + auxend[hdr->last_aux] : 0;
        });
    }
    Hdr h1;
    {
        Hdr *hh = host ? hdr : (Hdr *)r->rb;
        X.fetch(hh, hdr, sizeof(Hdr));
        X.sync();
        if (X.err) return fail(X.err);
        h1 = *hh;
    }
    lap("cut");
    if (h1.err) return fail(-1);
    if (h1.tot.v[C_RES] != nres) return fail(-1);   // a residual outside every block
    // every emulated-edge offset (a job's o0, a unit's src_off into the
    // scratch, the kernels' row * kEmuStride) is int32 pixels: a flush whose
    // scratch would pass 2^31 pixels fails instead of wrapping (a hostile
    // stream of all-compound, all-outside cells reaches that below the 2^21
    // cell limit)
    if ((h1.tot.v[C_EROWS] + 1) * kEmuStride + 256 > (long long)INT32_MAX) return fail(-1);
    if (h1.tot.v[C_CELLS] >= (1 << 21) || h1.tot.v[C_RAW] >= INT32_MAX || h1.tot.v[C_EDGE] >= INT32_MAX ||
        h1.aux_end >= INT32_MAX)
        return fail(-1);
    const int n = (int)h1.tot.v[C_CELLS], nx = (int)h1.tot.v[C_XU], n_emu = (int)h1.tot.v[C_EJOBS];
    const int32_t emu_rows = (int32_t)h1.tot.v[C_EROWS];
    const size_t edge_px = (size_t)h1.tot.v[C_EDGE], aux_end = (size_t)h1.aux_end;
    const int64_t n_raw = h1.tot.v[C_RAW];
    if (r->d_cu.grow((size_t)n * sizeof(Dav1dGpuUnit)) || r->d_crec.grow((size_t)n * sizeof(Dav1dGpuIntraEdge)) ||
        r->d_caux.grow((size_t)n * 4) || r->d_csort.grow((size_t)n * 4) || r->d_jobs.grow((size_t)n * sizeof(LvJob)) ||
        r->d_rawc.grow((size_t)(n + 1) * 4) || r->d_raws.grow((size_t)(n + 1) * 4) || r->d_raw.grow((size_t)n_raw * 4) ||
        r->d_pcnt.grow((size_t)(n + 1) * 4) || r->d_pstart.grow((size_t)(n + 1) * 4) ||
        r->d_prod.grow((size_t)n_raw * 4) || r->d_lv.grow((size_t)n * 4) || r->d_keys.grow((size_t)n * 8) ||
        r->d_keys2.grow((size_t)n * 8) || r->d_rank.grow((size_t)n * 4) || r->d_dcnt.grow((size_t)(n + 1) * 4) ||
        r->d_dstart.grow((size_t)(n + 1) * 4) || r->d_deps.grow((size_t)n_raw * 4) ||
        r->d_auxp.grow(aux_end) || r->d_emu_jobs.grow((size_t)n_emu * sizeof(EmuJob)) ||
        r->d_xu0.grow((size_t)nx * sizeof(Dav1dGpuUnit)) || r->d_xa0.grow((size_t)nx * 4) ||
        r->d_units.grow((size_t)n * sizeof(Dav1dGpuUnit)) || r->d_recs.grow((size_t)n * sizeof(Dav1dGpuIntraEdge)) ||
        r->d_aux.grow((size_t)n * 4))
        return fail(-3);
    // 2. the write pass (the aux pool zero-filled first: its alignment gaps
    //    and unwritten record bytes are zero)
    c.cu = r->d_cu.as<Dav1dGpuUnit>();
    c.crec = r->d_crec.as<Dav1dGpuIntraEdge>();
    c.caux = r->d_caux.as<int32_t>();
    c.csort = r->d_csort.as<int32_t>();
    c.rawc = r->d_rawc.as<int32_t>();
    c.jobs = r->d_jobs.as<LvJob>();
    c.auxp = r->d_auxp.as<uint8_t>();
    c.emu = r->d_emu_jobs.as<EmuJob>();
    c.xu = r->d_xu0.as<Dav1dGpuUnit>();
    c.xa = r->d_xa0.as<int32_t>();
    X.memset(c.auxp, 0, aux_end);
    X.memset(c.rawc + n, 0, 4);
    // the coefficient pool goes up on a stream of its own, beside the prep's
    // kernels (only the wavefront reads it); the flush waits for it before
    // returning, so the recording may reuse its staging
    if (host) {
        X.upload(r->d_coef.p, r->coefb.p, r->coefb.n);
    } else if (r->coefb.n && (hipMemcpyAsync(r->d_coef.p, r->coefb.p, r->coefb.n, hipMemcpyHostToDevice, r->cst) != hipSuccess ||
                              hipEventRecord(r->coef_ev, r->cst) != hipSuccess)) {
        return fail(-3);
    }
    X.each(nb, [=] __host__ __device__(int i) { (void)cut_block<true>(c, i); });
    // 3. levels and producers: a cell sits one level above every pixel its
    //    edges (or CfL luma, or an inter-intra residual's prediction) read;
    //    its producers are the cells that wrote them.  A pixel no cell of this
    //    flush wrote came from an earlier flush on the same stream: no
    //    producer, level 0 for it.
    struct Maps {
        int32_t *own[3];
        int32_t w[3];
    } mp = {{own[0], own[1], own[2]}, {mw[0], mw[1], mw[2]}};
    const LvJob *jobs = c.jobs;
    //    every cell stamps its 4x4s in the writer map (the only overlap in a
    //    flush: an inter-intra block's prediction cell under its residual
    //    cells, which come after it in decode order and win)
    X.each(n, [=] __host__ __device__(int ci) {
        const LvJob j = jobs[ci];
        if (j.fl & LvJob::IIC) return;
        int32_t *wp = mp.own[j.p];
        for (int cy = j.y4; cy < j.y4 + j.ch4; cy++)
            for (int cx = j.x4; cx < j.x4 + j.cw4; cx++) wp[(size_t)cy * mp.w[j.p] + cx] = cell_base + ci;
    });
    // the contract (include/dav1d_gpu.h, dav1d_gpu_recorder_flush): the
    // cells of one flush do not overlap, an inter-intra prediction under its
    // own residual cells excepted.  Two overlapping cells leave one stamp on
    // a shared 4x4, so the other finds a stamp not its own whatever order
    // they ran in; the flush then fails instead of scheduling reads before
    // writes
    X.each(n, [=] __host__ __device__(int ci) {
        const LvJob j = jobs[ci];
        if (j.fl & LvJob::IIC) return;
        const int32_t *wp = mp.own[j.p];
        for (int cy = j.y4; cy < j.y4 + j.ch4; cy++)
            for (int cx = j.x4; cx < j.x4 + j.cw4; cx++)
                if (wp[(size_t)cy * mp.w[j.p] + cx] != cell_base + ci) {
                    aor(&hdr->err, E_OVERLAP);
                    return;
                }
    });
    X.each(n, [=] __host__ __device__(int ci) {
        const LvJob j = jobs[ci];
        if (!(j.fl & LvJob::IIC)) return;
        int32_t *wp = mp.own[j.p];
        for (int cy = j.y4; cy < j.y4 + j.ch4; cy++)
            for (int cx = j.x4; cx < j.x4 + j.cw4; cx++) {
                int32_t &o = wp[(size_t)cy * mp.w[j.p] + cx];
                if (o < cell_base) o = cell_base + ci;   // (under its residual cells: theirs)
            }
    });
    //    every cell looks its producers up (a writer at or after the cell in
    //    decode order has not written yet: none), sorted, duplicate-free
    int32_t *raws = r->d_raws.as<int32_t>(), *raw = r->d_raw.as<int32_t>(), *pcnt = r->d_pcnt.as<int32_t>();
    int32_t *pstart = r->d_pstart.as<int32_t>(), *prod = r->d_prod.as<int32_t>();
    X.scan(c.rawc, raws, n + 1);
    X.memset(pcnt + n, 0, 4);
    X.each(n, [=] __host__ __device__(int ci) {
        const LvJob j = jobs[ci];
        int32_t *seg = raw + raws[ci];
        int m = 0;
        const int32_t lo = cell_base, hi = cell_base + ci;   // this flush, before the cell
        int32_t last = -1;   // (runs of one writer are common: a row of its 4x4s)
        lookups<true>(j, mp.own[j.p], mp.w[j.p], mp.own[0], mp.w[0], [&](int32_t o) {
            int32_t v;
            if (o <= -2) v = -2 - o;   // the inter-intra prediction cell, by index
            else if (o >= lo && o < hi) v = o - cell_base;
            else return;
            if (v != last) seg[m++] = v;
            last = v;
        });
        int u = 0;   // sorted, duplicate-free (lists are short: insertion sort in place)
        for (int a = 0; a < m; a++) {
            const int32_t v = seg[a];
            int b = u;
            while (b > 0 && seg[b - 1] > v) b--;
            if (b > 0 && seg[b - 1] == v) continue;
            for (int k = u; k > b; k--) seg[k] = seg[k - 1];
            seg[b] = v;
            u++;
        }
        pcnt[ci] = u;
    });
    X.scan(pcnt, pstart, n + 1);
    X.each(n, [=] __host__ __device__(int ci) {
        const int32_t *s = raw + raws[ci];
        int32_t *d = prod + pstart[ci];
        for (int k = 0, e = pstart[ci + 1] - pstart[ci]; k < e; k++) d[k] = s[k];
    });
    //    the levels in decode order, from the producers' (decode order is a
    //    topological order), and the sort keys
    int32_t *lv = r->d_lv.as<int32_t>();
    uint64_t *keys = r->d_keys.as<uint64_t>(), *keys2 = r->d_keys2.as<uint64_t>();
    if (n) {
        LevelArgs la{pstart, prod, c.csort, c.cu, lv, keys, hdr, n, kLevelSpinLimit};
        if (host) {
            for (int ci = 0; ci < n; ci++) {
                int d = -1;
                for (int k = pstart[ci]; k < pstart[ci + 1]; k++) d = std::max(d, lv[prod[k]]);
                lv[ci] = d + 1;
                keys[ci] = level_key(c.cu[ci], c.csort[ci], d + 1, ci);
                hdr->max_level = std::max(hdr->max_level, d + 1);
            }
        } else if (!X.err) {
            X.memset(lv, 0xff, (size_t)n * 4);
            k_levels<<<dim3((unsigned)((n + 63) / 64)), 64, 0, r->pst>>>(la);
            if (hipGetLastError() != hipSuccess) X.err = -3;
        }
    }
    // 4. level order, size classes inside a level, then kind / mode / type:
    //    one radix sort of the keys (distinct: they hold the decode index)
    X.sort(keys, keys2, n, 21, 21 + 20 + 16);
    // the rank of every decode-order cell, and the level / class ranges: a
    // (level, class) run ends where the sorted key's top bits change (levels
    // past 2^16 fail the flush below)
    const int lb = std::min(n, 1 << 16);
    if (r->d_ends.grow((size_t)lb * (NC + 1) * 4) || r->d_lend.grow((size_t)(lb + 1) * 4)) return fail(-3);
    int32_t *ends = r->d_ends.as<int32_t>(), *lend = r->d_lend.as<int32_t>(), *rank = r->d_rank.as<int32_t>();
    int32_t *dcnt = r->d_dcnt.as<int32_t>(), *dstart = r->d_dstart.as<int32_t>(), *deps = r->d_deps.as<int32_t>();
    X.memset(ends, 0, (size_t)lb * (NC + 1) * 4);
    X.memset(lend, 0, (size_t)(lb + 1) * 4);
    X.memset(dcnt + n, 0, 4);
    X.each(n, [=] __host__ __device__(int i) {
        const uint64_t k = keys2[i];
        const int ci = (int)(k & ((1u << 21) - 1));
        rank[ci] = i;
        const uint64_t lt = k >> 36;   // level | tx
        const int level = (int)(lt >> 5), tx = (int)(lt & 31);
        if (level < lb && (i + 1 == n || (keys2[i + 1] >> 36) != lt)) {   // the last of its (level, class) run
            ends[(size_t)level * (NC + 1) + tx + 1] = i + 1;
            if (i + 1 == n || (int)(keys2[i + 1] >> 41) != level) lend[level + 1] = i + 1;
        }
        dcnt[i] = pcnt[ci];   // (producer lists in level order)
    });
    X.scan(dcnt, dstart, n + 1);
    // 5. the image: units and records at their ranks, producers as ranks
    Dav1dGpuUnit *units = r->d_units.as<Dav1dGpuUnit>();
    Dav1dGpuIntraEdge *recs = r->d_recs.as<Dav1dGpuIntraEdge>();
    int32_t *aux = r->d_aux.as<int32_t>();
    {
        const Dav1dGpuUnit *cu = c.cu;
        const Dav1dGpuIntraEdge *crec = c.crec;
        const int32_t *caux = c.caux;
        X.each(n, [=] __host__ __device__(int i) {
            const int ci = (int)(keys2[i] & ((1u << 21) - 1));
            memcpy(&units[i], &cu[ci], sizeof(Dav1dGpuUnit));   // coef_off / edge_off are decode-order pool offsets
            aux[i] = caux[ci];
            Dav1dGpuIntraEdge e;
            memcpy(&e, &crec[ci], sizeof(e));
            e.unit = i;
            memcpy(&recs[i], &e, sizeof(e));
            int32_t *o = deps + dstart[i];
            for (int k = pstart[ci]; k < pstart[ci + 1]; k++) *o++ = rank[prod[k]];
        });
    }
    // 6. the launch-ahead units in class order (a stable sort by size class)
    //    and, with top_edge, the backup runs of those whose bottom row ends a
    //    superblock row (decode order; dav1d_backup_ipred_edge, run between
    //    that launch and the wavefront; a residual on them is added by a
    //    wavefront unit, which backs its row up again)
    if (r->d_xk.grow((size_t)nx * 8) || r->d_xk2.grow((size_t)nx * 8) ||
        r->d_xunits.grow((size_t)nx * sizeof(Dav1dGpuUnit)) || r->d_xaux.grow((size_t)nx * 4) ||
        r->d_xends.grow((NC + 1) * 4) || r->d_bkf.grow((size_t)(nx + 1) * 4) || r->d_bks.grow((size_t)(nx + 1) * 4) ||
        r->d_bk.grow((size_t)nx * sizeof(Dav1dGpuEdgeBackup)))
        return fail(-3);
    uint64_t *xk = r->d_xk.as<uint64_t>(), *xk2 = r->d_xk2.as<uint64_t>();
    Dav1dGpuUnit *xunits = r->d_xunits.as<Dav1dGpuUnit>();
    int32_t *xaux = r->d_xaux.as<int32_t>(), *xends = r->d_xends.as<int32_t>();
    int32_t *bkf = r->d_bkf.as<int32_t>(), *bks = r->d_bks.as<int32_t>();
    Dav1dGpuEdgeBackup *bk = r->d_bk.as<Dav1dGpuEdgeBackup>();
    {
        const Dav1dGpuUnit *xu0 = c.xu;
        const int32_t *xa0 = c.xa;
        X.memset(xends, 0, (NC + 1) * 4);
        X.each(nx, [=] __host__ __device__(int i) { xk[i] = (uint64_t)xu0[i].tx << 32 | (uint64_t)i; });
        X.sort(xk, xk2, nx, 32, 37);
        X.each(nx, [=] __host__ __device__(int k) {
            const int i = (int)(xk2[k] & 0xffffffffu), tx = (int)(xk2[k] >> 32);
            memcpy(&xunits[k], &xu0[i], sizeof(Dav1dGpuUnit));
            xaux[k] = xa0[i];
            if (k + 1 == nx || (int)(xk2[k + 1] >> 32) != tx) xends[tx + 1] = k + 1;
        });
        if (r->top_on && nx) {
            struct Tops {
                int32_t ds[3], tw[3], th[3], sbl[3];
            } tp;
            for (int p = 0; p < 3; p++) {
                tp.ds[p] = c.ds_px[p];
                tp.tw[p] = r->top[p].w;
                tp.th[p] = r->top[p].h;
                tp.sbl[p] = c.sbl[p];
            }
            auto run = [=] __host__ __device__(const Dav1dGpuUnit &u, Dav1dGpuEdgeBackup &o) -> bool {
                const int p = u.plane;
                const int uy = u.dst_off / tp.ds[p], ux = u.dst_off % tp.ds[p], y1 = uy + tx_h(u.tx);
                const int sby = (y1 >> tp.sbl[p]) - 1, w = min(tx_w(u.tx), tp.tw[p] - ux);
                o = Dav1dGpuEdgeBackup{p, sby, ux, w};
                return (y1 & ((1 << tp.sbl[p]) - 1)) == 0 && sby < tp.th[p] && w > 0;
            };
            X.memset(bkf + nx, 0, 4);
            X.each(nx, [=] __host__ __device__(int i) {
                Dav1dGpuEdgeBackup o;
                bkf[i] = run(xu0[i], o) ? 1 : 0;
            });
            X.scan(bkf, bks, nx + 1);
            X.each(nx, [=] __host__ __device__(int i) {
                Dav1dGpuEdgeBackup o;
                if (run(xu0[i], o)) bk[bks[i]] = o;
            });
        }
        const bool top_on = r->top_on;
        X.each(1, [=] __host__ __device__(int) {
            hdr->n_bk = top_on && nx ? bks[nx] : 0;
            hdr->pad_[0] = dstart[n];   // the producer entries
        });
    }
    // 7. read back: the level count, the class ranges, the backup runs
    Hdr h2;
    int32_t x_end[NC + 1];
    {
        Hdr *hh = host ? hdr : (Hdr *)r->rb;
        int32_t *xe = host ? xends : (int32_t *)((uint8_t *)r->rb + 256);
        if (!host && hipEventRecord(r->pt1, r->pst) != hipSuccess) return fail(-3);
        X.fetch(hh, hdr, sizeof(Hdr));
        X.fetch(xe, xends, (NC + 1) * 4);
        X.sync();
        if (X.err) return fail(X.err);
        h2 = *hh;
        if (!host && hipEventElapsedTime(&r->prep_ms, r->pt0, r->pt1) != hipSuccess) r->prep_ms = -1;
        memcpy(x_end, xe, sizeof(x_end));
    }
    if (h2.err & E_STALL) return fail(-3);
    if (h2.err) return fail(-1);   // overlapping cells
    const int max_level = n ? h2.max_level : 0;
    if (max_level >= (1 << 16)) return fail(-1);
    const int n_levels = n ? max_level + 1 : 0, n_bk = h2.n_bk;
    const int64_t n_deps = h2.pad_[0];
    r->unit_start.assign(n_levels + 1, 0);
    r->class_start.assign((size_t)n_levels * (NC + 1), 0);
    if (n_levels) {
        const size_t ce = (size_t)n_levels * (NC + 1) * 4, le = (size_t)(n_levels + 1) * 4;
        if (!host && ce + le > r->rb_cap) {
            (void)hipHostFree(r->rb);
            r->rb = nullptr;
            r->rb_cap = 0;
            if (hipHostMalloc(&r->rb, ce + le, 0) != hipSuccess) return fail(-3);
            r->rb_cap = ce + le;
        }
        int32_t *ce_h = host ? ends : (int32_t *)r->rb, *le_h = host ? lend : (int32_t *)((uint8_t *)r->rb + ce);
        X.fetch(ce_h, ends, ce);
        X.fetch(le_h, lend, le);
        X.sync();
        if (X.err) return fail(X.err);
        memcpy(r->class_start.data(), ce_h, ce);
        memcpy(r->unit_start.data(), le_h, le);
        r->unit_start[0] = 0;
    }
    {   // run ends -> counts: the runs are in (level, class) order, so a run
        // starts where the previous non-empty one ended
        int32_t prev = 0;
        for (int l = 0; l < n_levels; l++) {
            int32_t *cs = &r->class_start[(size_t)l * (NC + 1)];
            for (int k = 1; k <= NC; k++)
                if (cs[k]) {
                    const int32_t e = cs[k];
                    cs[k] = e - prev;
                    prev = e;
                }
        }
        for (int l = 0; l < n_levels; l++) {
            if (r->unit_start[l + 1] < r->unit_start[l]) r->unit_start[l + 1] = r->unit_start[l];   // (levels are dense)
            int32_t *cs = &r->class_start[(size_t)l * (NC + 1)];
            for (int k = 0; k < NC; k++) cs[k + 1] += cs[k];
        }
    }
    int32_t x_class[NC + 1];
    x_class[0] = 0;
    for (int k = 0; k < NC; k++) x_class[k + 1] = x_end[k + 1] ? x_end[k + 1] : x_class[k];
    lap("schedule");
    r->rec_start = r->unit_start;
    r->run_start.assign(n_levels + 1, 0);
    r->last_units = n;
    r->last_levels = n_levels;
    const size_t bu = (size_t)n * sizeof(Dav1dGpuUnit), br = (size_t)n * sizeof(Dav1dGpuIntraEdge), bc = r->coefb.n,
                 be = (size_t)n_emu * sizeof(EmuJob), ba = (size_t)n * 4, bxu = (size_t)nx * sizeof(Dav1dGpuUnit),
                 bxa = (size_t)nx * 4, bp = aux_end, bbk = (size_t)n_bk * sizeof(Dav1dGpuEdgeBackup);
    if (!host && r->coefb.n && hipEventSynchronize(r->coef_ev) != hipSuccess) return fail(-3);
    if (dump) {   // image: units | records | coefficients | emu jobs | per-unit aux |
                  // launch-ahead units (class order) | their aux | aux pool | backup runs
        if (FILE *f = fopen(dump, "ab")) {
            std::vector<uint8_t> tmp;
            auto put = [&](const void *p, size_t nbytes) {
                if (!nbytes) return;
                if (host) {
                    fwrite(p, 1, nbytes, f);
                    return;
                }
                tmp.resize(nbytes);
                if (hipMemcpy(tmp.data(), p, nbytes, hipMemcpyDeviceToHost) == hipSuccess) fwrite(tmp.data(), 1, nbytes, f);
            };
            const int64_t hdr4[4] = {n, n_levels, (int64_t)nx, (int64_t)(bu + br + bc + be + ba + bxu + bxa + bp + bbk)};
            fwrite(hdr4, 1, sizeof(hdr4), f);
            put(units, bu);
            put(recs, br);
            put(r->d_coef.p, bc);
            put(c.emu, be);
            put(aux, ba);
            put(xunits, bxu);
            put(xaux, bxa);
            put(c.auxp, bp);
            put(bk, bbk);
            fwrite(r->unit_start.data(), 1, r->unit_start.size() * 4, f);
            fwrite(r->class_start.data(), 1, r->class_start.size() * 4, f);
            put(dstart, (size_t)(n + 1) * 4);
            put(deps, (size_t)n_deps * 4);
            fwrite(x_class, 1, sizeof(x_class), f);
            fclose(f);
        }
    }
    if ((!n && !nx) || host || dump) {
        r->drop_recording();
        return 0;
    }

    // 8. the picture's work on the caller's stream, behind the prep
    hipStream_t st = (hipStream_t)stream;
    if (hipEventRecord(r->prep, r->pst) != hipSuccess || hipStreamWaitEvent(st, r->prep, 0) != hipSuccess)
        return fail(-3);
    Dav1dGpuIntraSchedule s;
    memset(&s, 0, sizeof(s));
    s.n_levels = n_levels;
    s.flags = DGPU_IS_FUSED | DGPU_IS_PERSISTENT | DGPU_IS_DEVICE_DEPS | DGPU_IS_LEVEL0_BATCH;
    s.unit_start = r->unit_start.data();
    s.class_start = r->class_start.data();
    s.rec_start = r->rec_start.data();
    s.run_start = r->run_start.data();
    s.dep_start = dstart;
    s.deps = deps;
    const int64_t wsb = n ? dav1d_gpu_intra_workspace_bytes(&s, n) : 16;
    if (wsb < 0) return fail(-2);
    if (r->d_edges.grow(edge_px * bpp) || r->d_work.grow((size_t)wsb) ||
        (n_emu && r->d_emu.grow((size_t)emu_rows * kEmuStride * bpp + 256)))
        return fail(-3);
    // once the caller's stream may use the buffers, a failure drains it too
    auto drained = [&](int rc) {
        (void)hipStreamSynchronize(st);
        return fail(rc);
    };
    if (n_emu) {   // the clamped footprints, before the wavefront reads them
        EmuArgs ea;
        memset(&ea, 0, sizeof(ea));
        for (int k = 0; k < DGPU_MAX_REFS - 1; k++)
            for (int p = 0; p < 3; p++) {
                ea.ref[k][p] = ref[k][p].data;
                ea.stride[k][p] = (int32_t)(ref[k][p].stride / bpp);
                ea.w[k][p] = ref[k][p].w;
                ea.h[k][p] = ref[k][p].h;
            }
        ea.out = r->d_emu.p;
        ea.jobs = c.emu;
        ea.n = n_emu;
        ea.rows = emu_rows;
        if (r->bpc == 8)
            k_emu_footprints<uint8_t><<<dim3(ea.n), 64, 0, st>>>(ea);
        else
            k_emu_footprints<uint16_t><<<dim3(ea.n), 64, 0, st>>>(ea);
        if (hipGetLastError() != hipSuccess) return drained(-3);
    }
    s.workspace = r->d_work.p;
    s.workspace_bytes = wsb;
#if DGPU_BOUNDS
    {   // every buffer of this flush with its exact byte size (whole 16-B
        // blocks: Stage reads the 16-B blocks holding a region's first and
        // last byte), for the launches' range tables
        auto &bx = dgpu::bnd_extra();
        bx.clear();
        auto reg = [&](const void *p, size_t nbytes, int id) {
            if (p && nbytes) bx.push_back(dgpu::BndRange{p, (nbytes + 15) & ~(size_t)15, id});
        };
        reg(units, bu, dgpu::BND_UNITS);
        reg(recs, br, dgpu::BND_RECS);
        // DAV1D_GPU_BND_SELFTEST=1: register the coefficient pool 64 bytes
        // short, so the diagnostics must report the last units' coefficient
        // reads (the check's positive control)
        static const bool selftest = getenv("DAV1D_GPU_BND_SELFTEST") != nullptr;
        reg(r->d_coef.p, selftest && bc > 128 ? bc - 64 : bc, dgpu::BND_COEF);
        reg(r->d_edges.p, edge_px * bpp, dgpu::BND_EDGES);
        reg(aux, ba, dgpu::BND_AUX);
        reg(c.auxp, bp, dgpu::BND_AUXPOOL);
        reg(r->d_work.p, (size_t)wsb, dgpu::BND_WORK);
        reg(dstart, (size_t)(n + 1) * 4, dgpu::BND_WORK);
        reg(deps, (size_t)n_deps * 4, dgpu::BND_WORK);
        if (n_emu) reg(r->d_emu.p, (size_t)emu_rows * kEmuStride * bpp, dgpu::BND_EMU);
        if (nx) {
            reg(xunits, bxu, dgpu::BND_XUNITS);
            reg(xaux, bxa, dgpu::BND_XAUX);
        }
    }
#endif
    Dav1dGpuFrameBatch fb;
    memset(&fb, 0, sizeof(fb));
    Dav1dGpuIntraEdgeBatch eb;
    memset(&eb, 0, sizeof(eb));
    for (int p = 0; p < 3; p++) {
        fb.dst[p] = dst[p];
        eb.pic[p] = dst[p];
        if (ref)
            for (int k = 0; k < DGPU_REC_EMU_SLOT; k++) fb.ref[k][p] = ref[k][p];
        if (n_emu) fb.ref[DGPU_REC_EMU_SLOT][p] = Dav1dGpuPlane{r->d_emu.p, (int64_t)kEmuStride * bpp, kEmuStride, emu_rows};
        eb.sb_log2[p] = c.sbl[p];
        if (r->top_on) eb.top_edge[p] = r->top[p];
    }
    fb.units = units;
    fb.n_units = n;
    fb.class_start[NC] = n;
    fb.coef = r->d_coef.p;
    fb.edges = r->d_edges.p;
    fb.bitdepth_max = r->bdmax;
    fb.cfl_luma = dst[0];
    fb.cfl_ss = 3;
    fb.aux = aux;
    fb.aux_pool = c.auxp;
    if (nx) {   // WARP / INTER_WMASK / INTER_OBMC / INTER_SCALED predictions ahead of the wavefront
        Dav1dGpuFrameBatch xb = fb;
        xb.units = xunits;
        xb.n_units = nx;
        for (int k = 0; k <= NC; k++) xb.class_start[k] = x_class[k];
        for (int k = 0; k < NC; k++) xb.class_warp[k] = x_class[k + 1] - x_class[k];
        xb.aux = xaux;
        const int xrc = r->bpc == 8 ? dav1d_gpu_recon_8bpc(&xb, stream) : dav1d_gpu_recon_16bpc(&xb, stream);
        if (xrc) return drained(xrc);
    }
    if (n_bk) {   // their superblock-bottom rows into top_edge, before the wavefront
        const int brc = r->bpc == 8 ? dav1d_gpu_backup_ipred_edge_8bpc(&eb, bk, n_bk, stream)
                                    : dav1d_gpu_backup_ipred_edge_16bpc(&eb, bk, n_bk, stream);
        if (brc) return drained(brc);
    }
    eb.units = units;
    eb.edges = r->d_edges.p;
    eb.recs = recs;
    eb.n_recs = n;
    eb.bitdepth_max = r->bdmax;
    if (n) {
        const int rc = r->bpc == 8 ? dav1d_gpu_recon_intra_frame_8bpc(&fb, &eb, &s, stream)
                                   : dav1d_gpu_recon_intra_frame_16bpc(&fb, &eb, &s, stream);
        lap("launch");
        if (rc) return drained(rc);
    }
#if DGPU_BOUNDS
    dgpu::bnd_extra().clear();   // this flush's launches have their tables
#endif
    if (!r->done && hipEventCreateWithFlags(&r->done, hipEventDisableTiming) != hipSuccess) return drained(-3);
    // the wavefront's error word (workspace int32 [1]) follows on the stream
    if (n && !r->flag && hipHostMalloc(&r->flag, 16, 0) != hipSuccess) return drained(-3);
    if (n && hipMemcpyAsync(r->flag, (const int32_t *)r->d_work.p + 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess)
        return drained(-3);
    if (hipEventRecord(r->done, st) != hipSuccess) return drained(-3);
    r->pending_check = n > 0;
    r->drop_recording();
    return 0;
}
