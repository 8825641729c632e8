// recorder.hip -- the batch recorder at the reconstruction seam (SURVEY 8(f)
// row 2; include/dav1d_gpu.h, Dav1dGpuRecorder).
//
// A decoder's recon_b_inter / recon_b_intra (src/recon_tmpl.c:1598, :1195)
// hand over, per block and plane, what they would have passed to the DSP
// (one Dav1dGpuRecBlock) and, per coded transform block, what they would
// have passed to inv_txfm_add (dav1d_gpu_rec_residual).  A flush turns the
// record into the device's work:
//   1. transform units in decode order: every transform cell of every block
//      (recon_b_* iterate the block's transform grid, :1258-1262), carrying
//      the block's prediction and the cell's residual if one was recorded;
//   2. per intra / CfL unit the dav1d_prepare_intra_edges record exactly as
//      recon_b_intra derives it: have_left / have_top against the tile start,
//      the tile end as (w, h), and the per-transform edge flags of
//      :1252-1266 from the block's intra_edge_flags;
//   3. dependency levels at 4x4 granularity: inter units read only their
//      references (level 0); an intra unit sits one level above every unit
//      whose pixels the edges of its remapped mode read (CfL: also the
//      co-located luma), and those units are its producers;
//   4. units sorted by (level, size class, kind, mode, type), records in the
//      same order, coefficients compacted to the stored region, and one
//      persistent wavefront launch (dav1d_gpu_recon_intra_frame_*) whose
//      waves wait for their producers only.
// Host code only; the device work runs on the caller's stream.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <atomic>
#include <mutex>
#include <numeric>
#include <thread>
#include <vector>

#include "bounds.hpp"
#include "dav1d_gpu.h"

#ifndef DGPU_BOUNDS
#define DGPU_BOUNDS 0
#endif

namespace {

struct TxDim { int w, h; };
constexpr TxDim kTx[DGPU_N_RECT_TX_SIZES] = {
    {4, 4}, {8, 8}, {16, 16}, {32, 32}, {64, 64}, {4, 8}, {8, 4}, {8, 16}, {16, 8}, {16, 32},
    {32, 16}, {32, 64}, {64, 32}, {4, 16}, {16, 4}, {8, 32}, {32, 8}, {16, 64}, {64, 16}};

// av1_intra_prediction_edges needs (src/ipred_prepare_tmpl.c:50-75):
// bit0 left, 1 top, 2 top-left, 3 top-right, 4 bottom-left
constexpr uint8_t kNeeds[14] = {3, 2, 1, 1, 2, 0, 14, 7, 21, 3, 3, 3, 7, 7};

// the mode remap of dav1d_prepare_intra_edges (:83-104)
int remap_mode(int mode, int angle, bool hl, bool ht) {
    static const int dir[8] = {90, 180, 45, 135, 113, 157, 203, 67};
    if (mode >= 1 && mode <= 8) {
        const int a = dir[mode - 1] + 3 * angle;
        if (a <= 90) return a < 90 && ht ? DGPU_Z1_PRED : DGPU_VERT_PRED;
        if (a < 180) return DGPU_Z2_PRED;
        return a > 180 && hl ? DGPU_Z3_PRED : DGPU_HOR_PRED;
    }
    if (mode == 0) return hl ? (ht ? DGPU_DC_PRED : DGPU_LEFT_DC_PRED) : (ht ? DGPU_TOP_DC_PRED : DGPU_DC_128_PRED);
    if (mode == 12) return hl ? (ht ? DGPU_PAETH_PRED : DGPU_HOR_PRED) : (ht ? DGPU_VERT_PRED : DGPU_DC_128_PRED);
    return mode;
}

struct Residual {
    int plane, x, y, tx, txtp, nzw, nzh;
    size_t coef;   // offset into the recorder's compact pool
};

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int grow(size_t n) {
        if (n <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        // rounded up to 256 bytes: the one read past a buffer's last element
        // the kernels make by design is Stage's (the 16-byte block holding a
        // region's last byte, at most 15 bytes further).  (Round 3 padded
        // every buffer with 64 KiB after an unexplained fault; the DGPU_BOUNDS
        // build, which checks every access against these buffers' exact
        // sizes, reports none)
        const size_t sz = (n + 255) & ~(size_t)255;
        if (hipMalloc(&p, sz) != hipSuccess) return -1;
        cap = n;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// page-locked staging, so the uploads do not wait for the stream.
// DAV1D_GPU_REC_PIN (tuning): "default" hipHostMalloc, otherwise (the
// default) non-coherent hipHostMalloc (CPU-cached: the fill writes it at
// memory speed).  Nothing in the library registers ordinary host memory:
// round 5 removed the hipHostRegister mode that rounds 3-4 suspected of the
// intermittent illegal-address faults
static int pin_mode() {
    static const int m = [] {
        const char *e = getenv("DAV1D_GPU_REC_PIN");
        return (e && !strcmp(e, "default")) ? 0 : 1;
    }();
    return m;
}
struct PinnedBuf {
    void *p = nullptr;
    size_t cap = 0;
    int grow(size_t n) {
        if (n <= cap) return 0;
        release();
        if (hipHostMalloc(&p, n, pin_mode() ? hipHostMallocNonCoherent : hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            return -1;
        }
        cap = n;
        return 0;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// A few host workers kept for a recorder's lifetime: every parallel step of
// a flush runs on them (no thread start per step).  run(nt, f) calls f(t) for
// t in [0, nt) and returns when all have; the caller runs t = 0.
class Pool {
public:
    explicit Pool(int n) : n_(std::max(1, n)) {
        for (int i = 1; i < n_; i++) th_.emplace_back([this, i] { loop(i); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> l(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return n_; }
    template <typename F> void run(int nt, F &&f) {
        nt = std::min(nt, n_);
        if (nt <= 1) {
            f(0);
            return;
        }
        {
            std::lock_guard<std::mutex> l(m_);
            job_ = [&f](int t) { f(t); };
            nt_ = nt;
            pending_ = nt - 1;
            gen_++;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [this] { return pending_ == 0; });
    }

private:
    void loop(int i) {
        unsigned seen = 0;
        for (;;) {
            std::function<void(int)> job;
            int nt;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                job = job_;
                nt = nt_;
            }
            if (i < nt) {
                job(i);
                std::lock_guard<std::mutex> l(m_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::function<void(int)> job_;
    int nt_ = 0, pending_ = 0;
    unsigned gen_ = 0;
    bool stop_ = false;
};

// LSD radix sort of 64-bit keys on bits [lo, hi), digits of at most 13 bits, by up to
// nt threads (per-thread digit counts over contiguous chunks, so it stays
// stable: keys whose low bits hold their input index need not sort those)
void radix_sort(std::vector<uint64_t> &k, std::vector<uint64_t> &tmp, int lo, int hi, Pool &pool) {
    int nt = pool.size();
    const int passes = (hi - lo + 12) / 13, DB = (hi - lo + passes - 1) / std::max(passes, 1), ND = 1 << DB;
    const size_t n = k.size();
    tmp.resize(n);
    nt = n < 65536 ? 1 : nt;
    std::vector<uint32_t> cnt((size_t)nt * ND);
    for (int sh = lo; sh < hi; sh += DB) {
        auto count = [&](int t) {
            uint32_t *c = &cnt[(size_t)t * ND];
            std::fill(c, c + ND, 0);
            for (size_t i = n * t / nt, e = n * (t + 1) / nt; i < e; i++) c[(k[i] >> sh) & (ND - 1)]++;
        };
        auto scatter = [&](int t) {
            uint32_t *c = &cnt[(size_t)t * ND];
            for (size_t i = n * t / nt, e = n * (t + 1) / nt; i < e; i++) tmp[c[(k[i] >> sh) & (ND - 1)]++] = k[i];
        };
        pool.run(nt, count);
        uint32_t acc = 0;   // digit-major, then thread: every thread's keys of a digit after the earlier threads'
        for (int d = 0; d < ND; d++)
            for (int t = 0; t < nt; t++) {
                const uint32_t v = cnt[(size_t)t * ND + d];
                cnt[(size_t)t * ND + d] = acc;
                acc += v;
            }
        pool.run(nt, scatter);
        k.swap(tmp);
    }
}

// emu_edge per transform / prediction unit (src/recon_tmpl.c:986-999,
// scaled :1036-1046, warp :1168-1177): a footprint that leaves its reference
// picture is copied, every read clamped, into a scratch plane of kEmuStride
// pixels per row (a band of rows per copy; warp 8x8s side by side)
constexpr int kEmuStride = 128;
struct EmuJob {
    int32_t x0, y0;   // the footprint's top-left in the reference (may be outside)
    int32_t o0;       // its top-left in the scratch plane (pixels)
    uint8_t w, h, slot, plane;
};
static_assert(sizeof(EmuJob) == 16, "EmuJob layout");

struct EmuArgs {
    const void *ref[DGPU_MAX_REFS - 1][3];
    int32_t stride[DGPU_MAX_REFS - 1][3];   // pixels
    int32_t w[DGPU_MAX_REFS - 1][3], h[DGPU_MAX_REFS - 1][3];
    void *out;
    const EmuJob *jobs;
    int32_t n, rows;   // rows: the scratch plane's (diagnostics)
};

// one 64-lane workgroup per footprint: lanes along the row, clamped reads
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

// per 4x4 cell of a plane: the decode-order cell that last wrote it, stored
// as the flush's cell base + the cell index, so the maps are never cleared:
// an entry below the current base was written by an earlier flush (no
// producer, level -1 for the level rule).

struct Unit {   // a transform cell before sorting
    Dav1dGpuUnit u;
    Dav1dGpuIntraEdge rec;
    int level;
    int sortmode;
    int32_t aux;   // aux_pool offset (INTER_MASK / PAL), else 0
};

// what the level pass needs of a cell (its geometry in 4x4 units, the edge
// needs of its remapped mode, the tile end) and which of its offsets are
// part-local until the parts are joined
struct LvJob {
    int16_t x4, y4, W4, H4;
    uint8_t p, cw4, ch4, nd, fl, fix;
    int32_t link;   // IIRES: its block's inter-intra prediction cell (part-local until the join)
    enum { HL = 1, HT = 2, TR = 4, BL = 8, CFL = 16, IIRES = 32, IIC = 64 };
};

// one thread's run of blocks, cut into cells with part-local offsets
struct CellPart {
    enum { F_AUX = 1, F_EDGE = 2, F_EMU0 = 4, F_EMU1 = 8, F_IIREC = 16 };
    std::vector<Unit> cells;
    std::vector<LvJob> jobs;
    std::vector<uint8_t> auxp;
    std::vector<EmuJob> emu;
    std::vector<Dav1dGpuUnit> xunits;
    std::vector<int32_t> xaux;
    std::vector<uint8_t> xfix;       // per launch-ahead unit: F_EMU0 / F_EMU1 (part-local src_off)
    std::vector<int32_t> emu_auxfix; // aux_pool offsets of int32 part-local scratch offsets (OBMC / scaled)
    int32_t emu_rows = 0;
    size_t edge_px = 0, n_res_used = 0;
    int32_t wm_off = -1, wm_w = 0, wm_h = 0;   // the last INTER_WMASK block's seg mask (4:2:0)
    int err = 0;
    void clear() {
        cells.clear();
        jobs.clear();
        auxp.clear();
        emu.clear();
        xunits.clear();
        xaux.clear();
        xfix.clear();
        emu_auxfix.clear();
        emu_rows = 0;
        edge_px = n_res_used = 0;
        wm_off = -1;
        wm_w = wm_h = 0;
        err = 0;
    }
    int32_t aux_alloc(size_t nbytes) {   // 16-byte aligned records
        const size_t o = (auxp.size() + 15) & ~(size_t)15;
        auxp.resize(o + nbytes);
        return (int32_t)o;
    }
    // a clamped copy of the fw x fh footprint at (x0, y0) of ref slot / plane
    // in a band of new scratch rows; returns its part-local scratch offset
    int32_t emu_band(int x0, int y0, int fw, int fh, int slot, int plane) {
        const int32_t o = emu_rows * kEmuStride;
        emu.push_back(EmuJob{x0, y0, o, (uint8_t)fw, (uint8_t)fh, (uint8_t)slot, (uint8_t)plane});
        emu_rows += fh;
        return o;
    }
};

// kinds recorded with block data (dav1d_gpu_rec_block_aux); the last four
// are predicted by the launch ahead of the wavefront
inline bool is_ext_kind(int k) {
    return k == DGPU_PRED_INTER_MASK || k == DGPU_PRED_PAL || k == DGPU_PRED_WARP || k == DGPU_PRED_INTER_WMASK ||
           k == DGPU_PRED_INTER_OBMC || k == DGPU_PRED_INTER_SCALED || k == DGPU_PRED_INTER_INTRA;
}
inline bool is_prelaunch_kind(int k) {
    return k == DGPU_PRED_WARP || k == DGPU_PRED_INTER_WMASK || k == DGPU_PRED_INTER_OBMC ||
           k == DGPU_PRED_INTER_SCALED;
}
inline bool is_mc_kind(int k) {   // the flow kinds that read references through src_off
    return k == DGPU_PRED_INTER || k == DGPU_PRED_INTER_AVG || k == DGPU_PRED_INTER_WAVG ||
           k == DGPU_PRED_INTER_MASK;
}
inline int tx_of(int w, int h) {
    for (int t = 0; t < DGPU_N_RECT_TX_SIZES; t++)
        if (kTx[t].w == w && kTx[t].h == h) return t;
    return -1;
}

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
              sizeof(ScaledUnitRef) == 16, "aux record layouts");

}  // namespace

struct Dav1dGpuRecorder {
    int bpc, bdmax, width, height, device;
    std::vector<Dav1dGpuRecBlock> blocks;
    std::vector<int64_t> block_aux;   // per block: offset into baux, -1 none
    std::vector<uint8_t> baux;        // dav1d_gpu_rec_block_aux data
    std::vector<Residual> residuals;
    std::vector<uint8_t> coefb;    // compact regions in the ABI's coefficient type (int16 / int32)
    // flush products (kept alive while the device may still read them)
    std::vector<int32_t> unit_start, class_start, rec_start, run_start;
    std::vector<Unit> cells;
    std::vector<LvJob> jobs;
    std::vector<CellPart> parts;
    std::unique_ptr<Pool> pool;   // host workers of the flush's parallel steps
    std::vector<uint64_t> keys, keys_tmp;
    std::vector<int32_t> rank;
    std::vector<int32_t> prod_start, prod, dep_start, deps;   // producers: decode order, then level order
    std::vector<EmuJob> emu;     // clamped footprint copies of this flush
    std::vector<uint8_t> auxp;   // the aux pool: masks, palette / warp / OBMC / scaled records
    std::vector<Dav1dGpuUnit> xunits;   // the launch ahead of the wavefront (class order)
    std::vector<int32_t> xaux;
    std::vector<Dav1dGpuEdgeBackup> bk;   // backup runs of launch-ahead predictions (top_edge)
    std::vector<uint8_t> h_host;   // DAV1D_GPU_REC_HOSTONLY: stands in for the pinned buffer
    // per-4x4 maps kept across flushes (generation-stamped): the residual
    // recorded at each cell (index + res_base) and its writer (cell_base + cell)
    std::vector<int32_t> res_at[3];
    std::vector<int32_t> own[3];
    std::vector<int32_t> lv;                 // per decode-order cell: its level
    std::vector<int32_t> prod_cnt;           // per decode-order cell: its producer count
    std::vector<std::vector<int32_t>> tprod; // producers found by each worker (its cell range)
    int32_t map_w4[3] = {0, 0, 0}, map_h4[3] = {0, 0, 0};
    int32_t res_base = 0, cell_base = 0;
    PinnedBuf pin;   // units | recs | coefficients | emu jobs, written in place by the fill
    PinnedBuf flag;  // the last flush's wavefront error word, copied back on its stream
    DevBuf d_units, d_recs, d_coef, d_edges, d_work, d_emu, d_emu_jobs, d_aux, d_auxp, d_xunits, d_xaux, d_bk;
    // dav1d_gpu_recorder_set_top_edge: the caller's f->ipred_edge planes
    // (superblock-top rows read from and backed up to them), luma superblock log2
    Dav1dGpuPlane top[3] = {};
    bool top_on = false;
    int sb_log2 = 6;
    hipEvent_t done = nullptr;
    bool pending_check = false;   // the last flush's error word not read yet
    int32_t last_units = 0, last_levels = 0;
};

// recorders alive in the process: a decoder with frame threads owns one per
// frame, and each sizes its worker pool to its share of the CPUs the process
// may run on (four recorders of 8 workers each oversubscribed
// the host)
static std::atomic<int> g_live_recorders{0};
static int rec_cpu_budget() {
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) return std::max(1, CPU_COUNT(&set));
    return (int)std::max(1u, std::thread::hardware_concurrency());
}

extern "C" Dav1dGpuRecorder *dav1d_gpu_recorder_new(int bpc, int bitdepth_max, int width, int height, int device) {
    if ((bpc != 8 && bpc != 16) || width <= 0 || height <= 0) return nullptr;
    g_live_recorders.fetch_add(1, std::memory_order_relaxed);
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
    g_live_recorders.fetch_sub(1, std::memory_order_relaxed);
    if (hipSetDevice(r->device) == hipSuccess) {
        if (r->done) {
            (void)hipEventSynchronize(r->done);
            (void)hipEventDestroy(r->done);
        }
        r->pin.release();
        r->flag.release();
        r->d_units.release();
        r->d_recs.release();
        r->d_coef.release();
        r->d_edges.release();
        r->d_work.release();
        r->d_emu.release();
        r->d_emu_jobs.release();
        r->d_aux.release();
        r->d_auxp.release();
        r->d_xunits.release();
        r->d_xaux.release();
        r->d_bk.release();
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
constexpr int kMapPad4 = 32;   // 4x4 cells past the grid a transform block can reach (128 px)

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
    const TxDim t = kTx[b->tx];
    if (b->x < 0 || b->y < 0 || b->w <= 0 || b->h <= 0 || b->x >= pw || b->y >= ph || b->w > 128 || b->h > 128)
        return -1;
    if ((b->x & 3) || (b->y & 3) || b->w % t.w || b->h % t.h) return -1;
    if (ext != is_ext_kind(b->kind)) return -1;
    const bool inter = b->kind == DGPU_PRED_INTER || b->kind == DGPU_PRED_INTER_AVG ||
                       b->kind == DGPU_PRED_INTER_WAVG || (ext && b->kind != DGPU_PRED_PAL);
    if (!inter && b->kind != DGPU_PRED_INTRA && b->kind != DGPU_PRED_CFL && b->kind != DGPU_PRED_PAL) return -1;
    if (b->kind == DGPU_PRED_CFL && (b->plane == 0 || b->w != t.w || b->h != t.h || t.w != t.h || t.w > 32))
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

extern "C" int dav1d_gpu_rec_block(Dav1dGpuRecorder *r, const Dav1dGpuRecBlock *b) {
    if (check_block(r, b, false)) return -1;
    r->blocks.push_back(*b);
    r->block_aux.push_back(-1);
    return 0;
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
            r->blocks.push_back(*b);
            r->block_aux.push_back(-1);
            return 0;
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
    case DGPU_PRED_INTER_WMASK:
        if (b->plane != 0 || b->weight > 1) return -1;
        r->blocks.push_back(*b);
        r->block_aux.push_back(-1);
        return 0;
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
    r->blocks.push_back(*b);
    r->block_aux.push_back((int64_t)r->baux.size());
    r->baux.insert(r->baux.end(), (const uint8_t *)aux, (const uint8_t *)aux + aux_bytes);
    return 0;
}

extern "C" int dav1d_gpu_rec_residual(Dav1dGpuRecorder *r, int plane, int x, int y, int tx, int txtp, int eob,
                                      const void *coef) {
    int pw, ph;
    if (!r || !coef || !plane_dims(r, plane, pw, ph) || tx < 0 || tx >= DGPU_N_RECT_TX_SIZES) return -1;
    if (txtp < 0 || txtp >= DGPU_N_TX_TYPES_PLUS_LL || eob < 0) return -1;
    const TxDim t = kTx[tx];
    if (x < 0 || y < 0 || x >= pw || y >= ph || (x & 3) || (y & 3)) return -1;   // starts inside the grid
    const int sw = std::min(t.w, 32), sh = std::min(t.h, 32);
    const size_t cb = r->bpc == 8 ? 2 : 4;
    Residual res{plane, x, y, tx, txtp, 0, 0, r->coefb.size() / cb};
    auto at = [&](int cx, int cy) -> int32_t {   // the reference's layout: coef[cy + cx * sh]
        return r->bpc == 8 ? ((const int16_t *)coef)[cy + cx * sh] : ((const int32_t *)coef)[cy + cx * sh];
    };
    auto put = [&](int cx, int cy) {   // appended in the ABI's coefficient type
        const size_t o = r->coefb.size();
        r->coefb.resize(o + cb);
        memcpy(&r->coefb[o], (const uint8_t *)coef + (size_t)(cy + cx * sh) * cb, cb);
    };
    if (eob == 0 && txtp == DGPU_DCT_DCT) {   // the DC-only call (src/itx_tmpl.c:53)
        put(0, 0);
    } else {   // the stored region: the bounding box of the non-zero coefficients
        int nzw = 1, nzh = 1;
        for (int cx = 0; cx < sw; cx++)
            for (int cy = 0; cy < sh; cy++)
                if (at(cx, cy)) {
                    nzw = std::max(nzw, cx + 1);
                    nzh = std::max(nzh, cy + 1);
                }
        res.nzw = nzw;
        res.nzh = nzh;
        for (int cx = 0; cx < nzw; cx++)
            for (int cy = 0; cy < nzh; cy++) put(cx, cy);
    }
    r->residuals.push_back(res);
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
    return *(volatile int32_t *)r->flag.p ? -6 : 0;
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

extern "C" int dav1d_gpu_recorder_flush(Dav1dGpuRecorder *r, const Dav1dGpuPlane dst[3],
                                        const Dav1dGpuPlane ref[DGPU_MAX_REFS][3], void *stream) {
    constexpr int NC = DGPU_N_RECT_TX_SIZES;
    if (!r || !dst) return -1;
    // DAV1D_GPU_REC_HOSTONLY=1 (diagnostics, no device needed): run the host
    // phases only and drop the recording before the upload
    static const bool host_only = getenv("DAV1D_GPU_REC_HOSTONLY") != nullptr;
    if (!host_only) {
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
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto t_0 = now();
    auto lap = [&](const char *what) {
        if (!timing) return;
        const auto t = now();
        fprintf(stderr, "recorder %-8s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t_0).count());
        t_0 = t;
    };
    const int bpp = r->bpc / 8;
    int pw[3], ph[3];
    for (int p = 0; p < 3; p++) plane_dims(r, p, pw[p], ph[p]);

    // per-4x4 maps over the grid plus the overhang transform blocks can reach
    int mw[3], mh[3];
    for (int p = 0; p < 3; p++) {
        mw[p] = pw[p] / 4 + kMapPad4;
        mh[p] = ph[p] / 4 + kMapPad4;
    }
    // the maps, kept across flushes; cleared only when their size changes or
    // the stamps would overflow
    size_t ncells = 0;   // an upper bound of this flush's cells (an inter-intra block adds one)
    for (const Dav1dGpuRecBlock &b : r->blocks) ncells += (size_t)(b.w / kTx[b.tx].w) * (b.h / kTx[b.tx].h) + 1;
    {
        bool reset = (int64_t)r->res_base + (int64_t)r->residuals.size() >= INT32_MAX ||
                     (int64_t)r->cell_base + (int64_t)ncells >= INT32_MAX;
        for (int p = 0; p < 3; p++) reset |= r->map_w4[p] != mw[p] || r->map_h4[p] != mh[p];
        if (reset) {
            for (int p = 0; p < 3; p++) {
                r->res_at[p].assign((size_t)mw[p] * mh[p], -1);
                r->own[p].assign((size_t)mw[p] * mh[p], -1);
                r->map_w4[p] = mw[p];
                r->map_h4[p] = mh[p];
            }
            r->res_base = r->cell_base = 0;
        }
    }
    const int32_t res_base = r->res_base, cell_base = r->cell_base;
    // the stamps of this flush, whatever its outcome, are below the next one's
    r->res_base += (int32_t)r->residuals.size();
    r->cell_base += (int32_t)ncells;
    // residual lookup: per plane, the top-left 4x4 cell of each residual
    std::vector<int32_t> *res_at = r->res_at;
    for (size_t i = 0; i < r->residuals.size(); i++) {
        const Residual &q = r->residuals[i];
        res_at[q.plane][(size_t)(q.y / 4) * mw[q.plane] + q.x / 4] = res_base + (int32_t)i;
    }

    // 1-3. transform units in decode order, their edge records and levels.
    //    The blocks are cut into cells by up to 8 threads, each over a run of
    //    blocks into its own part (cells, aux pool, emu jobs, launch-ahead
    //    units, with part-local offsets); the parts are then joined in
    //    decode order, their offsets rebased (which gives exactly the
    //    sequential layout), and one sequential pass assigns the levels and
    //    producers, which follow decode order.
    std::vector<Unit> &cells = r->cells;
    lap("maps");
    std::vector<int32_t> &prod_start = r->prod_start, &prod = r->prod;
    std::vector<uint8_t> &auxp = r->auxp;
    std::vector<Dav1dGpuUnit> &xunits = r->xunits;
    std::vector<int32_t> &xaux = r->xaux;
    // superblock height log2 per plane (4:2:0), and the TOP_SB_EDGE flag of an
    // edge record whose top row is a superblock's top (per transform block,
    // recon_tmpl.c:1276 / :1395; inter-intra per block, :1665 / :1794)
    const int sbl[3] = {r->sb_log2, r->sb_log2 - 1, r->sb_log2 - 1};
    auto top_sb = [&](int p, int y, bool ht) {
        return r->top_on && ht && (y & ((1 << sbl[p]) - 1)) == 0 ? DGPU_IE_TOP_SB_EDGE : 0;
    };
    auto build = [&](size_t bi, CellPart &P) -> int {
        const Dav1dGpuRecBlock &b = r->blocks[bi];
        const TxDim t = kTx[b.tx];
        const int p = b.plane, w4p = mw[p];
        // the part of the block the decoder iterates: w4 / h4 clipped to the
        // grid (recon_tmpl.c:1208); transform blocks start inside it
        const bool inter = is_mc_kind(b.kind);
        const bool cfl = b.kind == DGPU_PRED_CFL, pal = b.kind == DGPU_PRED_PAL;
        const bool pre = is_prelaunch_kind(b.kind);
        const uint8_t *bdata = r->block_aux[bi] >= 0 ? &r->baux[(size_t)r->block_aux[bi]] : nullptr;
        const int bw4 = b.w / 4, bh4 = b.h / 4, tw4 = t.w / 4, th4 = t.h / 4;
        const int bwc = std::min(b.w, pw[p] - b.x), bhc = std::min(b.h, ph[p] - b.y);
        const int bw4c = bwc / 4, bh4c = bhc / 4;
        const int ds_px = (int)(dst[p].stride / bpp);
        // every reference an inter block reads must be given
        if (inter || pre) {
            const int nref = b.kind == DGPU_PRED_INTER || b.kind == DGPU_PRED_WARP || b.kind == DGPU_PRED_INTER_OBMC ? 1
                             : b.kind == DGPU_PRED_INTER_SCALED ? *(const int32_t *)bdata : 2;
            for (int k = 0; k < nref; k++)
                if (!ref || !ref[b.ref[k]][p].data) return -1;
        }
        int32_t mask_base = 0, mask_stride = 0;   // INTER_MASK: the block's mask
        if (b.kind == DGPU_PRED_INTER_MASK) {
            if (bdata) {
                mask_base = P.aux_alloc((size_t)b.w * b.h);
                memcpy(&P.auxp[mask_base], bdata, (size_t)b.w * b.h);
                mask_stride = b.w;
            } else {   // COMPOUND_SEG chroma: the luma block's w_mask output
                if (P.wm_off < 0 || b.w != P.wm_w || b.h != P.wm_h) return -1;
                mask_base = P.wm_off;
                mask_stride = P.wm_w;
            }
        }
        if (pre) {   // prediction units of at most 32 x 32, no residual
            const int uw = std::min(b.w, 32), uh = std::min(b.h, 32), utx = tx_of(uw, uh);
            if (utx < 0) return -1;
            if (b.kind == DGPU_PRED_INTER_WMASK) {   // its seg mask at the 4:2:0 chroma resolution
                P.wm_w = b.w >> 1;
                P.wm_h = b.h >> 1;
                P.wm_off = P.aux_alloc((size_t)P.wm_w * P.wm_h);
            }
            // mc()'s emu_edge decision per prediction unit and reference
            // (src/recon_tmpl.c:986-999): the unit kernel reads a W+7 x H+7
            // footprint with aligned 16-byte row loads (up to 16 bytes past
            // it), so a direct read needs all of that inside the reference
            // picture, else the footprint is read from a clamped copy
            auto mc_inside = [&](int rr, int ix, int iy) {
                const int rw = ref[rr][p].w, rh = ref[rr][p].h;
                return ix - 3 >= 0 && iy - 3 >= 0 && ix + uw + 4 <= rw && iy + uh + 4 <= rh &&
                       (iy + uh + 4 < rh || (int64_t)(ix + uw + 4) * bpp + 16 <= ref[rr][p].stride);
            };
            auto mc_emu = [&](int rr, int ix, int iy) {   // the copy's (0, 0) pixel offset
                return P.emu_band(ix - 3, iy - 3, uw + 7, uh + 7, rr, p) + 3 * kEmuStride + 3;
            };
            for (int oy = 0; oy < bhc; oy += uh)
                for (int ox = 0; ox < bwc; ox += uw) {
                    const int ux = b.x + ox, uy = b.y + oy;
                    uint8_t xf = 0;   // CellPart::F_EMU0 / F_EMU1: src_off[k] is a part-local scratch offset
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
                        const int rs = ref && ref[rr][p].data ? (int)(ref[rr][p].stride / bpp) : 0;
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
                            xf |= k ? CellPart::F_EMU1 : CellPart::F_EMU0;
                        }
                    }
                    int32_t ao = 0;
                    if (b.kind == DGPU_PRED_INTER_WMASK) {
                        ao = P.wm_off + (oy >> 1) * P.wm_w + (ox >> 1);
                    } else if (b.kind == DGPU_PRED_WARP) {   // abcd, then the unit's 8x8s
                        const int gw = b.w / 8, nx = uw / 8, ny = uh / 8;
                        ao = P.aux_alloc(16 + 8 * (size_t)nx * ny);
                        memcpy(&P.auxp[ao], bdata, 8);
                        for (int sy = 0; sy < ny; sy++)
                            memcpy(&P.auxp[ao + 16 + 8 * sy * nx], bdata + 16 + 8 * ((oy / 8 + sy) * gw + ox / 8), 8 * nx);
                        // warp_affine's emu_edge (src/recon_tmpl.c:1168-1177): an
                        // 8x8 reads 15 x 15 pixels at (x - 3, y - 3); the kernel's
                        // aligned loads reach 16 bytes past column x + 11.  When
                        // any 8x8 of the unit leaves the picture, every 8x8 of it
                        // is read from a clamped copy (exact for the ones inside):
                        // 15-row strips, 8x8s 16 px apart, positions rewritten to
                        // the copy and the strip base in src_off[0] (the kernel
                        // adds it); otherwise src_off[0] = 0
                        const int rr = b.ref[0], rw = ref[rr][p].w, rh = ref[rr][p].h;
                        bool all_in = true;
                        for (int i = 0; i < nx * ny && all_in; i++) {
                            int16_t xy[2];
                            memcpy(xy, &P.auxp[ao + 16 + 8 * i], 4);
                            all_in = xy[0] - 3 >= 0 && xy[1] - 3 >= 0 && xy[0] + 12 <= rw && xy[1] + 12 <= rh &&
                                     (xy[1] + 12 < rh || (int64_t)(xy[0] + 12) * bpp + 16 <= ref[rr][p].stride);
                        }
                        u.p.inter.src_off[0] = 0;
                        if (!all_in) {
                            const int32_t band = P.emu_rows * kEmuStride;
                            for (int sy = 0; sy < ny; sy++)
                                for (int sx = 0; sx < nx; sx++) {
                                    uint8_t *e8 = &P.auxp[ao + 16 + 8 * (sy * nx + sx)];
                                    int16_t xy[2];
                                    memcpy(xy, e8, 4);
                                    P.emu.push_back(EmuJob{xy[0] - 3, xy[1] - 3, band + 15 * sy * kEmuStride + 16 * sx, 15, 15,
                                                           (uint8_t)rr, (uint8_t)p});
                                    const int16_t nxy[2] = {(int16_t)(16 * sx + 3), (int16_t)(15 * sy + 3)};
                                    memcpy(e8, nxy, 4);
                                }
                            P.emu_rows += 15 * ny;
                            u.p.inter.src_off[0] = band;
                            u.p.inter.ref[0] = (uint8_t)DGPU_REC_EMU_SLOT;
                            xf |= CellPart::F_EMU0;
                        }
                    } else if (b.kind == DGPU_PRED_INTER_OBMC) {   // the laps overlapping the unit
                        const int n = *(const int32_t *)bdata;
                        const ObmcBlockLap *lb = (const ObmcBlockLap *)(bdata + 16);
                        std::vector<ObmcUnitLap> ents;
                        std::vector<int> emu_ents;   // laps read through the scratch (the lap's
                                                     // prediction reads the unit's whole footprint)
                        for (int k = 0; k < n; k++) {
                            const ObmcBlockLap &e = lb[k];
                            const int x0 = std::max((int)e.x0 - ox, 0), x1 = std::min((int)e.x1 - ox, uw);
                            const int y0 = std::max((int)e.y0 - oy, 0), y1 = std::min((int)e.y1 - oy, uh);
                            if (x0 >= x1 || y0 >= y1) continue;
                            if (e.ref >= DGPU_REC_EMU_SLOT || !ref || !ref[e.ref][p].data || e.filter2d > 9) return -1;
                            const int rs = (int)(ref[e.ref][p].stride / bpp);
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
                            if (!mc_inside(e.ref, ix, iy)) {
                                q.src_off = mc_emu(e.ref, ix, iy);
                                q.ref = (uint8_t)DGPU_REC_EMU_SLOT;
                                emu_ents.push_back((int)ents.size());
                            }
                            ents.push_back(q);
                        }
                        ao = P.aux_alloc(16 + 16 * ents.size());
                        const int32_t ne = (int32_t)ents.size();
                        memset(&P.auxp[ao], 0, 16);
                        memcpy(&P.auxp[ao], &ne, 4);
                        if (ne) memcpy(&P.auxp[ao + 16], ents.data(), 16 * ents.size());
                        for (const int k : emu_ents) P.emu_auxfix.push_back(ao + 16 + 16 * k);   // (src_off first)
                    } else {   // INTER_SCALED: the unit's integer position and phase (running sums)
                        const int n = *(const int32_t *)bdata;
                        const ScaledBlockRef *sb = (const ScaledBlockRef *)(bdata + 16);
                        ao = P.aux_alloc(16 + 16 * (size_t)n);
                        memset(&P.auxp[ao], 0, 16 + 16 * (size_t)n);
                        memcpy(&P.auxp[ao], &n, 4);
                        for (int k = 0; k < n; k++) {
                            const int rr = b.ref[k];
                            const int rs = (int)(ref[rr][p].stride / bpp);
                            const int px_ = sb[k].mx + ox * sb[k].dx, py_ = sb[k].my + oy * sb[k].dy;
                            const int ix = sb[k].x + (px_ >> 10), iy = sb[k].y + (py_ >> 10);
                            ScaledUnitRef q;
                            q.src_off = iy * rs + ix;
                            q.mx = (uint16_t)(px_ & 1023), q.my = (uint16_t)(py_ & 1023);
                            q.dx = sb[k].dx, q.dy = sb[k].dy;
                            q.pad_ = 0;
                            // the scaled mc()'s emu_edge (src/recon_tmpl.c:1036-1046): the
                            // kernel reads columns ix - 3 .. ((mx + (W - 1) dx) >> 10) + 4
                            // past ix and rows iy - 3 .. ((my + (H - 1) dy) >> 10) + 4 past iy
                            // (its row count capped at 2H + 8), pixel by pixel
                            const int fw = ((q.mx + (uw - 1) * q.dx) >> 10) + 8;
                            const int fh = std::min(((q.my + (uh - 1) * q.dy) >> 10) + 8, 2 * uh + 8);
                            if (ix - 3 < 0 || iy - 3 < 0 || ix - 3 + fw > ref[rr][p].w || iy - 3 + fh > ref[rr][p].h) {
                                q.src_off = P.emu_band(ix - 3, iy - 3, fw, fh, rr, p) + 3 * kEmuStride + 3;
                                u.p.inter.ref[k] = (uint8_t)DGPU_REC_EMU_SLOT;
                                P.emu_auxfix.push_back(ao + 16 + 16 * k);
                            }
                            memcpy(&P.auxp[ao + 16 + 16 * k], &q, 16);
                        }
                        if (n == 1) u.p.inter.weight = 0;
                    }
                    P.xunits.push_back(u);
                    P.xaux.push_back(ao);
                    P.xfix.push_back(xf);
                }
        }
        // the transform cells; an INTER_INTRA block first gets one cell for
        // the whole block's prediction (recon_b_inter predicts the block,
        // :1540-1580, then adds the residuals), its transform cells become
        // residual-only cells that read it
        const bool iib = b.kind == DGPU_PRED_INTER_INTRA;
        const int ncx = (bwc + t.w - 1) / t.w, ncy = (bhc + t.h - 1) / t.h;
        const int32_t iic_at = (int32_t)P.cells.size();   // the inter-intra block's prediction cell
        for (int k = iib ? -1 : 0; k < ncx * ncy; k++)
            {
                const bool iic = k < 0;
                const int ox = iic ? 0 : (k % ncx) * t.w, oy = iic ? 0 : (k / ncx) * t.h;
                const int ctw = iic ? b.w : t.w, cth = iic ? b.h : t.h, ctw4 = ctw / 4, cth4 = cth / 4;
                P.cells.emplace_back();   // built in place (popped again when skipped)
                Unit &c = P.cells.back();
                memset(&c, 0, sizeof(c));
                uint8_t fix = 0;   // the part-local offsets this cell holds (CellPart::F_*)
                const int ux = b.x + ox, uy = b.y + oy, x4 = ux / 4, y4 = uy / 4;
                Dav1dGpuUnit &u = c.u;
                u.dst_off = uy * ds_px + ux;
                u.tx = (uint8_t)(iic ? tx_of(b.w, b.h) : b.tx);
                u.plane = (uint8_t)p;
                u.pred = (uint8_t)((pre || (iib && !iic)) ? DGPU_PRED_NONE : b.kind);
                u.txtp = DGPU_NO_RESIDUAL;
                const int32_t rs_ = iic ? -1 : res_at[p][(size_t)y4 * w4p + x4];
                const int ri = rs_ >= res_base ? rs_ - res_base : -1;   // (an earlier flush's: none)
                if (ri >= 0 && r->residuals[ri].tx == b.tx) {
                    const Residual &q = r->residuals[ri];
                    u.txtp = (uint8_t)q.txtp;
                    u.nzw = (uint8_t)q.nzw;
                    u.nzh = (uint8_t)q.nzh;
                    u.coef_off = (int32_t)q.coef;   // pool offset fixed below
                    P.n_res_used++;
                } else if (ri >= 0) {
                    return -1;   // a residual whose size differs from its block's transforms
                } else if (pre || (iib && !iic)) {
                    P.cells.pop_back();
                    continue;   // predicted elsewhere, nothing to add
                }
                Dav1dGpuIntraEdge &e = c.rec;
                e.unit = -1;
                e.x4 = (int16_t)x4;
                e.y4 = (int16_t)y4;
                e.w4 = (int16_t)(b.tile_x1 / 4);
                e.h4 = (int16_t)(b.tile_y1 / 4);
                int nd = 0;
                bool hl = ux > b.tile_x0, ht = uy > b.tile_y0;
                if (pre || (iib && !iic)) {   // PRED_NONE: the residual onto the prediction
                    c.sortmode = 0;
                } else if (pal) {   // pal_pred: palette, then the unit's rows of the index map
                    const int bw2 = b.w / 2;
                    c.aux = P.aux_alloc(16 + (size_t)(t.w / 2) * t.h);
                    fix |= CellPart::F_AUX;
                    memset(&P.auxp[c.aux], 0, 16);
                    memcpy(&P.auxp[c.aux], bdata, 8 * (size_t)bpp);
                    for (int yy = 0; yy < t.h; yy++)
                        memcpy(&P.auxp[c.aux + 16 + yy * (t.w / 2)], bdata + 8 * bpp + (size_t)(oy + yy) * bw2 + ox / 2,
                               t.w / 2);
                    c.sortmode = 15;
                } else if (inter || iic) {
                    u.bw4 = (uint8_t)bw4;
                    u.bh4 = (uint8_t)bh4;
                    for (int k = 0; k < 2; k++) {
                        const int rr = b.ref[k];
                        // every reference an inter block reads must be given
                        const bool used = k == 0 || (b.kind != DGPU_PRED_INTER && !iic);
                        if (used && (!ref || !ref[rr][p].data)) return -1;
                        const int rs = ref ? (int)(ref[rr][p].stride / bpp) : 0;
                        const int ix = ux + (b.mvx[k] >> 4), iy = uy + (b.mvy[k] >> 4);
                        u.p.inter.src_off[k] = iy * rs + ix;
                        u.p.inter.mx[k] = (uint8_t)(b.mvx[k] & 15);
                        u.p.inter.my[k] = (uint8_t)(b.mvy[k] & 15);
                        u.p.inter.ref[k] = (uint8_t)rr;
                        if (used) {
                            // the unit kernel reads the footprint with both
                            // 8-tap margins whatever the fraction, and its
                            // aligned row loads may run up to 16 bytes past
                            // the last pixel: direct only when all of that
                            // stays inside the picture, else a clamped copy
                            const int rw = ref[rr][p].w, rh = ref[rr][p].h;
                            const bool inside = ix - 3 >= 0 && iy - 3 >= 0 && ix + ctw + 4 <= rw &&
                                                iy + cth + 4 <= rh && (iy + cth + 4 < rh || (ix + ctw + 4) * bpp + 16 <= rs * bpp);
                            if (!inside) {
                                u.p.inter.src_off[k] = P.emu_band(ix - 3, iy - 3, ctw + 7, cth + 7, rr, p) + 3 * kEmuStride + 3;
                                fix |= k ? CellPart::F_EMU1 : CellPart::F_EMU0;
                                u.p.inter.ref[k] = (uint8_t)DGPU_REC_EMU_SLOT;
                            }
                        }
                    }
                    u.p.inter.filter2d = b.filter2d;
                    u.p.inter.weight = b.kind == DGPU_PRED_INTER_WAVG ? b.weight : 0;
                    if (b.kind == DGPU_PRED_INTER_MASK) {
                        c.aux = mask_base + oy * mask_stride + ox;
                        fix |= CellPart::F_AUX;
                    }
                    c.sortmode = b.filter2d;
                    if (iic) {   // the intra half: edges gathered by the wavefront like an INTRA unit's
                        // record: edge_off (unused when gathered), mode, angle, then the mask offset
                        c.aux = P.aux_alloc(16 + (size_t)b.w * b.h);
                        fix |= CellPart::F_AUX | CellPart::F_IIREC;
                        const int32_t moff = c.aux + 16, zero = 0;
                        memset(&P.auxp[c.aux], 0, 16);
                        memcpy(&P.auxp[c.aux], &zero, 4);
                        P.auxp[c.aux + 4] = b.mode;
                        memcpy(&P.auxp[c.aux + 8], &moff, 4);
                        memcpy(&P.auxp[moff], bdata, (size_t)b.w * b.h);
                        // prepare_intra_edges with no edge flags, no edge filter, angle 0 (:1551-1566)
                        e.mode = b.mode;
                        e.angle = 0;
                        e.flags = (uint8_t)((hl ? DGPU_IE_HAVE_LEFT : 0) | (ht ? DGPU_IE_HAVE_TOP : 0) | top_sb(p, uy, ht));
                        const int m = remap_mode(e.mode, 0, hl, ht);
                        nd = kNeeds[m];
                        c.sortmode = 16 + m;
                    }
                } else {
                    int fl = (hl ? DGPU_IE_HAVE_LEFT : 0) | (ht ? DGPU_IE_HAVE_TOP : 0) | top_sb(p, uy, ht);
                    if (!cfl) {   // recon_tmpl.c:1252-1266 (blocks up to 64 wide: one 64x64 step)
                        const int x = ox / 4, y = oy / 4;
                        const bool sb_tr = b.flags & DGPU_IE_TOP_HAS_RIGHT, sb_bl = b.flags & DGPU_IE_LEFT_HAS_BOTTOM;
                        if (!((y > 0 || !sb_tr) && x + tw4 >= bw4c)) fl |= DGPU_IE_TOP_HAS_RIGHT;
                        if (!(x > 0 || (!sb_bl && y + th4 >= bh4c))) fl |= DGPU_IE_LEFT_HAS_BOTTOM;
                        fl |= b.flags & (DGPU_IE_FILTER_EDGE | DGPU_IE_SMOOTH);
                        e.mode = b.mode;
                        e.angle = b.angle;
                        u.p.intra.max_w = (uint16_t)(pw[p] - ux);
                        u.p.intra.max_h = (uint16_t)(ph[p] - uy);
                    } else {
                        e.mode = DGPU_DC_PRED;   // cfl_pred's DC source (:1395-1410)
                        e.angle = 0;
                        u.p.cfl.alpha = b.cfl_alpha;
                        u.p.cfl.pad_wh = b.mode;   // cfl_ac's w_pad | h_pad << 4 (:1372-1380)
                        u.p.cfl.luma_off = (2 * uy) * (int)(dst[0].stride / bpp) + 2 * ux;
                    }
                    e.flags = (uint8_t)fl;
                    u.p.intra.edge_off = (int32_t)(P.edge_px + 2 * t.h);   // CFL: the same field
                    P.edge_px += 2 * t.h + 2 * t.w + 1;
                    fix |= CellPart::F_EDGE;
                    const int m = remap_mode(e.mode, e.angle, hl, ht);
                    nd = kNeeds[m];
                    c.sortmode = 16 + m;
                }
                // the level pass (below) reads the cell's geometry and edge needs
                P.jobs.emplace_back();
                LvJob &j = P.jobs.back();
                j.x4 = (int16_t)x4;
                j.y4 = (int16_t)y4;
                j.W4 = e.w4;
                j.H4 = e.h4;
                j.p = (uint8_t)p;
                j.cw4 = (uint8_t)ctw4;
                j.ch4 = (uint8_t)cth4;
                j.nd = (uint8_t)nd;
                j.fl = (uint8_t)((hl ? LvJob::HL : 0) | (ht ? LvJob::HT : 0) |
                                 ((e.flags & DGPU_IE_TOP_HAS_RIGHT) ? LvJob::TR : 0) |
                                 ((e.flags & DGPU_IE_LEFT_HAS_BOTTOM) ? LvJob::BL : 0) | (cfl ? LvJob::CFL : 0) |
                                 ((iib && !iic) ? LvJob::IIRES : 0) | (iic ? LvJob::IIC : 0));
                j.fix = fix;
                j.link = iib && !iic ? iic_at : -1;
            }
        return 0;
    };

    {   // DAV1D_GPU_REC_THREADS (diagnostics): the worker count; default this
        // recorder's share of the process's CPUs, at most 8, taken from the
        // live recorders at EACH flush (a pool sized at the first
        // flush kept 8 workers when the other frame threads' recorders came
        // later); the pool is rebuilt between flushes when the share changes
        const int live = std::max(1, g_live_recorders.load(std::memory_order_relaxed));
        int nthr = std::max(1, std::min(8, rec_cpu_budget() / live));
        if (const char *e = getenv("DAV1D_GPU_REC_THREADS")) nthr = std::max(1, atoi(e));
        if (!r->pool || r->pool->size() != nthr) r->pool.reset(new Pool(nthr));
    }
    const size_t nb = r->blocks.size();
    const int nt = nb < 4096 ? 1 : r->pool->size();
    if (r->parts.size() < (size_t)nt) r->parts.resize(nt);
    std::vector<size_t> bcut(nt + 1, nb);   // part boundaries on luma blocks (a block's chroma stays with it)
    bcut[0] = 0;
    for (int t = 1; t < nt; t++) {
        size_t c = std::max(bcut[t - 1], nb * t / nt);
        while (c < nb && r->blocks[c].plane != 0) c++;
        bcut[t] = c;
    }
    auto run_part = [&](int t) {
        CellPart &P = r->parts[t];
        P.clear();
        P.cells.reserve((size_t)((double)ncells * (bcut[t + 1] - bcut[t]) / std::max<size_t>(nb, 1)) + 64);
        for (size_t bi = bcut[t]; bi < bcut[t + 1] && !P.err; bi++) P.err = build(bi, P);
    };
    r->pool->run(nt, run_part);
    lap("cut");
    // join: part bases (the aux pool keeps its 16-byte alignment rule)
    size_t n_cells = 0, n_x = 0, n_emu = 0, aux_end = 0, n_res_used = 0;
    std::vector<size_t> cb0(nt), xb0(nt), eb0(nt), ab0(nt), pb0(nt);
    std::vector<int32_t> erow0(nt);
    int64_t emu_rows64 = 0;
    size_t edge_px = 0;
    for (int t = 0; t < nt; t++) {
        const CellPart &P = r->parts[t];
        if (P.err) return P.err;
        cb0[t] = n_cells;
        xb0[t] = n_x;
        eb0[t] = n_emu;
        erow0[t] = (int32_t)std::min<int64_t>(emu_rows64, INT32_MAX);
        pb0[t] = edge_px;
        ab0[t] = P.auxp.empty() ? aux_end : (aux_end + 15) & ~(size_t)15;
        if (!P.auxp.empty()) aux_end = ab0[t] + P.auxp.size();
        n_cells += P.cells.size();
        n_x += P.xunits.size();
        n_emu += P.emu.size();
        emu_rows64 += P.emu_rows;
        edge_px += P.edge_px;
        n_res_used += P.n_res_used;
    }
    // every emulated-edge offset (a job's o0, a unit's src_off into the
    // scratch, the kernels' row * kEmuStride) is int32 pixels: a flush whose
    // scratch would pass 2^31 pixels fails instead of wrapping (a hostile
    // stream of all-compound, all-outside cells reaches that below the 2^21
    // cell limit).  The cut's part-local offsets may have wrapped
    // already; none of them is used past this point
    if ((emu_rows64 + 1) * kEmuStride + 256 > (int64_t)INT32_MAX) return -1;
    const int32_t emu_rows = (int32_t)emu_rows64;
    if (n_res_used != r->residuals.size()) return -1;   // a residual outside every block
    cells.resize(n_cells);
    r->jobs.resize(n_cells);
    auxp.resize(aux_end);
    r->emu.resize(n_emu);
    xunits.resize(n_x);
    xaux.resize(n_x);
    auto join_part = [&](int t) {
        const CellPart &P = r->parts[t];
        const int32_t ab = (int32_t)ab0[t], er = erow0[t], pb = (int32_t)pb0[t];
        if (!P.auxp.empty()) memcpy(&auxp[ab0[t]], P.auxp.data(), P.auxp.size());
        for (size_t i = 0; i < P.cells.size(); i++) {
            Unit c = P.cells[i];
            const uint8_t f = P.jobs[i].fix;
            if (f & CellPart::F_AUX) c.aux += ab;
            if (f & CellPart::F_EDGE) c.u.p.intra.edge_off += pb;
            if (f & CellPart::F_EMU0) c.u.p.inter.src_off[0] += er * kEmuStride;
            if (f & CellPart::F_EMU1) c.u.p.inter.src_off[1] += er * kEmuStride;
            if (f & CellPart::F_IIREC) {   // the inter-intra record's mask offset
                int32_t mo;
                memcpy(&mo, &auxp[(size_t)c.aux + 8], 4);
                mo += ab;
                memcpy(&auxp[(size_t)c.aux + 8], &mo, 4);
            }
            cells[cb0[t] + i] = c;
            LvJob j = P.jobs[i];
            if (j.link >= 0) j.link += (int32_t)cb0[t];
            r->jobs[cb0[t] + i] = j;
        }
        for (size_t i = 0; i < P.emu.size(); i++) {
            EmuJob e = P.emu[i];
            e.o0 += er * kEmuStride;
            r->emu[eb0[t] + i] = e;
        }
        for (size_t i = 0; i < P.xunits.size(); i++) {
            Dav1dGpuUnit u = P.xunits[i];
            if (P.xfix[i] & CellPart::F_EMU0) u.p.inter.src_off[0] += er * kEmuStride;
            if (P.xfix[i] & CellPart::F_EMU1) u.p.inter.src_off[1] += er * kEmuStride;
            xunits[xb0[t] + i] = u;
            xaux[xb0[t] + i] = P.xaux[i] + ab;
        }
        for (const int32_t o : P.emu_auxfix) {   // OBMC laps / scaled refs read through the scratch
            int32_t v;
            memcpy(&v, &auxp[(size_t)ab + o], 4);
            v += er * kEmuStride;
            memcpy(&auxp[(size_t)ab + o], &v, 4);
        }
    };
    r->pool->run(nt, join_part);
    lap("join");
    // levels and producers: a cell sits one level above every pixel its
    // edges (or CfL luma, or an inter-intra residual's prediction) read; its
    // producers are the cells that wrote them.  A pixel no cell of this flush
    // wrote came from an earlier flush on the same stream: no producer, level
    // 0 for it.  Three steps, the first two on the worker pool:
    //   1. every cell stamps its 4x4s in the writer map (the only overlap in a
    //      flush: an inter-intra block's prediction cell under its residual
    //      cells, which come after it in decode order and win);
    //   2. every cell looks its producers up (a writer at or after the cell in
    //      decode order has not written yet: none), sorted, duplicate-free;
    //   3. the levels in decode order, from the producers' (decode order is a
    //      topological order).
    const int nlv = n_cells < 32768 ? 1 : r->pool->size();
    {
        auto stamp = [&](size_t ci, bool iic_pass) {
            const LvJob &j = r->jobs[ci];
            const bool iic = j.fl & LvJob::IIC;
            if (iic != iic_pass) return;
            int32_t *wp = r->own[j.p].data();
            const int w4p = mw[j.p];
            const int32_t v = cell_base + (int32_t)ci;
            for (int cy = j.y4; cy < j.y4 + j.ch4; cy++)
                for (int cx = j.x4; cx < j.x4 + j.cw4; cx++) {
                    int32_t &o = wp[(size_t)cy * w4p + cx];
                    if (!iic_pass || o < cell_base) o = v;   // (under its residual cells: theirs)
                }
        };
        r->pool->run(nlv, [&](int t) {
            for (size_t ci = n_cells * t / nlv, e = n_cells * (t + 1) / nlv; ci < e; ci++) stamp(ci, false);
        });
        // the contract (include/dav1d_gpu.h, dav1d_gpu_recorder_flush): the
        // cells of one flush do not overlap, an inter-intra prediction under
        // its own residual cells excepted.  Checked after the parallel stamp:
        // two overlapping cells leave one stamp on a shared 4x4, so the other
        // finds a stamp not its own whatever order the workers ran in; the
        // flush then fails instead of scheduling reads before writes
        // 
        std::atomic<int> overlap{0};
        r->pool->run(nlv, [&](int t) {
            int bad = 0;
            for (size_t ci = n_cells * t / nlv, e = n_cells * (t + 1) / nlv; ci < e && !bad; ci++) {
                const LvJob &j = r->jobs[ci];
                if (j.fl & LvJob::IIC) continue;
                const int32_t *wp = r->own[j.p].data();
                const int w4p = mw[j.p];
                const int32_t v = cell_base + (int32_t)ci;
                for (int cy = j.y4; cy < j.y4 + j.ch4 && !bad; cy++)
                    for (int cx = j.x4; cx < j.x4 + j.cw4; cx++)
                        if (wp[(size_t)cy * w4p + cx] != v) {
                            bad = 1;
                            break;
                        }
            }
            if (bad) overlap.store(1, std::memory_order_relaxed);
        });
        if (overlap.load()) return -1;
        r->pool->run(nlv, [&](int t) {
            for (size_t ci = n_cells * t / nlv, e = n_cells * (t + 1) / nlv; ci < e; ci++) stamp(ci, true);
        });
    }
    lap("stamp");
    r->prod_cnt.resize(n_cells);
    if (r->tprod.size() < (size_t)nlv) r->tprod.resize(nlv);
    r->pool->run(nlv, [&](int t) {
        std::vector<int32_t> &out = r->tprod[t];
        out.clear();
        for (size_t ci = n_cells * t / nlv, e = n_cells * (t + 1) / nlv; ci < e; ci++) {
            const LvJob &j = r->jobs[ci];
            const int p = j.p, w4p = mw[p], x4 = j.x4, y4 = j.y4, cw4 = j.cw4, ch4 = j.ch4, W4 = j.W4, H4 = j.H4;
            const int nd = j.nd;
            const bool hl = j.fl & LvJob::HL, ht = j.fl & LvJob::HT;
            const int32_t *mp = r->own[p].data();
            const int32_t lo = cell_base, hi = cell_base + (int32_t)ci;   // this flush, before the cell
            const size_t p0 = out.size();
            auto put = [&](int32_t o) {
                if (o < lo || o >= hi) return;
                o -= cell_base;
                if (out.size() == p0 || out.back() != o) out.push_back(o);
            };
            auto cell = [&](int cx, int cy) { put(mp[(size_t)cy * w4p + cx]); };
            if (nd & 1) {
                if (hl) {
                    for (int q = y4; q < std::min(y4 + ch4, H4); q++) cell(x4 - 1, q);
                    if ((nd & 16) && y4 + ch4 < H4 && (j.fl & LvJob::BL))
                        for (int q = y4 + ch4; q < std::min(y4 + 2 * ch4, H4); q++) cell(x4 - 1, q);
                } else if (ht) {
                    cell(x4, y4 - 1);
                }
            }
            if (nd & 2) {
                if (ht) {
                    for (int q = x4; q < std::min(x4 + cw4, W4); q++) cell(q, y4 - 1);
                    if ((nd & 8) && x4 + cw4 < W4 && (j.fl & LvJob::TR))
                        for (int q = x4 + cw4; q < std::min(x4 + 2 * cw4, W4); q++) cell(q, y4 - 1);
                } else if (hl) {
                    cell(x4 - 1, y4);
                }
            }
            if (j.fl & LvJob::IIRES) put(cell_base + j.link);   // the block's inter-intra prediction
            if (nd & 4) {
                if (hl && ht) cell(x4 - 1, y4 - 1);
                else if (hl) cell(x4 - 1, y4);
                else if (ht) cell(x4, y4 - 1);
            }
            if (j.fl & LvJob::CFL) {
                const int lw4 = mw[0];
                const int32_t *ml = r->own[0].data();
                for (int cy = 2 * y4; cy < 2 * (y4 + ch4); cy++)
                    for (int cx = 2 * x4; cx < 2 * (x4 + cw4); cx++) put(ml[(size_t)cy * lw4 + cx]);
            }
            if (out.size() - p0 > 1) {   // sorted, duplicate-free (lists are short: insertion sort)
                int32_t *q = out.data() + p0;
                const size_t m = out.size() - p0;
                size_t u = 1;
                for (size_t a_ = 1; a_ < m; a_++) {
                    const int32_t v = q[a_];
                    size_t b_ = u;
                    while (b_ > 0 && q[b_ - 1] > v) b_--;
                    if (b_ > 0 && q[b_ - 1] == v) continue;   // a duplicate
                    for (size_t c_ = u; c_ > b_; c_--) q[c_] = q[c_ - 1];
                    q[b_] = v;
                    u++;
                }
                out.resize(p0 + u);
            }
            r->prod_cnt[ci] = (int32_t)(out.size() - p0);
        }
    });
    lap("prods");
    // the producer lists in decode order (CSR), then the levels
    prod_start.resize(n_cells + 1);
    prod_start[0] = 0;
    for (size_t ci = 0; ci < n_cells; ci++) prod_start[ci + 1] = prod_start[ci] + r->prod_cnt[ci];
    prod.resize((size_t)prod_start[n_cells]);
    r->pool->run(nlv, [&](int t) {
        const size_t c0 = n_cells * t / nlv;
        if (!r->tprod[t].empty()) memcpy(&prod[(size_t)prod_start[c0]], r->tprod[t].data(), r->tprod[t].size() * 4);
    });
    {   // (a compact level array: the walk touches 4 bytes per cell)
        r->lv.resize(n_cells);
        int32_t *lv = r->lv.data();
        const int32_t *ps = prod_start.data(), *pp = prod.data();
        for (size_t ci = 0; ci < n_cells; ci++) {
            int d = -1;
            for (int32_t k = ps[ci]; k < ps[ci + 1]; k++) d = std::max(d, lv[pp[k]]);
            lv[ci] = d + 1;
        }
        r->pool->run(nlv, [&](int t) {
            for (size_t ci = n_cells * t / nlv, e = n_cells * (t + 1) / nlv; ci < e; ci++) cells[ci].level = lv[ci];
        });
    }
    lap("levels");
    const int n = (int)cells.size();

    // 4. level order, size classes inside a level, then kind / mode / type:
    //    one LSD radix sort of (key << 21 | decode index) on the key bits only
    //    (stable: equal keys stay in decode order).  Key: level | tx (5) |
    //    pred (4) | mode (6) | type (5, NO_RESIDUAL last)
    if (n >= (1 << 21)) return -1;
    const int nthreads = r->pool->size();
    const int npar = n < 32768 ? 1 : nthreads;   // (the O(n) passes below on the pool)
    std::vector<uint64_t> &keys = r->keys;
    keys.resize(n);
    int max_level = 0;
    {
        std::vector<int> tmax(npar, 0);
        r->pool->run(npar, [&](int t) {
            int m = 0;
            for (int i = (int)((int64_t)n * t / npar), e = (int)((int64_t)n * (t + 1) / npar); i < e; i++) {
                const Unit &c = cells[i];
                m = std::max(m, c.level);
                const uint64_t key = (uint64_t)c.level << 20 | (uint64_t)c.u.tx << 15 | (uint64_t)c.u.pred << 11 |
                                     (uint64_t)(c.sortmode & 63) << 5 |
                                     (uint64_t)(c.u.txtp == DGPU_NO_RESIDUAL ? 31 : c.u.txtp);
                keys[i] = key << 21 | (uint64_t)i;
            }
            tmax[t] = m;
        });
        for (int t = 0; t < npar; t++) max_level = std::max(max_level, tmax[t]);
        if (max_level >= (1 << 16)) return -1;
    }
    {
        int lb = 0;
        while ((1 << lb) <= max_level) lb++;
        radix_sort(keys, r->keys_tmp, 21, 21 + 20 + lb, *r->pool);
    }
    lap("sort");
    const int n_levels = n ? max_level + 1 : 0;
    r->unit_start.assign(n_levels + 1, 0);
    r->class_start.assign((size_t)n_levels * (NC + 1), 0);
    const size_t cb = r->bpc == 8 ? 2 : 4;
    // the rank of every decode-order cell, and the level / class ranges: a
    // (level, class) run ends where the sorted key's top bits change
    std::vector<int32_t> &rank = r->rank;
    rank.resize(n);
    r->dep_start.assign((size_t)n + 1, 0);
    r->pool->run(npar, [&](int t) {
        for (int i = (int)((int64_t)n * t / npar), e = (int)((int64_t)n * (t + 1) / npar); i < e; i++) {
            const uint64_t k = keys[i];
            const int ci = (int)(k & ((1u << 21) - 1));
            rank[ci] = i;
            const uint64_t lt = k >> 36;   // level | tx
            if (i + 1 == n || (keys[i + 1] >> 36) != lt) {   // the last of its (level, class) run
                const int level = (int)(lt >> 5), tx = (int)(lt & 31);
                r->class_start[(size_t)level * (NC + 1) + tx + 1] = i + 1;   // an end, made a count below
                if (i + 1 == n || (int)(keys[i + 1] >> 41) != level) r->unit_start[level + 1] = i + 1;
            }
            r->dep_start[i + 1] = prod_start[ci + 1] - prod_start[ci];   // (producer lists in level order)
        }
    });
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
    }
    for (int i = 0; i < n; i++) r->dep_start[i + 1] += r->dep_start[i];
    r->deps.resize(prod.size());
    for (int l = 0; l < n_levels; l++) {
        if (r->unit_start[l + 1] < r->unit_start[l]) r->unit_start[l + 1] = r->unit_start[l];   // (levels are dense)
        int32_t *cs = &r->class_start[(size_t)l * (NC + 1)];
        for (int k = 0; k < NC; k++) cs[k + 1] += cs[k];
    }
    // 5. the upload image, written in place (page-locked, or a host vector
    //    for DAV1D_GPU_REC_HOSTONLY): units and records scattered to their
    //    ranks, the coefficient pool (decode order) and the emu jobs, by
    //    several threads over disjoint ranges
    const size_t coef_at = r->coefb.size() / cb;
    // image: units | records | coefficients | emu jobs | per-unit aux |
    //        launch-ahead units (class order) | their aux | aux pool
    const size_t nx = r->xunits.size();
    // with top_edge: the launch-ahead predictions whose bottom row ends a
    // superblock row are backed up once that launch is done (backup runs
    // between it and the wavefront, dav1d_backup_ipred_edge); a residual on
    // them is added by a wavefront unit, which backs its row up again
    std::vector<Dav1dGpuEdgeBackup> &bk = r->bk;
    bk.clear();
    if (r->top_on)
        for (const Dav1dGpuUnit &u : r->xunits) {
            const int p = u.plane, ds_px = (int)(dst[p].stride / bpp);
            const int uy = u.dst_off / ds_px, ux = u.dst_off % ds_px, y1 = uy + kTx[u.tx].h;
            const int sby = (y1 >> sbl[p]) - 1, w = std::min(kTx[u.tx].w, r->top[p].w - ux);
            if ((y1 & ((1 << sbl[p]) - 1)) == 0 && sby < r->top[p].h && w > 0)
                bk.push_back(Dav1dGpuEdgeBackup{p, sby, ux, w});
        }
    const size_t bu = (size_t)n * sizeof(Dav1dGpuUnit), br = (size_t)n * sizeof(Dav1dGpuIntraEdge),
                 bc = coef_at * cb, be = r->emu.size() * sizeof(EmuJob), ba = (size_t)n * 4,
                 bxu = nx * sizeof(Dav1dGpuUnit), bxa = nx * 4, bp = r->auxp.size(),
                 bbk = bk.size() * sizeof(Dav1dGpuEdgeBackup);
    const size_t o_c = bu + br, o_e = o_c + bc, o_a = o_e + be, o_xu = o_a + ba, o_xa = o_xu + bxu,
                 o_p = o_xa + bxa, o_bk = o_p + bp, o_end = o_bk + bbk;
    uint8_t *img;
    if (host_only) {
        r->h_host.resize(o_end);
        img = r->h_host.data();
    } else {
        if (r->pin.grow(o_end)) return -3;
        img = (uint8_t *)r->pin.p;
    }
    Dav1dGpuUnit *hu = (Dav1dGpuUnit *)img;
    Dav1dGpuIntraEdge *hr = (Dav1dGpuIntraEdge *)(img + bu);
    int32_t *ha = (int32_t *)(img + o_a);
    // the launch-ahead units in class order (a counting sort by size class)
    int32_t x_class[DGPU_N_RECT_TX_SIZES + 1] = {0};
    if (nx) {
        for (const Dav1dGpuUnit &u : r->xunits) x_class[u.tx + 1]++;
        for (int k = 0; k < NC; k++) x_class[k + 1] += x_class[k];
        int32_t at[DGPU_N_RECT_TX_SIZES];
        memcpy(at, x_class, sizeof(at));
        Dav1dGpuUnit *xu = (Dav1dGpuUnit *)(img + o_xu);
        int32_t *xa = (int32_t *)(img + o_xa);
        for (size_t i = 0; i < nx; i++) {
            const int k = at[r->xunits[i].tx]++;
            xu[k] = r->xunits[i];
            xa[k] = r->xaux[i];
        }
    }
    if (bp) memcpy(img + o_p, r->auxp.data(), bp);
    if (bbk) memcpy(img + o_bk, bk.data(), bbk);
    {   // in rank order: the image is written sequentially, the cells read by index
        const int nt = n < 32768 ? 1 : nthreads;
        int32_t *deps = r->deps.data();
        const int32_t *ds = r->dep_start.data();
        auto work = [&](int t) {
            const int i0 = (int)((int64_t)n * t / nt), i1 = (int)((int64_t)n * (t + 1) / nt);
            for (int i = i0; i < i1; i++) {
                const int ci = (int)(keys[i] & ((1u << 21) - 1));
                const Unit &c = cells[ci];
                hu[i] = c.u;   // coef_off / edge_off are decode-order pool offsets
                ha[i] = c.aux;
                Dav1dGpuIntraEdge e = c.rec;
                e.unit = i;
                hr[i] = e;
                int32_t *o = deps + ds[i];
                for (int k = prod_start[ci]; k < prod_start[ci + 1]; k++) *o++ = rank[prod[k]];
            }
            const size_t b0 = bc * t / nt, b1 = bc * (t + 1) / nt;
            if (b1 > b0) memcpy(img + o_c + b0, r->coefb.data() + b0, b1 - b0);
        };
        r->pool->run(nt, work);
        if (be) memcpy(img + o_e, r->emu.data(), be);
    }
    lap("fill");
    r->rec_start = r->unit_start;
    r->run_start.assign(n_levels + 1, 0);
    r->last_units = n;
    r->last_levels = n_levels;
    auto drop_recording = [&] {
        r->blocks.clear();
        r->block_aux.clear();
        r->baux.clear();
        r->residuals.clear();
        r->coefb.clear();
    };
    if ((!n && !nx) || host_only) {
        // DAV1D_GPU_REC_DUMP=<file> with DAV1D_GPU_REC_HOSTONLY (diagnostics):
        // the upload image and the schedule, appended, to compare host builds
        static const char *dump = getenv("DAV1D_GPU_REC_DUMP");
        if (host_only && dump) {
            if (FILE *f = fopen(dump, "ab")) {
                auto put = [&](const void *p, size_t nb) { if (nb) fwrite(p, 1, nb, f); };
                const int64_t hdr[4] = {n, n_levels, (int64_t)nx, (int64_t)o_end};
                put(hdr, sizeof(hdr));
                put(r->h_host.data(), o_end);
                put(r->unit_start.data(), r->unit_start.size() * 4);
                put(r->class_start.data(), r->class_start.size() * 4);
                put(r->dep_start.data(), r->dep_start.size() * 4);
                put(r->deps.data(), r->deps.size() * 4);
                put(x_class, sizeof(x_class));
                fclose(f);
            }
        }
        drop_recording();
        return 0;
    }

    // upload and launch
    hipStream_t st = (hipStream_t)stream;
    Dav1dGpuIntraSchedule s;
    memset(&s, 0, sizeof(s));
    s.n_levels = n_levels;
    s.flags = DGPU_IS_FUSED | DGPU_IS_PERSISTENT;
    s.unit_start = r->unit_start.data();
    s.class_start = r->class_start.data();
    s.rec_start = r->rec_start.data();
    s.run_start = r->run_start.data();
    s.dep_start = r->dep_start.data();
    s.deps = r->deps.data();
    const int64_t wsb = n ? dav1d_gpu_intra_workspace_bytes(&s, n) : 16;
    if (wsb < 0) return -2;
    if (r->d_units.grow((size_t)n * sizeof(Dav1dGpuUnit)) || r->d_recs.grow((size_t)n * sizeof(Dav1dGpuIntraEdge)) ||
        r->d_coef.grow(std::max<size_t>(coef_at * cb, 16)) || r->d_edges.grow(std::max<size_t>(edge_px * bpp, 16)) ||
        r->d_work.grow((size_t)wsb))
        return -3;
    if (be && (r->d_emu_jobs.grow(be) || r->d_emu.grow((size_t)emu_rows * kEmuStride * bpp + 256))) return -3;
    if (r->d_aux.grow(ba) || r->d_auxp.grow(std::max<size_t>(bp, 16)) ||
        (nx && (r->d_xunits.grow(bxu) || r->d_xaux.grow(bxa))) || (bbk && r->d_bk.grow(bbk)))
        return -3;
    const uint8_t *pin = img;
    // once a copy from the pinned image may be queued, a failure drains the
    // stream before returning: a retry rewrites that image and may regrow the
    // device buffers, which the queued copies and kernels still use
    auto drained = [&](int rc) {
        (void)hipStreamSynchronize(st);
        return rc;
    };
    if ((bu && hipMemcpyAsync(r->d_units.p, pin, bu, hipMemcpyHostToDevice, st)) ||
        (br && hipMemcpyAsync(r->d_recs.p, pin + bu, br, hipMemcpyHostToDevice, st)) ||
        (bc && hipMemcpyAsync(r->d_coef.p, pin + o_c, bc, hipMemcpyHostToDevice, st)) ||
        (be && hipMemcpyAsync(r->d_emu_jobs.p, pin + o_e, be, hipMemcpyHostToDevice, st)) ||
        (ba && hipMemcpyAsync(r->d_aux.p, pin + o_a, ba, hipMemcpyHostToDevice, st)) ||
        (nx && hipMemcpyAsync(r->d_xunits.p, pin + o_xu, bxu, hipMemcpyHostToDevice, st)) ||
        (nx && hipMemcpyAsync(r->d_xaux.p, pin + o_xa, bxa, hipMemcpyHostToDevice, st)) ||
        (bp && hipMemcpyAsync(r->d_auxp.p, pin + o_p, bp, hipMemcpyHostToDevice, st)) ||
        (bbk && hipMemcpyAsync(r->d_bk.p, pin + o_bk, bbk, hipMemcpyHostToDevice, st)))
        return drained(-3);
    if (be) {   // the clamped footprints, before the wavefront reads them
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
        ea.jobs = (const EmuJob *)r->d_emu_jobs.p;
        ea.n = (int32_t)r->emu.size();
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
        auto reg = [&](const void *p, size_t nb, int id) {
            if (p && nb) bx.push_back(dgpu::BndRange{p, (nb + 15) & ~(size_t)15, id});
        };
        reg(r->d_units.p, bu, dgpu::BND_UNITS);
        reg(r->d_recs.p, br, dgpu::BND_RECS);
        // DAV1D_GPU_BND_SELFTEST=1: register the coefficient pool 64 bytes
        // short, so the diagnostics must report the last units' coefficient
        // reads (the check's positive control)
        static const bool selftest = getenv("DAV1D_GPU_BND_SELFTEST") != nullptr;
        reg(r->d_coef.p, selftest && bc > 128 ? bc - 64 : bc, dgpu::BND_COEF);
        reg(r->d_edges.p, edge_px * bpp, dgpu::BND_EDGES);
        reg(r->d_aux.p, ba, dgpu::BND_AUX);
        reg(r->d_auxp.p, bp, dgpu::BND_AUXPOOL);
        reg(r->d_work.p, (size_t)wsb, dgpu::BND_WORK);
        if (be) reg(r->d_emu.p, (size_t)emu_rows * kEmuStride * bpp, dgpu::BND_EMU);
        if (nx) {
            reg(r->d_xunits.p, bxu, dgpu::BND_XUNITS);
            reg(r->d_xaux.p, bxa, dgpu::BND_XAUX);
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
        if (be) fb.ref[DGPU_REC_EMU_SLOT][p] = Dav1dGpuPlane{r->d_emu.p, (int64_t)kEmuStride * bpp, kEmuStride, emu_rows};
    }
    for (int p = 0; p < 3; p++) {
        eb.sb_log2[p] = sbl[p];
        if (r->top_on) eb.top_edge[p] = r->top[p];
    }
    fb.units = (const Dav1dGpuUnit *)r->d_units.p;
    fb.n_units = n;
    fb.class_start[NC] = n;
    fb.coef = r->d_coef.p;
    fb.edges = r->d_edges.p;
    fb.bitdepth_max = r->bdmax;
    fb.cfl_luma = dst[0];
    fb.cfl_ss = 3;
    fb.aux = (const int32_t *)r->d_aux.p;
    fb.aux_pool = r->d_auxp.p;
    if (nx) {   // WARP / INTER_WMASK / INTER_OBMC / INTER_SCALED predictions ahead of the wavefront
        Dav1dGpuFrameBatch xb = fb;
        xb.units = (const Dav1dGpuUnit *)r->d_xunits.p;
        xb.n_units = (int32_t)nx;
        for (int k = 0; k <= NC; k++) xb.class_start[k] = x_class[k];
        for (int k = 0; k < NC; k++) xb.class_warp[k] = x_class[k + 1] - x_class[k];
        xb.aux = (const int32_t *)r->d_xaux.p;
        const int xrc = r->bpc == 8 ? dav1d_gpu_recon_8bpc(&xb, stream) : dav1d_gpu_recon_16bpc(&xb, stream);
        if (xrc) return drained(xrc);
    }
    if (bbk) {   // their superblock-bottom rows into top_edge, before the wavefront
        const auto *runs = (const Dav1dGpuEdgeBackup *)r->d_bk.p;
        const int brc = r->bpc == 8 ? dav1d_gpu_backup_ipred_edge_8bpc(&eb, runs, (int)bk.size(), stream)
                                    : dav1d_gpu_backup_ipred_edge_16bpc(&eb, runs, (int)bk.size(), stream);
        if (brc) return drained(brc);
    }
    eb.units = (Dav1dGpuUnit *)r->d_units.p;
    eb.edges = r->d_edges.p;
    eb.recs = (const Dav1dGpuIntraEdge *)r->d_recs.p;
    eb.n_recs = n;
    eb.bitdepth_max = r->bdmax;
    lap("upload");
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
    if (n && (r->flag.grow(16) ||
              hipMemcpyAsync(r->flag.p, (const int32_t *)r->d_work.p + 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess))
        return drained(-3);
    if (hipEventRecord(r->done, st) != hipSuccess) return drained(-3);
    r->pending_check = n > 0;
    drop_recording();
    return 0;
}
