// recon_impl.hpp -- batch-tier launch logic (instantiated per bitdepth in
// recon8.hip / recon16.hip so the two heavy TUs compile in parallel).
//
// Three kernels per frame batch, one per class group (small: w*h <= 128,
// large: up to 32x32, huge: the 64-point sides), each with its own
// register and LDS budget.  Within a kernel the waves are scheduled (segment, class):
// every class's unit range (units are sorted by class and, within a class,
// by position) is cut into kSegments runs of equal wave count, so waves
// that run at the same time touch the same band of the picture.  Blocks are mapped so each
// XCD works through a contiguous run of bands: a picture line is then
// written by one XCD's L2 instead of partially by several.
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <type_traits>
#include <utility>

#include "recon_kernel.hpp"

namespace dgpu {


// waves per workgroup: waves never share LDS, so small workgroups only
// serve to pack the CU's LDS tightly (one wave for the 64-point classes)
template <int BPC, int GRP> __host__ __device__ constexpr int waves_per_block() {
    return base_group(GRP) == GROUP_HUGE ? 1 : 2;
}

// log2(lanes_per_unit) of every class packed 3 bits each into a constant
__host__ __device__ constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v >> 1); }
template <int... TX> constexpr uint64_t pack_log2_lanes(std::integer_sequence<int, TX...>) {
    uint64_t v = 0;
    ((v |= (uint64_t)ilog2c(lanes_per_unit(TX)) << (3 * TX)), ...);
    return v;
}
constexpr uint64_t kLog2Lanes = pack_log2_lanes(std::make_integer_sequence<int, DGPU_N_RECT_TX_SIZES>());

template <int BPC, int TX, int GRP, typename WaitT = NoWait>
__device__ __forceinline__ void run_class(const ReconArgs<BPC> &a, const PlaneTab<BPC> &pt, const Dav1dGpuUnit &u,
                                          const Dav1dGpuIntraEdge &rec, int first, int count, uint8_t *lds, int gw,
                                          const WaitT &wait = WaitT()) {
    if constexpr (TX < DGPU_N_RECT_TX_SIZES && in_group(TX, GRP)) {
        if constexpr (GRP == GROUP_WARP) {
            // the second launch: w_mask / OBMC / scaled units in their own
            // function, warp and inter-intra in recon_units (per unit: a wave
            // at the boundary of the two sorted runs holds both)
            const bool ext = u.pred == DGPU_PRED_INTER_WMASK || u.pred == DGPU_PRED_INTER_OBMC ||
                             u.pred == DGPU_PRED_INTER_SCALED;
            if (ext) recon_units_ext<BPC, TX>(a, pt, u, first, count, lds);
            else recon_units<BPC, TX, true, false>(a, pt, u, rec, first, count, lds, gw, GRP, wait);
        } else {
            recon_units<BPC, TX, false, gathers(GRP)>(a, pt, u, rec, first, count, lds, gw, GRP, wait);
        }
    }
}

// One switch (a compact compare tree) instead of a chain of class tests
// spread between the inlined class bodies: the chain's targets were cold
// instruction-cache lines on every wave's way to its class.
template <int BPC, int GRP, typename WaitT = NoWait>
__device__ __forceinline__ void dispatch(const ReconArgs<BPC> &a, const PlaneTab<BPC> &pt, const Dav1dGpuUnit &u,
                                         const Dav1dGpuIntraEdge &rec, int cls, int first, int count, uint8_t *lds,
                                         int gw, const WaitT &wait = WaitT()) {
#define DGPU_CASE(T) \
    case T: run_class<BPC, T, GRP>(a, pt, u, rec, first, count, lds, gw, wait); break;
    switch (cls) {
        DGPU_CASE(0) DGPU_CASE(1) DGPU_CASE(2) DGPU_CASE(3) DGPU_CASE(4) DGPU_CASE(5) DGPU_CASE(6)
        DGPU_CASE(7) DGPU_CASE(8) DGPU_CASE(9) DGPU_CASE(10) DGPU_CASE(11) DGPU_CASE(12) DGPU_CASE(13)
        DGPU_CASE(14) DGPU_CASE(15) DGPU_CASE(16) DGPU_CASE(17) DGPU_CASE(18)
        default: break;
    }
#undef DGPU_CASE
}
static_assert(DGPU_N_RECT_TX_SIZES == 19, "dispatch switch lists 19 classes");

// Minimum waves per SIMD the register allocator must allow, per bitdepth
// and group: 5 for the 8-bit main group (small + large classes) fits in 96
// VGPRs without spills (left alone it takes ~102, 4 waves: measured 2 us
// slower); the others are left to the compiler (forcing them spills).
template <int BPC, int GRP> constexpr int min_waves_per_eu() {
    return (BPC == 8 && GRP == GROUP_SMALL) ? 5 : 1;
}

template <int BPC, int GRP>
__global__ __launch_bounds__((64 * waves_per_block<BPC, GRP>()))
__attribute__((amdgpu_waves_per_eu(min_waves_per_eu<BPC, GRP>()))) void k_recon(ReconArgs<BPC> a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const unsigned long long t_entry = DGPU_TRACE ? __builtin_amdgcn_s_memtime() : 0;
    constexpr int WL = wave_lds<BPC, GRP>();
    constexpr int NC = DGPU_N_RECT_TX_SIZES;
    // XCD-contiguous block order: hardware deals blocks round-robin over the
    // 8 XCDs, so logical block (b % 8) * (nb / 8) + b / 8 gives XCD x the
    // x-th contiguous eighth of the schedule (gridDim.x is a multiple of 8)
    // Prologue, one memory round trip deep: every kernel argument the wave
    // needs is a scalar load issued here; the schedule is arithmetic on them;
    // the unit descriptors are loaded before the plane table is written and
    // the class code is entered.
    const int nb = gridDim.x, b = blockIdx.x;
    const int lb = (b & 7) * (nb >> 3) + (b >> 3);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gw = lb * waves_per_block<BPC, GRP>() + wave;
    // Every kernel argument of the prologue by constant index, pinned in
    // SGPRs at the top (the empty asm uses them), so the scalar loads go out
    // as one batch with one wait instead of a chain of dependent waits.
    int wpre[NC + 1];
#pragma unroll
    for (int c = 0; c <= NC; c++) wpre[c] = a.wpre[c];
    using P = typename Px<BPC>::pixel;
    const int nwaves = a.nwaves;
    const Dav1dGpuUnit *units = a.units;
    asm volatile("" ::"s"(nwaves), "s"(units));
#pragma unroll
    for (int c = 0; c <= NC; c += 4)
        asm volatile("" ::"s"(wpre[c]), "s"(wpre[cmin(c + 1, NC)]), "s"(wpre[cmin(c + 2, NC)]),
                     "s"(wpre[cmin(c + 3, NC)]));
    if (gw >= nwaves) return;
    // (segment, class) of this wave from the per-segment wave prefix
    // schedule: (segment group, class position, segment in group); a group
    // of kSegInner segments runs its classes largest first as a whole
    constexpr int SL = kSegInner;
    const int wgrp = wpre[NC] * SL;
    const int sg = gw / wgrp, r = gw - sg * wgrp;
    int pos = 0, wpre_p = 0;   // schedule position inside the group (kOrder)
#pragma unroll
    for (int c = 1; c < NC; c++) {
        const bool ge = r >= wpre[c] * SL;
        pos = ge ? c : pos;
        wpre_p = ge ? wpre[c] : wpre_p;
    }
    const int cls = order_class(pos);
    // the position's wave count and the class's unit range: three scalar
    // loads in one round trip (holding every class's values in SGPRs made
    // the compiler re-load them, measured slower)
    const int wp = a.wps[pos], cs0 = a.class_start[cls], cs1 = a.class_end[cls];
    const int lg = (int)((kLog2Lanes >> (3 * cls)) & 7);   // log2 lanes per unit, no table load
    const int U = 64 >> lg;
    const int r2 = r - wpre_p * SL;
    const int sl = SL == 1 ? 0 : r2 / wp;
    const int s = sg * SL + sl;
    const int first = cs0 + (s * wp + r2 - sl * wp) * U;
    const int count = min(U, cs1 - first);
    if (count <= 0) return;
    // this lane's unit descriptor (lanes past the last unit re-read it)
    const int ui_ = first + min((int)(threadIdx.x & 63) >> lg, count - 1);
    // (a struct load: assembling it from vector loads spilled it to scratch)
    const Dav1dGpuUnit u = bld(units + ui_);
    Dav1dGpuIntraEdge rec{};
    if constexpr (gathers(GRP)) rec = bld(a.recs + ui_);   // its edge record, in the same round trip
    // per-wave copy of the plane table: lane-indexed vector loads of the
    // argument segment, in flight together with the descriptor loads (no
    // workgroup barrier: the waves do not wait for each other)
    using PT = std::conditional_t<gathers(GRP), PlaneTabIE<BPC>, PlaneTab<BPC>>;
    __shared__ PT ptab[waves_per_block<BPC, GRP>()];
    PT &pt = ptab[wave];
    {
        const int t = threadIdx.x & 63;
        const int tr = min(t, DGPU_MAX_REFS * 3 - 1), td = min(t, 2);   // clamped: loads need no branch
        const P *rp = (&a.ref[0][0])[tr];
        const int rs = (&a.ref_stride[0][0])[tr];
        P *dp = a.dst[td];
        const int dsd = a.dst_stride[td];
        if (t < DGPU_MAX_REFS * 3) {
            pt.ref[t] = rp;
            pt.ref_stride[t] = rs;
        }
        if (t < 3) {
            pt.dst[t] = dp;
            pt.dst_stride[t] = dsd;
        }
        if constexpr (gathers(GRP)) {
            P *tp = a.top[td];
            const int ts = a.top_stride[td], tr_ = a.top_rows[td], sl = a.sb_log2[td];
            if (t < 3) {
                pt.top[t] = tp;
                pt.top_stride[t] = ts;
                pt.top_rows[t] = tr_;
                pt.sb_log2[t] = sl;
            }
        }
    }
    wave_sync();
    if constexpr (DGPU_TRACE) {   // kernel-entry and post-prologue times of this wave
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const unsigned long long t_sched = __builtin_amdgcn_s_memtime();
        if ((threadIdx.x & 63) == 0) {
            unsigned long long *tr = a.trace + ((size_t)GRP << 20) + (size_t)gw * 16;
            tr[15] = t_entry;
            tr[13] = t_entry;
            tr[14] = t_sched;
        }
    }
    if constexpr (GRP == GROUP_WARP) {   // the warp filter table in this wave's LDS (after its slots)
        uint2 *wt = reinterpret_cast<uint2 *>(lds + wave * WL + kWarpTabOff<BPC>);
        for (int i = threadIdx.x & 63; i < 193; i += 64) wt[i] = reinterpret_cast<const uint2 *>(dspt_warp)[i];
        wave_sync();
    }
    dispatch<BPC, GRP>(a, pt, u, rec, cls, first, count, lds + wave * WL, gw);
}

// (round 5: the main group as resident waves walking this schedule measured
// 84-477 us against 56; deleted in round 6)

template <int BPC, int GRP>
static int launch_group(ReconArgs<BPC> &a, const Dav1dGpuFrameBatch *b, unsigned classmask, hipStream_t stream) {
    constexpr int NC = DGPU_N_RECT_TX_SIZES;
    int acc = 0;
    for (int k = 0; k < NC; k++) {   // wps / wpre indexed by schedule position
        const int c = kOrder[k];
        a.wpre[k] = acc;
        a.wps[k] = 0;
        // this launch's range of class c: the WARP units at the end of the
        // class for the warp launch, the rest for the class's own group
        const int nw = b->class_warp[c];
        a.class_start[c] = GRP == GROUP_WARP ? b->class_start[c + 1] - nw : b->class_start[c];
        a.class_end[c] = GRP == GROUP_WARP ? b->class_start[c + 1] : b->class_start[c + 1] - nw;
        if (!in_group(c, GRP) || !((classmask >> c) & 1)) continue;
        const int n = a.class_end[c] - a.class_start[c];
        const int U = 64 / lanes_per_unit(c);
        a.wps[k] = ((n + U - 1) / U + kSegments - 1) / kSegments;
        acc += a.wps[k];
    }
    a.wpre[NC] = acc;
    acc *= kSegments;
    a.nwaves = acc;
    if (!acc) return 0;
    constexpr int WPB = waves_per_block<BPC, GRP>();
    const int nblk = ((acc + WPB - 1) / WPB + 7) & ~7;
    constexpr int lds = WPB * wave_lds<BPC, GRP>();
    static std::once_flag once;
    std::call_once(once, [] {
        (void)hipFuncSetAttribute((const void *)k_recon<BPC, GRP>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    });
    k_recon<BPC, GRP><<<dim3(nblk), 64 * WPB, lds, stream>>>(a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "dav1d-gpu: recon launch failed: %s\n", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

template <int BPC>
static int launch(const Dav1dGpuFrameBatch *b, hipStream_t stream) {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    constexpr int B = BPC / 8;
    if (!b || !b->units || b->n_units < 0) return -1;
    for (int c = 0; c < DGPU_N_RECT_TX_SIZES; c++)
        if (b->class_start[c + 1] < b->class_start[c]) return -2;
    if (b->class_start[0] != 0 || b->class_start[DGPU_N_RECT_TX_SIZES] != b->n_units) return -2;
    for (int p = 0; p < 3; p++) {   // output rows are stored with aligned 4/8-byte stores
        if (((uintptr_t)b->dst[p].data & 15) || (b->dst[p].stride & 15)) return -4;
        // row offsets are 24-bit multiplies in the kernels (__mul24): strides in [0, 2^23) bytes
        if (!stride24(b->dst[p].stride)) return -4;
        for (int r = 0; r < DGPU_MAX_REFS; r++)
            if (b->ref[r][p].data && !stride24(b->ref[r][p].stride)) return -4;
        for (int r = 0; r < DGPU_MAX_REFS; r++)   // footprint rows are read as aligned dwords
            if (b->ref[r][p].data && (b->ref[r][p].stride & 3)) return -4;
    }
    if (b->n_units == 0) return 0;
#if DGPU_BOUNDS
    {
        DgpuBndTab t{};
        for (int p = 0; p < 3; p++) {
            bnd_add(t, b->dst[p], BND_DST);
            for (int r = 0; r < DGPU_MAX_REFS; r++) bnd_add(t, b->ref[r][p], BND_REF);
        }
        bnd_add(t, b->cfl_luma, BND_CFL);
        bnd_range(t, b->units, (unsigned long long)b->n_units * sizeof(Dav1dGpuUnit), BND_UNITS);
        bnd_add_extra(t);
        bnd_print<P>(t, "recon");
        if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_dgpu_bnd), &t, sizeof(t), 0, hipMemcpyHostToDevice, stream) != hipSuccess ||
            hipStreamSynchronize(stream) != hipSuccess)
            return -3;
    }
#endif

    ReconArgs<BPC> a;
    memset(&a, 0, sizeof(a));
    for (int p = 0; p < 3; p++) {
        a.dst[p] = (P *)b->dst[p].data;
        a.dst_stride[p] = (int)(b->dst[p].stride / B);
        for (int r = 0; r < DGPU_MAX_REFS; r++) {
            a.ref[r][p] = (const P *)b->ref[r][p].data;
            a.ref_stride[r][p] = (int)(b->ref[r][p].stride / B);
            a.ref_w[r][p] = b->ref[r][p].w;
            a.ref_h[r][p] = b->ref[r][p].h;
        }
    }
    a.units = b->units;
    a.coef = (C *)b->coef;
    a.edges = (const P *)b->edges;
    a.cfl_luma = (const P *)b->cfl_luma.data;
    if (b->cfl_luma.data && !stride24(b->cfl_luma.stride)) return -4;
    a.cfl_luma_stride = (int)(b->cfl_luma.stride / B);
    a.cfl_ss = b->cfl_ss;
    a.aux = b->aux;
    a.aux_pool = (const uint8_t *)b->aux_pool;
    for (int c = 0; c < DGPU_N_RECT_TX_SIZES; c++) {   // WARP sub-ranges: classes with both sides >= 8
        const int nw = b->class_warp[c];
        if (nw < 0 || nw > b->class_start[c + 1] - b->class_start[c] || (nw && !in_group(c, GROUP_WARP))) return -2;   // no 64-point class
    }
    a.bdmax = BPC == 8 ? 255 : b->bitdepth_max;
    a.zero_coefs = b->zero_coefs;
    // debug-only profiling knob (never set in production):
    //   DAV1D_GPU_CLASSMASK restrict to some size classes (others stale)
    const char *cm = getenv("DAV1D_GPU_CLASSMASK");
    const unsigned classmask = cm ? (unsigned)strtoul(cm, nullptr, 0) : ~0u;

    // Group kernels in order on the caller's stream (cross-stream fork/join
    // measured ~25 us of event overhead per frame on MI355X: slower).
    static unsigned long long *trace_buf = nullptr;   // DGPU_TRACE builds only
    if (DGPU_TRACE && !trace_buf && hipMalloc(&trace_buf, (size_t)3 << 23) != hipSuccess) return -3;
    a.trace = trace_buf;
    int nw[3] = {0, 0, 0};
    int rc = launch_group<BPC, GROUP_WARP>(a, b, classmask, stream);
    if (!rc) rc = launch_group<BPC, GROUP_HUGE>(a, b, classmask, stream);
    nw[2] = a.nwaves;
    if (!rc) rc = launch_group<BPC, GROUP_LARGE>(a, b, classmask, stream);
    nw[1] = a.nwaves;
    if (!rc) rc = launch_group<BPC, GROUP_SMALL>(a, b, classmask, stream);
    nw[0] = a.nwaves;
    if (DGPU_TRACE && !rc) {   // debug: synchronous dump of the phase timestamps
        const char *f = getenv("DAV1D_GPU_TRACE_FILE");
        if (f && hipStreamSynchronize(stream) == hipSuccess) {
            FILE *fp = fopen(f, "ab");
            for (int g = 0; g < 3 && fp; g++) {
                const size_t n = (size_t)nw[g] * 16;
                unsigned long long *h = (unsigned long long *)malloc(n * 8 + 8);
                if (n && h && hipMemcpy(h, trace_buf + ((size_t)g << 20), n * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                    const int hdr[2] = {g, nw[g]};
                    fwrite(hdr, sizeof(hdr), 1, fp);
                    fwrite(h, 8, n, fp);
                }
                free(h);
            }
            if (fp) fclose(fp);
            (void)hipMemset(trace_buf, 0, (size_t)3 << 23);
        }
    }
    return rc;
}

}  // namespace dgpu

