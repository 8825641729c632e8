// recon_kernel.hpp -- the batch tier: one grid launch per class group
// reconstructs a frame's worth of transform-block units (Dav1dGpuUnit).
//
// Per unit the work the reference does in recon_b_inter / recon_b_intra
// (src/recon_tmpl.c:1598, :1195) for one transform block: the prediction
// (mc put, or mct x2 + avg, src/recon_tmpl.c:957-1059, :1845; or intra_pred,
// :1294) then inv_txfm_add (:816 / :1347), fused so the prediction never
// round-trips through HBM.
//
// Mapping (wave64, v3).  Units are sorted by transform size class.  A unit
// is cut into 4x2-pixel output tasks; a class gives each unit G lanes (one
// task per lane up to the width of the 1-D transform passes, see
// lanes_per_unit) and a wave owns 64/G units.
//   P1  global loads: descriptor, the compact coefficient region and intra
//       edge array (16-B chunks into LDS), the mc footprint rows (dwordx4
//       per row and 4-px quad, straight into registers)
//   P2  mc horizontal pass, both refs: one task = 2 footprint rows x 4
//       outputs; 8bpc uses v_alignbyte + v_dot4 on bias-shifted bytes, 16bpc
//       v_dot2 on pixel pairs.  Intermediates are stored as (row 2p, row
//       2p+1) int16 pairs so the vertical pass is v_dot2 as well.
//   P3  row transforms (rows >= nzh are zero and skip the math)
//   P4  column transforms -> residual, column-major
//   P5  intra edge preparation / filter-intra wavefront
//   P6  per task: vertical pass (+ compound average) or intra formula, add
//       the residual, clip, and store 4-px rows straight to the picture.
// Every 8-tap and bilinear case runs the same h+v pipeline: m == 0 is the
// identity tap and bilinear is the (64 - 4m, 4m) bank, which give the
// reference's h-only / v-only / copy / bilinear results exactly (the
// rounding identities are spelled out in DESIGN.md section 4).
// Every LDS hand-off stays inside one wave (no workgroup barrier).
#pragma once
#include "dav1d_gpu.h"
#include "bounds.hpp"
#include "dsp_common.hpp"
#include "intra_edge_dev.hpp"

#include <stddef.h>

#include <utility>

#ifndef DGPU_TRACE
#define DGPU_TRACE 0       // diagnostics: per-wave phase timestamps (tools/wave_trace.py)
#endif
#ifndef DGPU_TRACE_RT
#define DGPU_TRACE_RT 0    // diagnostics: the trace in the 100 MHz clock of the flow trace
#endif

namespace dgpu {

// Measured variants of this kernel that lost (phase ablations, row skipping,
// realigned odd rows, padded residual columns, aligned 16bpc rows, paired
// 8-byte stores, nontemporal streams, resident waves) were deleted in round
// 6; their A/B results stay under profiles/r3..r5 and in DESIGN.md.
constexpr int kSegments = 16;      // spatial segments per class (task ordering; 8 / 32: 67 / 64 us)
// segments whose classes are scheduled as one group (2 / 4 / 16: 58.9 / 59.2
// / 67.4 against 56.9 us, profiles/r6/r6j_krecon_seg_group_ab.json)
constexpr int kSegInner = 1;
// compound refs one after the other through one tile up to this many tasks
// per lane (0: 60.2 against 56.8 us; profiles/r6/r6k_krecon_seqref_ch_ab.json)
constexpr int kSeqRefMaxTpl = 2;

template <int BPC> struct ReconArgs {
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    P *dst[3];
    int dst_stride[3];                   // pixels
    const P *ref[DGPU_MAX_REFS][3];
    int ref_stride[DGPU_MAX_REFS][3];    // pixels
    const Dav1dGpuUnit *units;
    C *coef;
    const P *edges;
    const P *cfl_luma;    // luma read by CFL units
    int cfl_luma_stride;  // pixels
    int cfl_ss;           // ss_hor | ss_ver << 1
    const int32_t *aux;       // per unit: aux_pool offset (INTER_MASK mask, PAL record)
    const uint8_t *aux_pool;
    int class_start[DGPU_N_RECT_TX_SIZES + 1];   // this launch's unit range per class: [start, end)
    int class_end[DGPU_N_RECT_TX_SIZES];
    // wave schedule, ordered (segment, class position): every one of the
    // kSegments segments gives the class at position k (kOrder) wps[k]
    // waves (its unit range cut into kSegments runs of wps[k] * U units);
    // wpre is the prefix of wps, so a wave's (segment, class, first unit)
    // is arithmetic, no search.
    int wps[DGPU_N_RECT_TX_SIZES];
    int wpre[DGPU_N_RECT_TX_SIZES + 1];
    int nwaves;
    unsigned long long *trace;   // DGPU_TRACE builds only: [group][wave][16] s_memtime
    int bdmax;
    int zero_coefs;
    // intra wavefront launches only (GROUP_*_IE): recs[i] is units[i]'s
    // edge record; the edges are gathered from the picture in the kernel,
    // the rewritten mode / angle go back to units_rw, and superblock-bottom
    // rows are also stored to top[] (dav1d_backup_ipred_edge) when set
    const Dav1dGpuIntraEdge *recs;
    Dav1dGpuUnit *units_rw;
    P *top[3];
    int top_stride[3];   // pixels
    int top_rows[3];
    int sb_log2[3];
    // the reference planes' visible sizes: DGPU_MX_CLAMP units (second
    // launch) clamp every footprint pixel to them (emu_edge)
    int ref_w[DGPU_MAX_REFS][3], ref_h[DGPU_MAX_REFS][3];
};

// Plane pointers and strides, copied once per workgroup into LDS so the
// per-unit (ref, plane) lookup is an LDS read, not a dependent load from
// the kernel-argument segment.
template <int BPC> struct PlaneTab {
    using P = typename Px<BPC>::pixel;
    const P *ref[DGPU_MAX_REFS * 3];
    P *dst[3];
    int ref_stride[DGPU_MAX_REFS * 3];   // pixels
    int dst_stride[3];
};

template <int BPC> struct PlaneTabIE : PlaneTab<BPC> {
    using P = typename Px<BPC>::pixel;
    P *top[3];
    int top_stride[3];   // pixels
    int top_rows[3];
    int sb_log2[3];
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the kernels form row offsets with 24-bit multiplies (__mul24 / __umul24)
__host__ __device__ constexpr bool stride24(ptrdiff_t s) { return s >= 0 && s < (1 << 23); }
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }
__host__ __device__ constexpr int cmin(int a, int b) { return a < b ? a : b; }
__host__ __device__ constexpr int a16(int v) { return (v + 15) & ~15; }

// lanes per unit: one 4x2 output task per lane (W*H/8), but no more lanes
// than the 1-D transform passes can use (max(W, min(H, 32)) lines), 2..64;
// 32x32 takes a whole wave so its LDS slot (9 KB) does not set the budget
// of the large group
#ifndef DGPU_IE_SMALL_LANES
// lanes per unit of the 4x4 / 4x8 / 8x4 classes, for the intra wavefront
// TUs (recon_ie{8,16}.hip set 8; 0 here: the class's own count).  Above level
// 0 a wavefront task holds at most 8 units, so at 2-4 lanes per unit most of
// its wave idles while the small units' edge preparation runs per lane
#define DGPU_IE_SMALL_LANES 0
#endif
#ifndef DGPU_IE_WIDE_LANES
// the intra wavefront TUs (A/B, round 6): one 4x2 output task per lane for
// every class (W*H/8, at most 64), not the unit batch's LDS-bound counts --
// a wavefront task holds at most 8 units above level 0, and the flow trace
// shows the tall classes (4x16: 4 lanes, 8x16: 8) as the levels' slowest
#define DGPU_IE_WIDE_LANES 0
#endif
__host__ __device__ constexpr int lanes_per_unit(int tx) {
    const int w = tx_info(tx).w, h = tx_info(tx).h;
    if (DGPU_IE_SMALL_LANES && w * h <= 32) return DGPU_IE_SMALL_LANES;
    if (DGPU_IE_WIDE_LANES) return cmin(cmax(w * h / 8, 2), 64);
    if (w * h >= 1024) return 64;
    // tall classes: as few lanes as the column pass has lines (or half as
    // many for 8x32), so the column transforms leave no lane idle, within
    // the 8 KB-per-wave LDS budget of the main group (round 3; the rule
    // below gives 16 / 8 / 32 lanes, half of them idle in the column pass)
    if (w == 8 && h == 16) return 8;
    if (w == 4 && h == 16) return 4;
    if (w == 8 && h == 32) return 16;
    return cmin(cmax(cmin(w * h / 8, cmax(w, cmin(h, 32))), 2), 64);
}
// HPass advances a lane's row pairs by G / QW from a first pair l / QW: every
// class a product kernel runs has at most as many lane rows as footprint row
// pairs (G / QW <= RP), so no lane starts past the footprint (the r5j fault:
// a negative row-pair offset through an unsigned 24-bit multiply).  Only the
// wavefront TUs' small-unit lanes (DGPU_IE_SMALL_LANES) exceed it, and HPass
// clamps their base pair at compile time for exactly that case.
__host__ __device__ constexpr bool lanes_fit_row_pairs() {
    for (int tx = 0; tx < DGPU_N_RECT_TX_SIZES; tx++) {
        const int w = tx_info(tx).w, h = tx_info(tx).h;
        if (DGPU_IE_SMALL_LANES && w * h <= 32) continue;
        if (lanes_per_unit(tx) % (w / 4) || lanes_per_unit(tx) / (w / 4) > (h + 8) / 2) return false;
    }
    return true;
}
static_assert(lanes_fit_row_pairs(), "a product class gives a unit more lane rows than footprint row pairs");
// class groups, each its own kernel with its own register / LDS budget:
// small (w*h <= 128), large (up to 32x32), huge (the 64-point sides).
// Small and large are one launch: the large classes' long-latency waves
// then overlap the small classes' work (measured 76 -> 64 us per 4K frame
// against two launches back to back); GROUP_LARGE stays as a name only.
enum { GROUP_SMALL = 0, GROUP_LARGE = 1, GROUP_HUGE = 2, GROUP_WARP = 3, N_GROUPS = 4,
       // the intra wavefront's variants of SMALL / HUGE: edges gathered in
       // the kernel (intra_edge_dev.hpp) instead of read from the edge pool
       GROUP_SMALL_IE = 4, GROUP_HUGE_IE = 6,
       // the persistent intra wavefront kernel (flow_impl.hpp): every class
       GROUP_ALL_IE = 8 };
__host__ __device__ constexpr int base_group(int grp) {
    return grp == GROUP_ALL_IE ? GROUP_HUGE : grp >= N_GROUPS ? grp - N_GROUPS : grp;
}
__host__ __device__ constexpr bool gathers(int grp) { return grp >= N_GROUPS; }
__host__ __device__ constexpr int class_group(int tx) {
    const int w = tx_info(tx).w, h = tx_info(tx).h;
    return (w == 64 || h == 64) ? GROUP_HUGE
         : GROUP_SMALL;
}
// Order of the classes inside one schedule segment: largest first, so
// their long-latency waves start early.  kOrder[position] = class.
constexpr int kOrder[DGPU_N_RECT_TX_SIZES] = {3, 9, 10, 2, 15, 16, 7, 8, 1, 13, 14, 5, 6, 0, 4, 11, 12, 17, 18};
__host__ __device__ constexpr uint64_t pack_order(int half) {
    uint64_t v = 0;
    for (int i = 0; i < 12; i++) {
        const int k = half * 12 + i;
        if (k < DGPU_N_RECT_TX_SIZES) v |= (uint64_t)kOrder[k] << (5 * i);
    }
    return v;
}
__device__ __forceinline__ int order_class(int k) {   // kOrder[k] without a memory load
    constexpr uint64_t lo = pack_order(0), hi = pack_order(1);
    return (int)(((k < 12 ? lo : hi) >> (5 * (k < 12 ? k : k - 12))) & 31);
}

// classes a launch of group GRP runs: the warp launch takes every class with
// both sides >= 8 (its units are the WARP sub-ranges), the others by size
__host__ __device__ constexpr bool in_group(int tx, int grp_) {
    if (grp_ == GROUP_ALL_IE) return true;
    const int grp = base_group(grp_);
    return grp == GROUP_WARP ? class_group(tx) != GROUP_HUGE : class_group(tx) == grp;
}

template <int TX> struct Cls {
    static constexpr int W = tx_info(TX).w, H = tx_info(TX).h, SHIFT = tx_info(TX).shift;
    static constexpr int SW = cmin(W, 32), SH = cmin(H, 32);
    static constexpr int G = lanes_per_unit(TX), U = 64 / G;
    static constexpr bool RECT2 = W * 2 == H || H * 2 == W;
    static constexpr int QW = W / 4;            // 4-px quads per row
    static constexpr int NT = H / 2 * QW;       // 4x2 output tasks
    static constexpr int RP = (H + 8) / 2;      // mc intermediate row pairs (rows 0..H+7)
    static constexpr int NH = RP * QW;          // h-pass tasks
    static constexpr int TPL = (NT + G - 1) / G;  // output tasks per lane
    // compound refs run one after the other through one intermediate tile,
    // the first ref's predictions held in registers across the second
    static constexpr bool SEQREF = TPL <= kSeqRefMaxTpl;
};

template <int BPC> struct Tmp { using T = int32_t; };
template <> struct Tmp<8> { using T = int16_t; };   // 8-bit row output / residual fit int16

// LDS slot of one unit (bytes): [coefs | residual] [row-pass tmp] [mc | intra]
// (FE serves the directional modes, PT filter intra: never both)
template <int BPC, int TX> struct Slot {
    using CL = Cls<TX>;
    static constexpr int W = CL::W, H = CL::H, B = BPC / 8;
    static constexpr int CB = sizeof(typename Px<BPC>::coef);
    static constexpr int TB = sizeof(typename Tmp<BPC>::T);
    static constexpr int CF = a16(CL::SW * CL::SH * CB + 16);   // compact coefs at their 16-B skew
    // residual, column-major [x][y] with a column stride of RS elements
    // (padding the columns against the 4/8-way bank conflicts measured no
    // gain: 56.0 against 56.1 us, profiles/r5/r5c_krecon_ab.json)
    static constexpr int RS = H;
    static constexpr int RES = W * RS * TB;
    static constexpr int CFR = a16(cmax(CF, RES));
    static constexpr int TMP = a16(CL::SH * W * TB);             // row-pass output [y][x]
    static constexpr int MID = CL::RP * W * 4;                   // one ref: [row pair][x] int16 x2
    static constexpr int EDGE = 2 * H + 2 * W + 1;               // topleft[-2h..2w]
    static constexpr int EB = a16(EDGE * B + 16);                // raw edge pixels at their skew
    static constexpr int FE = a16(EDGE * 2);                     // prepared edge, int16
    static constexpr int PT = a16(W * H * 2);                    // filter-intra tile, int16 (aliases FE)
    static constexpr int SRC = cmax((CL::SEQREF ? 1 : 2) * MID, EB + cmax(FE, PT));
    static constexpr int BYTES = CFR + TMP + SRC;
    static constexpr int WAVE = CL::U * BYTES;
    // the second launch (WARP group): INTER_SCALED keeps its h-pass output
    // as int16 [rows][W] with rows <= 2H + 8 (steps dx, dy <= 2048)
    static constexpr int SCALED = a16((2 * H + 8) * W * 2);
    static constexpr int BYTES_W = CFR + TMP + cmax(SRC, SCALED);
    static constexpr int WAVE_W = CL::U * BYTES_W;
};

// LDS bytes per wave of a launch group: its largest class slot set; the warp
// launch adds its copy of the warp filter table (193 x 8 int8) after that
template <int BPC, int GRP, int... TX>
__host__ __device__ constexpr int group_wave_lds(std::integer_sequence<int, TX...>) {
    int m = 0;
    if constexpr (GRP == GROUP_WARP)
        ((m = (in_group(TX, GRP) && Slot<BPC, TX>::WAVE_W > m) ? Slot<BPC, TX>::WAVE_W : m), ...);
    else
        ((m = (in_group(TX, GRP) && Slot<BPC, TX>::WAVE > m) ? Slot<BPC, TX>::WAVE : m), ...);
    return m;
}
template <int BPC> inline constexpr int kWarpTabOff =
    group_wave_lds<BPC, GROUP_WARP>(std::make_integer_sequence<int, DGPU_N_RECT_TX_SIZES>());
template <int BPC, int GRP> __host__ __device__ constexpr int wave_lds() {
    return group_wave_lds<BPC, GRP>(std::make_integer_sequence<int, DGPU_N_RECT_TX_SIZES>()) +
           (GRP == GROUP_WARP ? 193 * 8 + 8 : 0);
}

// ------------------------------------------------------------ primitives ---

typedef short v2i16 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3a1 __attribute__((ext_vector_type(3), aligned(1)));
typedef uint32_t u32x2a1 __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t u32x4a2 __attribute__((ext_vector_type(4), aligned(2)));
typedef uint32_t u32x2a2 __attribute__((ext_vector_type(2), aligned(2)));

// Packed dot products.  Chains start from an inline constant (0 .. 64) so
// the compiler keeps the three-operand form for the first step and the
// accumulating two-operand form after it (no accumulator copies).
__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, a), __builtin_bit_cast(v2i16, b), c, false);
}
__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}
// Dot-product blocks in inline assembly, four independent chains per
// block.  The compiler's own selection always starts a chain with a copy
// of the start value into the accumulator (two-operand v_dot*c forms); the
// three-operand forms here take it as an inline constant or SGPR.  The
// compiler cannot see a hazard inside asm, so each block keeps it itself:
// a DOT result is read by another VALU op only >= 3 instructions later
// (gfx950 DOT-write -> VALU-read wait states); chains are interleaved and
// every block ends in plain VALU ops.
//
// m[i] = (dot4(hi[i], ty, dot4(lo[i], tx, 2))) >> 2
__device__ __forceinline__ void hdot4x4(const uint32_t *lo, const uint32_t *hi, uint32_t tx, uint32_t ty, int *m) {
    asm("v_dot4_i32_i8 %0, %4, %12, 2\n\t"
        "v_dot4_i32_i8 %1, %5, %12, 2\n\t"
        "v_dot4_i32_i8 %2, %6, %12, 2\n\t"
        "v_dot4_i32_i8 %3, %7, %12, 2\n\t"
        "v_dot4_i32_i8 %0, %8, %13, %0\n\t"
        "v_dot4_i32_i8 %1, %9, %13, %1\n\t"
        "v_dot4_i32_i8 %2, %10, %13, %2\n\t"
        "v_dot4_i32_i8 %3, %11, %13, %3\n\t"
        "v_ashrrev_i32 %0, 2, %0\n\t"
        "v_ashrrev_i32 %1, 2, %1\n\t"
        "v_ashrrev_i32 %2, 2, %2\n\t"
        "v_ashrrev_i32 %3, 2, %3"
        : "=&v"(m[0]), "=&v"(m[1]), "=&v"(m[2]), "=&v"(m[3])
        : "v"(lo[0]), "v"(lo[1]), "v"(lo[2]), "v"(lo[3]), "v"(hi[0]), "v"(hi[1]), "v"(hi[2]), "v"(hi[3]),
          "v"(tx), "v"(ty));
}
// t[i] = (sum_k dot2(a[k][i], tap pair k) + kk) >> sh, k = 0..3; the chains
// start from kk (an SGPR operand), so no separate add
__device__ __forceinline__ void vdot4x4(const uint32_t (*a)[4], const uint4 &tv, int kk, int sh, int *t) {
    asm("v_dot2_i32_i16 %0, %4, %20, %24\n\t"
        "v_dot2_i32_i16 %1, %5, %20, %24\n\t"
        "v_dot2_i32_i16 %2, %6, %20, %24\n\t"
        "v_dot2_i32_i16 %3, %7, %20, %24\n\t"
        "v_dot2_i32_i16 %0, %8, %21, %0\n\t"
        "v_dot2_i32_i16 %1, %9, %21, %1\n\t"
        "v_dot2_i32_i16 %2, %10, %21, %2\n\t"
        "v_dot2_i32_i16 %3, %11, %21, %3\n\t"
        "v_dot2_i32_i16 %0, %12, %22, %0\n\t"
        "v_dot2_i32_i16 %1, %13, %22, %1\n\t"
        "v_dot2_i32_i16 %2, %14, %22, %2\n\t"
        "v_dot2_i32_i16 %3, %15, %22, %3\n\t"
        "v_dot2_i32_i16 %0, %16, %23, %0\n\t"
        "v_dot2_i32_i16 %1, %17, %23, %1\n\t"
        "v_dot2_i32_i16 %2, %18, %23, %2\n\t"
        "v_dot2_i32_i16 %3, %19, %23, %3\n\t"
        "v_ashrrev_i32 %0, %25, %0\n\t"
        "v_ashrrev_i32 %1, %25, %1\n\t"
        "v_ashrrev_i32 %2, %25, %2\n\t"
        "v_ashrrev_i32 %3, %25, %3"
        : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3])
        : "v"(a[0][0]), "v"(a[0][1]), "v"(a[0][2]), "v"(a[0][3]), "v"(a[1][0]), "v"(a[1][1]), "v"(a[1][2]),
          "v"(a[1][3]), "v"(a[2][0]), "v"(a[2][1]), "v"(a[2][2]), "v"(a[2][3]), "v"(a[3][0]), "v"(a[3][1]),
          "v"(a[3][2]), "v"(a[3][3]), "v"(tv.x), "v"(tv.y), "v"(tv.z), "v"(tv.w), "s"(kk), "s"(sh));
}

// Global-memory access through pointers that came from LDS (the plane
// table): tell the compiler the address space so it emits global_*
// instead of flat_* instructions.
#ifndef DGPU_BOUNDS
#define DGPU_BOUNDS 0
#endif
#if DGPU_BOUNDS
// Diagnostics builds only (tools/build_variants.sh `bounds`): every device
// range a launch may touch, [lo, hi) each -- the planes it was given
// ([data, data + stride * h)) and, when the caller registered them
// (dgpu::bnd_extra(): the recorder registers every buffer of its flush with
// its exact byte size), the unit / record / coefficient / edge / aux /
// workspace / scratch buffers.  Strict tables (any buffer registered): an
// access inside none of the ranges is printed with its source line and the
// range table's ids, and skipped.  Otherwise (planes only: direct callers of
// the batch entries) only an access within 4 MiB of a plane is judged.
struct DgpuBndTab {
    unsigned long long r[64][2];
    int id[64];
    int n, strict;
};
static __device__ DgpuBndTab g_dgpu_bnd;
static __device__ int g_dgpu_bnd_hits;   // printed at most 256 times per process
__device__ __noinline__ bool bnd_ok(const void *p, int n, int line) {
    const unsigned long long a = (unsigned long long)(uintptr_t)p;
    bool near = false;
    for (int i = 0; i < g_dgpu_bnd.n; i++) {
        const unsigned long long lo = g_dgpu_bnd.r[i][0], hi = g_dgpu_bnd.r[i][1];
        if (a >= lo && a + n <= hi) return true;
        if (a + (4ull << 20) > lo && a < hi + (4ull << 20)) near = true;
    }
    if (!g_dgpu_bnd.strict && !near) return true;
    if (atomicAdd(&g_dgpu_bnd_hits, 1) < 256)
        printf("DGPU_BOUNDS line %d addr %llx bytes %d block %d lane %d\n", line, a, n, (int)blockIdx.x,
               (int)(threadIdx.x & 63));
    return false;
}
static inline void bnd_range(DgpuBndTab &t, const void *p, unsigned long long bytes, int id) {
    if (p && bytes && t.n < (int)(sizeof(t.r) / sizeof(t.r[0]))) {
        t.r[t.n][0] = (unsigned long long)(uintptr_t)p;
        t.r[t.n][1] = t.r[t.n][0] + bytes;
        t.id[t.n] = id;
        t.n++;
    }
}
static inline void bnd_add(DgpuBndTab &t, const Dav1dGpuPlane &pl, int id = 0) {
    if (pl.data) bnd_range(t, pl.data, (unsigned long long)pl.stride * (unsigned long long)pl.h, id);
}
// the caller's registered buffers (strict mode when there are any)
static inline void bnd_add_extra(DgpuBndTab &t) {
    for (const BndRange &e : bnd_extra()) {
        bnd_range(t, e.p, e.bytes, e.id);
        t.strict = 1;
    }
}
template <typename P>
static inline void bnd_print(const DgpuBndTab &t, const char *who) {
    for (int i = 0; i < t.n; i++)
        fprintf(stderr, "DGPU_BOUNDS %s range %d id %d %llx..%llx%s\n", who, i, t.id[i], t.r[i][0], t.r[i][1],
                t.strict ? " strict" : "");
}
#define DGPU_LINE , int line = __builtin_LINE()
#define DGPU_CHK(p, n, fail) if (!bnd_ok(p, n, line)) fail
#else
#define DGPU_LINE
#define DGPU_CHK(p, n, fail)
#endif
template <typename T> __device__ __forceinline__ T gld(const void *p DGPU_LINE) {
    DGPU_CHK(p, (int)sizeof(T), return T{});
    return *(const __attribute__((address_space(1))) T *)p;
}
template <typename T> __device__ __forceinline__ void gst(void *p, T v DGPU_LINE) {
    DGPU_CHK(p, (int)sizeof(T), return);
    *(__attribute__((address_space(1))) T *)p = v;
}
// Plain loads / stores of the descriptor, record, aux-index and workspace
// arrays: exactly `*p` / `*p = v` in product builds, checked in DGPU_BOUNDS
// builds; bnd_touch checks the address of an atomic
template <typename T> __device__ __forceinline__ T bld(const T *p DGPU_LINE) {
    DGPU_CHK(p, (int)sizeof(T), return T{});
    return *p;
}
template <typename T> __device__ __forceinline__ void bst(T *p, T v DGPU_LINE) {
    DGPU_CHK(p, (int)sizeof(T), return);
    *p = v;
}
template <typename T> __device__ __forceinline__ void bnd_touch(const T *p DGPU_LINE) {
    DGPU_CHK(p, (int)sizeof(T), return);
}

// ({hi, lo} >> 8s)[31:0]
__device__ __forceinline__ uint32_t alb(uint32_t hi, uint32_t lo, int s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}
// (lo16(lo), lo16(hi)) -- int16 truncation, as the reference's int16_t stores
__device__ __forceinline__ uint32_t pack16(int lo, int hi) {
    return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u);
}

// The odd output rows of a 4x2 task from the same (row 2p, row 2p+1) pairs
// as the even ones: row 2j+1+m needs taps shifted by one row, i.e. pairs
// (0, t0) (t1, t2) (t3, t4) (t5, t6) (t7, 0) over P[0..4] -- five dot2 per
// output instead of four on realigned pairs (v_alignbyte) (s: the shifted
// tap pairs, see vtaps_odd).  Two blocks (operand limit); the first ends
// with wait states, its outputs being DOT results.
__device__ __forceinline__ void vtaps_odd(const uint4 &tv, uint32_t *s) {
    s[0] = tv.x << 16;
    s[1] = alb(tv.y, tv.x, 2);
    s[2] = alb(tv.z, tv.y, 2);
    s[3] = alb(tv.w, tv.z, 2);
    s[4] = tv.w >> 16;
}
__device__ __forceinline__ void vdot5x4(const uint32_t (*a)[4], const uint32_t *s, int kk, int sh, int *t) {
    int u0, u1, u2, u3;
    asm("v_dot2_i32_i16 %0, %4, %16, %19\n\t"
        "v_dot2_i32_i16 %1, %5, %16, %19\n\t"
        "v_dot2_i32_i16 %2, %6, %16, %19\n\t"
        "v_dot2_i32_i16 %3, %7, %16, %19\n\t"
        "v_dot2_i32_i16 %0, %8, %17, %0\n\t"
        "v_dot2_i32_i16 %1, %9, %17, %1\n\t"
        "v_dot2_i32_i16 %2, %10, %17, %2\n\t"
        "v_dot2_i32_i16 %3, %11, %17, %3\n\t"
        "v_dot2_i32_i16 %0, %12, %18, %0\n\t"
        "v_dot2_i32_i16 %1, %13, %18, %1\n\t"
        "v_dot2_i32_i16 %2, %14, %18, %2\n\t"
        "v_dot2_i32_i16 %3, %15, %18, %3\n\t"
        "s_nop 2"
        : "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3)
        : "v"(a[0][0]), "v"(a[0][1]), "v"(a[0][2]), "v"(a[0][3]), "v"(a[1][0]), "v"(a[1][1]), "v"(a[1][2]),
          "v"(a[1][3]), "v"(a[2][0]), "v"(a[2][1]), "v"(a[2][2]), "v"(a[2][3]), "v"(s[0]), "v"(s[1]), "v"(s[2]),
          "s"(kk));
    asm("v_dot2_i32_i16 %0, %4, %12, %0\n\t"
        "v_dot2_i32_i16 %1, %5, %12, %1\n\t"
        "v_dot2_i32_i16 %2, %6, %12, %2\n\t"
        "v_dot2_i32_i16 %3, %7, %12, %3\n\t"
        "v_dot2_i32_i16 %0, %8, %13, %0\n\t"
        "v_dot2_i32_i16 %1, %9, %13, %1\n\t"
        "v_dot2_i32_i16 %2, %10, %13, %2\n\t"
        "v_dot2_i32_i16 %3, %11, %13, %3\n\t"
        "v_ashrrev_i32 %0, %14, %0\n\t"
        "v_ashrrev_i32 %1, %14, %1\n\t"
        "v_ashrrev_i32 %2, %14, %2\n\t"
        "v_ashrrev_i32 %3, %14, %3"
        : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3)
        : "v"(a[3][0]), "v"(a[3][1]), "v"(a[3][2]), "v"(a[3][3]), "v"(a[4][0]), "v"(a[4][1]), "v"(a[4][2]),
          "v"(a[4][3]), "v"(s[3]), "v"(s[4]), "s"(sh));
    t[0] = u0;
    t[1] = u1;
    t[2] = u2;
    t[3] = u3;
}

// Copies bytes [src, src + n) into 16-B aligned LDS at their own 16-B skew
// with 16-byte loads, in two steps so other loads can be issued in between:
// load() issues the global loads, commit() writes LDS and returns the skew.
// Reads stay inside the 16-B blocks holding the first and last byte.
template <int MAXN, int G> struct Stage {
    static constexpr int IT = ((MAXN + 30) / 16 + G - 1) / G;
    u32x4 v[IT];
    int sk, nch;
    __device__ __forceinline__ void load(const void *src, int n, int l) {
        sk = (int)(reinterpret_cast<uintptr_t>(src) & 15);
        const uint8_t *s = reinterpret_cast<const uint8_t *>(src) - sk;
        nch = (sk + n + 15) >> 4;   // >= 1 for n >= 1
#pragma unroll
        for (int k = 0; k < IT; k++)   // clamped
            v[k] = gld<u32x4>(s + 16 * min(l + k * G, nch - 1));
    }
    __device__ __forceinline__ int commit(uint8_t *dst, int l) const {
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const int i = l + k * G;
            if (i < nch) reinterpret_cast<u32x4 *>(dst)[i] = v[k];
        }
        return sk;
    }
};

// ---------------------------------------------------------------- intra ---

__device__ __forceinline__ int ip_strength(int wh, int angle, int is_sm) {  // ipred_tmpl.c:327
    if (is_sm) {
        if (wh <= 8) return angle >= 64 ? 2 : angle >= 40 ? 1 : 0;
        if (wh <= 16) return angle >= 48 ? 2 : angle >= 20 ? 1 : 0;
        if (wh <= 24) return angle >= 4 ? 3 : 0;
        return 3;
    }
    if (wh <= 8) return angle >= 56 ? 1 : 0;
    if (wh <= 16) return angle >= 40 ? 1 : 0;
    if (wh <= 24) return angle >= 32 ? 3 : angle >= 16 ? 2 : angle >= 8 ? 1 : 0;
    if (wh <= 32) return angle >= 32 ? 3 : angle >= 4 ? 2 : 1;
    return 3;
}
__device__ __forceinline__ int ip_upsample(int wh, int angle, int is_sm) {
    return angle < 40 && wh <= (16 >> is_sm);
}
// filter_edge element (src/ipred_tmpl.c:362-385), `in` indexed from 0
template <typename T>
__device__ __forceinline__ int ip_smooth(const T *in, int i, int lim_from, int lim_to, int from, int to, int st) {
    if (i < lim_from || i >= lim_to) return in[clampi(i, from, to - 1)];
    const int k0 = st == 3 ? 2 : 0, k1 = st == 2 ? 5 : 4, k2 = st == 1 ? 8 : st == 2 ? 6 : 4;
    const int s = k0 * (in[clampi(i - 2, from, to - 1)] + in[clampi(i + 2, from, to - 1)]) +
                  k1 * (in[clampi(i - 1, from, to - 1)] + in[clampi(i + 1, from, to - 1)]) +
                  k2 * in[clampi(i, from, to - 1)];
    return (s + 8) >> 4;
}
// upsample_edge element (src/ipred_tmpl.c:391-406)
template <typename T>
__device__ __forceinline__ int ip_up(const T *in, int o, int hsz, int from, int to, int bdmax) {
    const int i = o >> 1;
    if (!(o & 1) || i >= hsz - 1) return in[clampi(i, from, to - 1)];
    const int s = -in[clampi(i - 1, from, to - 1)] + 9 * in[clampi(i, from, to - 1)] +
                  9 * in[clampi(i + 1, from, to - 1)] - in[clampi(i + 2, from, to - 1)];
    return clampi((s + 8) >> 4, 0, bdmax);
}

// Per-unit intra state after edge preparation.
struct IntraState {
    int mode, up, upl, d1, d2, maxb, dc;
};

// Edge preparation for the directional modes (into fe) and the DC-family
// value; all G lanes of the unit.  tl = topleft pixel in the staged edge.
template <int BPC, int TX, typename P>
__device__ __forceinline__ IntraState intra_prep(const Dav1dGpuUnit &u, const P *tl, int16_t *fe, int l,
                                                 int bdmax) {
    using CL = Cls<TX>;
    constexpr int W = CL::W, H = CL::H, G = CL::G;
    IntraState s{u.p.intra.mode, 0, 0, 0, 0, 0, 0};
    const int ang = u.p.intra.angle & 511, is_sm = (u.p.intra.angle >> 9) & 1, filt = u.p.intra.angle >> 10;
    if (s.mode == DGPU_Z1_PRED) {   // src/ipred_tmpl.c:408-443
        s.d1 = dspt_dr_deriv[ang >> 1];
        s.up = filt ? ip_upsample(W + H, 90 - ang, is_sm) : 0;
        const int st = (!s.up && filt) ? ip_strength(W + H, 90 - ang, is_sm) : 0;
        if (s.up) {
            for (int o = l; o < 2 * (W + H) - 1; o += G) fe[o] = ip_up(tl + 1, o, W + H, -1, W + cmin(W, H), bdmax);
            s.maxb = 2 * (W + H) - 2;
            s.d1 <<= 1;
        } else if (st) {
            for (int i = l; i < W + H; i += G) fe[i] = ip_smooth(tl + 1, i, 0, W + H, -1, W + cmin(W, H), st);
            s.maxb = W + H - 1;
        } else {
            for (int i = l; i < W + cmin(W, H); i += G) fe[i] = tl[1 + i];
            s.maxb = W + cmin(W, H) - 1;
        }
    } else if (s.mode == DGPU_Z3_PRED) {   // src/ipred_tmpl.c:542-581; fe[maxb - i] == left[-i]
        s.d1 = dspt_dr_deriv[(270 - ang) >> 1];
        s.up = filt ? ip_upsample(W + H, ang - 180, is_sm) : 0;
        const int st = (!s.up && filt) ? ip_strength(W + H, ang - 180, is_sm) : 0;
        if (s.up) {
            for (int o = l; o < 2 * (W + H) - 1; o += G)
                fe[o] = ip_up(tl - (W + H), o, W + H, cmax(W - H, 0), W + H + 1, bdmax);
            s.maxb = 2 * (W + H) - 2;
            s.d1 <<= 1;
        } else if (st) {
            for (int i = l; i < W + H; i += G)
                fe[i] = ip_smooth(tl - (W + H), i, 0, W + H, cmax(W - H, 0), W + H + 1, st);
            s.maxb = W + H - 1;
        } else {
            s.maxb = H + cmin(W, H) - 1;
            for (int i = l; i <= s.maxb; i += G) fe[i] = tl[-1 - s.maxb + i];
        }
    } else if (s.mode == DGPU_Z2_PRED) {   // src/ipred_tmpl.c:462-513
        s.d2 = dspt_dr_deriv[(ang - 90) >> 1];   // dy
        s.d1 = dspt_dr_deriv[(180 - ang) >> 1];  // dx
        s.upl = filt ? ip_upsample(W + H, 180 - ang, is_sm) : 0;
        s.up = filt ? ip_upsample(W + H, ang - 90, is_sm) : 0;
        int16_t *c = fe + 2 * H;   // corner
        if (s.up) {
            for (int o = l; o < 2 * W + 1; o += G) c[o] = ip_up(tl, o, W + 1, 0, W + 1, bdmax);
        } else {
            const int st = filt ? ip_strength(W + H, ang - 90, is_sm) : 0;
            for (int i = l; i < W; i += G)
                c[1 + i] = st ? ip_smooth(tl + 1, i, 0, u.p.intra.max_w, -1, W, st) : tl[1 + i];
        }
        if (s.upl) {
            for (int o = l; o < 2 * H + 1; o += G) c[-2 * H + o] = ip_up(tl - H, o, H + 1, 0, H + 1, bdmax);
        } else {
            const int st = filt ? ip_strength(W + H, 180 - ang, is_sm) : 0;
            for (int i = l; i < H; i += G)
                c[-H + i] = st ? ip_smooth(tl - H, i, H - u.p.intra.max_h, H, 0, H + 1, st) : tl[-H + i];
        }
        wave_sync();
        if (l == 0) c[0] = tl[0];
        if (s.up) s.d1 <<= 1;
        if (s.upl) s.d2 <<= 1;
    } else if (s.mode != DGPU_VERT_PRED && s.mode != DGPU_HOR_PRED && s.mode <= DGPU_DC_128_PRED) {
        // DC family: group reduction of the edge sums (src/ipred_tmpl.c:86-166)
        unsigned st = 0, sl = 0;
        for (int i = l; i < W; i += G) st += tl[1 + i];
        for (int i = l; i < H; i += G) sl += tl[-1 - i];
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            st += __shfl_xor(st, off, 64);
            sl += __shfl_xor(sl, off, 64);
        }
        unsigned v;
        if (s.mode == DGPU_DC_128_PRED) v = (bdmax + 1) >> 1;
        else if (s.mode == DGPU_TOP_DC_PRED) v = (st + (W >> 1)) >> __builtin_ctz(W);
        else if (s.mode == DGPU_LEFT_DC_PRED) v = (sl + (H >> 1)) >> __builtin_ctz(H);
        else {
            v = (st + sl + ((W + H) >> 1)) >> __builtin_ctz(W + H);
            if (W != H) {
                const bool r4 = W > 2 * H || H > 2 * W;
                if (BPC == 8) v = (v * (r4 ? 0x3334u : 0x5556u)) >> 16;
                else v = (v * (r4 ? 0x6667u : 0xAAABu)) >> 17;
            }
        }
        s.dc = (int)v;
    }
    return s;
}

// Intra prediction of one 4x2 task (x0 = 4q, rows y0, y0 + 1) into pv[8]
// (row-major), for every mode but FILTER_PRED.
template <int TX, typename P>
__device__ __forceinline__ void intra_task(const IntraState &s, const P *tl, const int16_t *fe, int x0, int y0,
                                           int *pv) {
    using CL = Cls<TX>;
    constexpr int W = CL::W, H = CL::H;
    switch (s.mode) {
    case DGPU_VERT_PRED:
#pragma unroll
        for (int i = 0; i < 8; i++) pv[i] = tl[1 + x0 + (i & 3)];
        break;
    case DGPU_HOR_PRED:
#pragma unroll
        for (int i = 0; i < 8; i++) pv[i] = tl[-(1 + y0 + (i >> 2))];
        break;
    case DGPU_PAETH_PRED: {   // src/ipred_tmpl.c:244-265
        const int c0 = tl[0];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int top = tl[1 + x0 + (i & 3)], left = tl[-(1 + y0 + (i >> 2))];
            const int base = left + top - c0;
            const int dl = abs(left - base), dt = abs(top - base), dd = abs(c0 - base);
            pv[i] = (dl <= dt && dl <= dd) ? left : dt <= dd ? top : c0;
        }
        break;
    }
    case DGPU_SMOOTH_PRED: {   // src/ipred_tmpl.c:267-325
        const int bl = tl[-H], tr = tl[W];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int x = x0 + (i & 3), y = y0 + (i >> 2);
            const int wv = dspt_sm_weights[H + y], wh = dspt_sm_weights[W + x];
            pv[i] = (wv * tl[1 + x] + (256 - wv) * bl + wh * tl[-(1 + y)] + (256 - wh) * tr + 256) >> 9;
        }
        break;
    }
    case DGPU_SMOOTH_V_PRED: {
        const int bl = tl[-H];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int wv = dspt_sm_weights[H + y0 + (i >> 2)];
            pv[i] = (wv * tl[1 + x0 + (i & 3)] + (256 - wv) * bl + 128) >> 8;
        }
        break;
    }
    case DGPU_SMOOTH_H_PRED: {
        const int tr = tl[W];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int wh = dspt_sm_weights[W + x0 + (i & 3)];
            pv[i] = (wh * tl[-(1 + y0 + (i >> 2))] + (256 - wh) * tr + 128) >> 8;
        }
        break;
    }
    case DGPU_Z1_PRED:
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int x = x0 + (i & 3), y = y0 + (i >> 2);
            const int xpos = __mul24(y + 1, s.d1), frac = xpos & 0x3e;
            const int base = (xpos >> 6) + (x << s.up);   // s.up is 0 or 1
            pv[i] = base < s.maxb ? (fe[base] * (64 - frac) + fe[base + 1] * frac + 32) >> 6 : fe[s.maxb];
        }
        break;
    case DGPU_Z3_PRED:
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int x = x0 + (i & 3), y = y0 + (i >> 2);
            const int ypos = __mul24(x + 1, s.d1), frac = ypos & 0x3e;
            const int base = (ypos >> 6) + (y << s.up);
            pv[i] = base < s.maxb ? (fe[s.maxb - base] * (64 - frac) + fe[s.maxb - base - 1] * frac + 32) >> 6
                                  : fe[0];
        }
        break;
    case DGPU_Z2_PRED: {
        const int16_t *c = fe + 2 * H;
        const int16_t *lft = c - (1 + s.upl);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int x = x0 + (i & 3), y = y0 + (i >> 2);
            const int xpos = ((1 + s.up) << 6) - __mul24(y + 1, s.d1);
            const int bx = (xpos >> 6) + (x << s.up);
            int t;
            if (bx >= 0) {
                const int fx = xpos & 0x3e;
                t = c[bx] * (64 - fx) + c[bx + 1] * fx;
            } else {
                const int ypos = (y << (6 + s.upl)) - __mul24(x + 1, s.d2);
                const int by = ypos >> 6, fy = ypos & 0x3e;
                t = lft[-by] * (64 - fy) + lft[-(by + 1)] * fy;
            }
            pv[i] = (t + 32) >> 6;
        }
        break;
    }
    default:   // DC family
#pragma unroll
        for (int i = 0; i < 8; i++) pv[i] = s.dc;
        break;
    }
}

// Filter intra (src/ipred_tmpl.c:617-655): 4x2 cells == output tasks, run in
// anti-diagonal waves, into ptile.
template <int TX, typename P>
__device__ __forceinline__ void filter_intra(const Dav1dGpuUnit &u, const P *tl, int16_t *ptile, int l, int bdmax) {
    using CL = Cls<TX>;
    constexpr int W = CL::W, H = CL::H, G = CL::G, QW = CL::QW, NT = CL::NT;
    constexpr int TPL = (NT + G - 1) / G;
    const signed char *taps = &dspt_filter_intra[(u.p.intra.angle & 511) * 56];
    for (int step = 0; step < QW + H / 2 - 1; step++) {
#pragma unroll
        for (int k = 0; k < TPL; k++) {
            const int t = l + k * G;
            const int cy = t / QW, cx = t % QW;
            if (t < NT && cx + cy == step) {
                const int x = cx * 4, y = cy * 2;
                int p0, p1, p2, p3, p4, p5, p6;
                if (y == 0) {
                    p0 = tl[x];
                    p1 = tl[1 + x]; p2 = tl[2 + x]; p3 = tl[3 + x]; p4 = tl[4 + x];
                } else {
                    const int16_t *upr = ptile + (y - 1) * W + x;
                    p0 = x == 0 ? (int)tl[-y] : upr[-1];
                    p1 = upr[0]; p2 = upr[1]; p3 = upr[2]; p4 = upr[3];
                }
                p5 = x == 0 ? (int)tl[-(y + 1)] : ptile[y * W + x - 1];
                p6 = x == 0 ? (int)tl[-(y + 2)] : ptile[(y + 1) * W + x - 1];
#pragma unroll
                for (int o = 0; o < 8; o++) {
                    const signed char *tk = taps + o * 7;
                    const int acc = tk[0] * p0 + tk[1] * p1 + tk[2] * p2 + tk[3] * p3 + tk[4] * p4 +
                                    tk[5] * p5 + tk[6] * p6;
                    ptile[(y + (o >> 2)) * W + x + (o & 3)] = (int16_t)clampi((acc + 8) >> 4, 0, bdmax);
                }
            }
        }
        wave_sync();
    }
}

// ------------------------------------------------------------------ mc -----

// filter bank for one direction: bilinear (x4), 8-tap, or the 4-tap bank
// for a block extent <= 4 (src/mc_tmpl.c:99-107); m == 0 is the identity
__device__ __forceinline__ int mc_bank(int type, bool bil, int len) {
    return bil ? 5 : len > 4 ? type : 3 + (type & 1);
}

// Horizontal pass of one reference: NH tasks of (row pair p, quad q) ->
// mid[p * W + 4q .. +3] = (row 2p, row 2p+1) int16 pairs.  `org` is the
// footprint origin (block position - 3 rows - 3 columns).  Rows are read
// with unaligned 12-byte (8bpc) / 24-byte (16bpc) loads, one per row and
// quad.  G is a multiple of QW for every class, so a lane's quad is fixed
// and its row pairs advance by G / QW.  Split in steps so the loads of the
// first chunk (all of them below the 64-point classes) are issued together
// with the unit's other loads: init + load(0) ... compute(0) + rest().
template <int BPC, int TX, bool CLAMPABLE = false> struct HPass {
    using CL = Cls<TX>;
    static constexpr int W = CL::W, H = CL::H, G = CL::G, QW = CL::QW, NH = CL::NH, RP = CL::RP;
    static constexpr int IT = (NH + G - 1) / G;
    static constexpr int PS = G / QW;   // row-pair step per task
    static_assert(G % QW == 0, "lane quads must be fixed");
    static constexpr int B = BPC / 8;
    static constexpr int CH = cmin(IT, BPC == 8 ? 3 : 2);   // tasks whose loads are in flight together (2-6: within noise)
    // 8bpc rows are read with dword-aligned loads from the row's dword and
    // realigned in registers (v_alignbyte by the byte skew): the texture
    // path splits an unaligned multi-dword load, measured 2.4-3.3x the cost
    // of an aligned one (tools/probe/ta_rate.hip); 16bpc rows the same way
    // spilled (measured), so they stay unaligned 24-byte loads
    static constexpr bool AL = BPC == 8;
    typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
    using Raw = typename std::conditional<AL, u32x4, typename std::conditional<BPC == 8, u32x3a1, u32x4a2>::type>::type;
    using RawB = typename std::conditional<AL, u32x3, u32x2a2>::type;   // 16bpc: the row's tail
    Raw ra[CH][2];
    RawB rb[CH][2];
    unsigned sh;         // byte skew of the footprint rows (all rows share it; AL only)
    const uint8_t *rp;
    uint32_t *mp;
    unsigned sb;
    int p0;
    int prow;            // the row pair rp points at (p0, or the last one, see init)
    uint4 th;            // taps: 8bpc .x/.y int8 x4, 16bpc int16 pairs

    // CLAMPABLE (the second launch): a DGPU_MX_CLAMP reference, every
    // footprint pixel read at its position clamped to the plane, as
    // emu_edge_c provides them (src/mc_tmpl.c:827-875, src/recon_tmpl.c:
    // 986-999): each of a lane's 12 columns is read at its clamped column,
    // each row at its clamped row (such units are rare: only footprints
    // that leave the picture are flagged).
    bool cl = false;
    int cy0, cxs, cw, chh;   // first footprint row (y - 3), this lane's first column, plane size
    const uint8_t *cbase;    // the plane's (0, 0)
    __device__ __forceinline__ void init_clamp(const typename Px<BPC>::pixel *plane, int stride_px, int w, int h,
                                               int x, int y, uint32_t *mid, int bank, int m, int l) {
        init(plane, stride_px, mid, bank, m, l);
        cl = true;
        const int q = l % QW;
        cbase = reinterpret_cast<const uint8_t *>(plane);
        cy0 = y - 3;
        cxs = x - 3 + 4 * q;
        cw = w;
        chh = h;
        sh = 0;   // the rows are gathered already aligned
    }
    __device__ __forceinline__ void load_clamp(int k0) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            const int p = cmin(p0 + (k0 + c) * PS, RP - 1);
#pragma unroll
            for (int rr = 0; rr < 2; rr++) {
                const int yy = clampi(cy0 + cmin(2 * p + rr, H + 6), 0, chh - 1);
                const uint8_t *row = cbase + (size_t)yy * sb;
                uint32_t w[6];
#pragma unroll
                for (int i = 0; i < (BPC == 8 ? 3 : 6); i++) {
                    uint32_t v = 0;
#pragma unroll
                    for (int j = 0; j < 4 / B; j++) {
                        const int x = clampi(cxs + (4 / B) * i + j, 0, cw - 1);
                        const uint32_t px = BPC == 8 ? (uint32_t)gld<uint8_t>(row + x)
                                                     : (uint32_t)gld<uint16_t>(row + 2 * x);
                        v |= px << (8 * B * j);
                    }
                    w[i] = v;
                }
                if constexpr (BPC == 8) {
                    ra[c][rr][0] = w[0];
                    ra[c][rr][1] = w[1];
                    ra[c][rr][2] = w[2];
                    ra[c][rr][3] = 0;
                } else {
                    ra[c][rr][0] = w[0];
                    ra[c][rr][1] = w[1];
                    ra[c][rr][2] = w[2];
                    ra[c][rr][3] = w[3];
                    rb[c][rr][0] = w[4];
                    rb[c][rr][1] = w[5];
                }
            }
        }
    }
    __device__ __forceinline__ void init(const typename Px<BPC>::pixel *org, int stride_px, uint32_t *mid, int bank,
                                         int m, int l) {
        sb = (unsigned)stride_px * B;
        const int q = l % QW;
        p0 = l / QW;
        // a lane's first row pair; with more lanes than row pairs (PS > RP:
        // DGPU_IE_SMALL_LANES builds) the lanes past the footprint load (and
        // discard) its last pair: load() forms each row as (p - base) * 2
        // rows from rp in unsigned 24-bit arithmetic, which must not go
        // negative (it did, and faulted, before this guard)
        int pb = p0;
        if constexpr (PS > RP) pb = cmin(p0, RP - 1);
        prow = pb;
        rp = reinterpret_cast<const uint8_t *>(org) + (size_t)__umul24(2u * pb, sb) + 4 * B * q;
        sh = 0;
        if constexpr (AL) {
            sh = (unsigned)reinterpret_cast<uintptr_t>(rp) & 3u;   // strides are dword multiples (launch check)
            rp -= sh;
        }
        mp = mid + p0 * W + 4 * q;
        if constexpr (BPC == 8) {
            const uint2 t = reinterpret_cast<const uint2 *>(dspt_mc8)[bank * 16 + m];
            th = make_uint4(t.x, t.y, 0, 0);
        } else {
            th = reinterpret_cast<const uint4 *>(dspt_mc16)[bank * 16 + m];
        }
    }
    __device__ __forceinline__ void load(int k0) {
        if constexpr (CLAMPABLE) {
            if (cl) {
                load_clamp(k0);
                return;
            }
        }
#pragma unroll
        for (int c = 0; c < CH; c++) {   // clamped: the loads stay inside the footprint
            const int pu = p0 + (k0 + c) * PS;
            const int p = cmin(pu, RP - 1);
            // every footprint row is loaded, also those no vertical tap reads
            // (skipping them measured slower: 60 -> 63 us with a spill)
            const uint8_t *a0 = rp + (size_t)__umul24((unsigned)(p - (PS > RP ? prow : p0)) * 2u, sb);
            // row 2p+1 == H+7 (last pair) is never used: re-read row 2p
            const uint8_t *a1 = 2 * p + 1 < H + 7 ? a0 + sb : a0;
            ra[c][0] = gld<Raw>(a0);
            ra[c][1] = gld<Raw>(a1);
            if constexpr (BPC == 16) {
                rb[c][0] = gld<RawB>(a0 + 16);
                rb[c][1] = gld<RawB>(a1 + 16);
            }
        }
    }
    __device__ __forceinline__ void compute(int k0, int ib) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            const int p = p0 + (k0 + c) * PS;
            if (k0 + c < IT && p < RP) {
                int mm[2][4];
#pragma unroll
                for (int rr = 0; rr < 2; rr++) {
                    if constexpr (BPC == 8) {
                        // taps sum to 64 and p ^ 0x80 == p - 128 as int8: s = acc + 128 * 64,
                        // and the reference's mid = (s + 2) >> 2 (intermediate_bits 4) is
                        // stored as mid - 2048 = (acc + 2) >> 2; the vertical pass adds back
                        // 64 * 2048 (kMidBias).  Both forms fit int16 for 8-bit input.
                        uint32_t w0 = ra[c][rr].x, w1 = ra[c][rr].y, w2 = ra[c][rr].z;
                        if constexpr (AL) {
                            w0 = alb(ra[c][rr].y, ra[c][rr].x, sh);
                            w1 = alb(ra[c][rr].z, ra[c][rr].y, sh);
                            w2 = alb(ra[c][rr][3], ra[c][rr].z, sh);
                        }
                        w0 ^= 0x80808080u;
                        w1 ^= 0x80808080u;
                        w2 ^= 0x80808080u;
                        const uint32_t lo[4] = {w0, alb(w1, w0, 1), alb(w1, w0, 2), alb(w1, w0, 3)};
                        const uint32_t hi[4] = {w1, alb(w2, w1, 1), alb(w2, w1, 2), alb(w2, w1, 3)};
                        hdot4x4(lo, hi, th.x, th.y, mm[rr]);
                    } else {
                        const int sh = 6 - ib, rnd = (1 << sh) >> 1;
                        // e: pixel pairs (2i, 2i+1), o: (2i+1, 2i+2)
                        uint32_t e[6] = {ra[c][rr][0], ra[c][rr][1], ra[c][rr][2], ra[c][rr][3],
                                         rb[c][rr][0], rb[c][rr][1]};
                        if constexpr (AL) {
                            const uint32_t d[7] = {ra[c][rr][0], ra[c][rr][1], ra[c][rr][2], ra[c][rr][3],
                                                   rb[c][rr][0], rb[c][rr][1], rb[c][rr][2]};
#pragma unroll
                            for (int i = 0; i < 6; i++) e[i] = alb(d[i + 1], d[i], sh);
                        }
                        uint32_t o[5];
#pragma unroll
                        for (int i = 0; i < 5; i++) o[i] = alb(e[i + 1], e[i], 2);
                        mm[rr][0] = (dot2(e[3], th.w, dot2(e[2], th.z, dot2(e[1], th.y, dot2(e[0], th.x, 0)))) + rnd) >> sh;
                        mm[rr][1] = (dot2(o[3], th.w, dot2(o[2], th.z, dot2(o[1], th.y, dot2(o[0], th.x, 0)))) + rnd) >> sh;
                        mm[rr][2] = (dot2(e[4], th.w, dot2(e[3], th.z, dot2(e[2], th.y, dot2(e[1], th.x, 0)))) + rnd) >> sh;
                        mm[rr][3] = (dot2(o[4], th.w, dot2(o[3], th.z, dot2(o[2], th.y, dot2(o[1], th.x, 0)))) + rnd) >> sh;
                    }
                }
                uint4 o;
                o.x = pack16(mm[0][0], mm[1][0]);
                o.y = pack16(mm[0][1], mm[1][1]);
                o.z = pack16(mm[0][2], mm[1][2]);
                o.w = pack16(mm[0][3], mm[1][3]);
                *reinterpret_cast<uint4 *>(mp + (k0 + c) * PS * W) = o;
            }
        }
    }
    __device__ __forceinline__ void rest(int ib) {   // chunks after the first (64-point classes)
#pragma unroll
        for (int k0 = CH; k0 < IT; k0 += CH) {
            load(k0);
            compute(k0, ib);
        }
    }
};

// Vertical pass of one reference for a 4x2 task: t[i] = (the 8-tap sum over
// stored intermediates + kk) >> sh, rows j*2 (i < 4) and j*2+1 (i >= 4),
// columns 4q + (i & 3).  kk includes kMidBias<BPC> (the reference's sum is
// the stored one + kMidBias).
template <int BPC> inline constexpr int kMidBias = BPC == 8 ? 64 * 2048 : 0;
template <int W>
__device__ __forceinline__ void mc_vtask(const uint32_t *mid, int j, int q, const uint4 tv, int kk, int sh, int *t) {
    uint32_t P[5][4];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint4 v = *reinterpret_cast<const uint4 *>(mid + (j + k) * W + 4 * q);
        P[k][0] = v.x; P[k][1] = v.y; P[k][2] = v.z; P[k][3] = v.w;
    }
    vdot4x4(P, tv, kk, sh, t);
    uint32_t so[5];   // odd rows: the same pairs with shifted taps (vtaps_odd)
    vtaps_odd(tv, so);
    vdot5x4(P, so, kk, sh, t + 4);
}

// ------------------------------------------------------------------ cfl ---


// Chroma-from-luma for one unit (the whole chroma block, square <= 32):
// cfl_ac on the co-located luma (src/ipred_tmpl.c:657-703), then cfl_pred
// with the DC of the edge array (:71-84, :103-218), task by task through
// `emit`.  The 4:2:0 no-padding case sums luma pairs with packed dots.
template <int BPC, int TX, typename P, typename Emit>
__device__ __forceinline__ void cfl_units(const ReconArgs<BPC> &a, const Dav1dGpuUnit &u, const P *tl, int16_t *fe,
                                          int l, int bdmax, Emit &emit) {
    using CL = Cls<TX>;
    constexpr int W = CL::W, H = CL::H, G = CL::G, QW = CL::QW, NT = CL::NT, TPL = CL::TPL;
    const IntraState dcs = intra_prep<BPC, TX>(u, tl, fe, l, bdmax);   // DC family only reads tl
    const int ssh = a.cfl_ss & 1, ssv = (a.cfl_ss >> 1) & 1;
    const int wpad = u.p.cfl.pad_wh & 15, hpad = u.p.cfl.pad_wh >> 4;
    const int vw = W - 4 * wpad, vh = H - 4 * hpad;
    const int ys = a.cfl_luma_stride;
    const P *yp = a.cfl_luma + u.p.cfl.luma_off;
    const bool fast = ssh && ssv && !wpad && !hpad;
    const int acsh = 1 + !ssv + !ssh;
    int ac[TPL][8];
    int sum = 0;
#pragma unroll
    for (int k = 0; k < TPL; k++) {
        const int t = l + k * G;
        if (t >= NT) break;
        const int j = t / QW, q = t % QW;
        if (fast) {   // luma rows 4j..4j+3, columns 8q..8q+7
#pragma unroll
            for (int rr = 0; rr < 2; rr++) {
                const P *r0 = yp + __mul24(4 * j + 2 * rr, ys) + 8 * q;
                if constexpr (BPC == 8) {
                    const u32x2 v0 = gld<u32x2a1>(r0), v1 = gld<u32x2a1>(r0 + ys);
                    // byte pairs summed over both rows: dot4 with 1-masks
                    ac[k][4 * rr + 0] = (int)__builtin_amdgcn_udot4(v1.x, 0x00000101u, __builtin_amdgcn_udot4(v0.x, 0x00000101u, 0, false), false) << 1;
                    ac[k][4 * rr + 1] = (int)__builtin_amdgcn_udot4(v1.x, 0x01010000u, __builtin_amdgcn_udot4(v0.x, 0x01010000u, 0, false), false) << 1;
                    ac[k][4 * rr + 2] = (int)__builtin_amdgcn_udot4(v1.y, 0x00000101u, __builtin_amdgcn_udot4(v0.y, 0x00000101u, 0, false), false) << 1;
                    ac[k][4 * rr + 3] = (int)__builtin_amdgcn_udot4(v1.y, 0x01010000u, __builtin_amdgcn_udot4(v0.y, 0x01010000u, 0, false), false) << 1;
                } else {
                    const u32x4 v0 = gld<u32x4a2>(r0), v1 = gld<u32x4a2>(r0 + ys);
                    const uint32_t d0[4] = {v0.x, v0.y, v0.z, v0.w}, d1[4] = {v1.x, v1.y, v1.z, v1.w};
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        ac[k][4 * rr + i] = (int)((d0[i] & 0xffff) + (d0[i] >> 16) + (d1[i] & 0xffff) + (d1[i] >> 16)) << 1;
                }
            }
        } else {   // general: clamp to the visible part, any subsampling
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int sx = min(4 * q + (i & 3), vw - 1), sy = min(2 * j + (i >> 2), vh - 1);
                const P *p = yp + __mul24(sy << ssv, ys) + (sx << ssh);
                int v = gld<P>(p);
                if (ssh) v += gld<P>(p + 1);
                if (ssv) {
                    v += gld<P>(p + ys);
                    if (ssh) v += gld<P>(p + ys + 1);
                }
                ac[k][i] = v << acsh;
            }
        }
#pragma unroll
        for (int i = 0; i < 8; i++) sum += ac[k][i];
    }
#pragma unroll
    for (int off = 1; off < G; off <<= 1) sum += __shfl_xor(sum, off, 64);
    constexpr int LG = __builtin_ctz(W) + __builtin_ctz(H);
    const int avg = (sum + ((1 << LG) >> 1)) >> LG;
    const int alpha = u.p.cfl.alpha;
#pragma unroll
    for (int k = 0; k < TPL; k++) {
        const int t = l + k * G;
        if (t >= NT) break;
        int pv[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int d = alpha * (int)(int16_t)(ac[k][i] - avg);   // ac is int16 in the reference
            const int mag = (abs(d) + 32) >> 6;
            pv[i] = clampi(dcs.dc + (d < 0 ? -mag : mag), 0, bdmax);
        }
        emit(t / QW, t % QW, pv);
    }
}

// The visible size of reference plane (r, plane), by a lane-varying index
// straight from the kernel-argument segment (indexing the by-value argument
// would copy all of it to scratch).  Only for code that runs in k_recon,
// whose argument is the ReconArgs (the second launch's kinds).
template <int BPC> __device__ __forceinline__ void ref_plane_wh(int r, int plane, int &rw, int &rh) {
#if defined(__HIP_DEVICE_COMPILE__)
    const __attribute__((address_space(4))) int *ka =
        (const __attribute__((address_space(4))) int *)__builtin_amdgcn_kernarg_segment_ptr();
    rw = ka[(offsetof(ReconArgs<BPC>, ref_w) >> 2) + r * 3 + plane];
    rh = ka[(offsetof(ReconArgs<BPC>, ref_h) >> 2) + r * 3 + plane];
#else
    rw = rh = 1;
#endif
}
// A pixel of a plane at (x, y) clamped to its visible w x h (emu_edge_c,
// src/mc_tmpl.c:827-875); `base` is the plane's (0, 0), `sb` its pitch in bytes
template <typename P>
__device__ __forceinline__ uint32_t clamped_px(const uint8_t *base, unsigned sb, int x, int y, int w, int h) {
    return (uint32_t)gld<P>(reinterpret_cast<const P *>(base + (size_t)__umul24((unsigned)clampi(y, 0, h - 1), sb)) +
                            clampi(x, 0, w - 1));
}

// ----------------------------------------------------------------- warp ---

// One WARP unit (w, h multiples of 8): warp_affine_8x8_c (src/mc_tmpl.c:
// 758-791) for each of its 8x8s, 8 rows at a time.  Per strip the 15 x W
// horizontal intermediates (each column with its own filter) go to the
// unit's LDS mid area; then each 4x2 task takes its 8 vertical taps per
// output from it and is emitted (+ residual) like every other prediction.
template <int BPC, int TX, typename P, typename Emit>
__device__ __forceinline__ void warp_unit(const ReconArgs<BPC> &a, const PlaneTab<BPC> &pt, const Dav1dGpuUnit &u,
                                          int auxo, int16_t *mid, const uint2 *wtab, int l, int bdmax, Emit &emit) {
    using CL = Cls<TX>;
    constexpr int W = CL::W, H = CL::H, G = CL::G, QW = CL::QW, NBX = W / 8;
    const uint8_t *rec = a.aux_pool + auxo;
    const u32x2 abcd = gld<u32x2>(rec);
    const int a0 = (int16_t)(abcd[0] & 0xffff), a1 = (int)abcd[0] >> 16;
    const int a2 = (int16_t)(abcd[1] & 0xffff), a3 = (int)abcd[1] >> 16;
    const int ri = u.p.inter.ref[0] * 3 + u.plane;
    // src_off[0]: a base the 8x8 positions are relative to (0, or the
    // recorder's clamped-copy strip in its scratch plane); with
    // DGPU_MX_CLAMP in mx[0] (round 6) the positions are the plane's own and
    // every footprint pixel is read clamped to it, as warp_affine's
    // emu_edge call provides it (src/recon_tmpl.c:1168-1177)
    const bool clamp = u.p.inter.mx[0] & DGPU_MX_CLAMP;
    const P *ref = pt.ref[ri] + (clamp ? 0 : u.p.inter.src_off[0]);
    const int rs = pt.ref_stride[ri];
    int cw = 1, ch = 1;
    if (clamp) ref_plane_wh<BPC>(u.p.inter.ref[0], u.plane, cw, ch);
    const int ib = Px<BPC>::ibits(bdmax);
    const int hsh = 7 - ib, hrnd = (1 << hsh) >> 1;
    constexpr int NHT = 15 * QW, NVT = 4 * QW;
#pragma unroll 1
    for (int sy = 0; sy < H / 8; sy++) {
        // horizontal: (row, quad) tasks; every task's source row and
        // parameters are loaded first (all in flight together), then computed
        constexpr int KH = (NHT + G - 1) / G;
        using Raw = typename std::conditional<BPC == 8, u32x4, u32x4a2>::type;
        Raw raw[KH];
        u32x2a2 raw2[KH];   // 16bpc: pixels 8..11
        int mxs[KH];
        unsigned shs[KH];
#pragma unroll
        for (int k = 0; k < KH; k++) {
            const int t = cmin(l + k * G, NHT - 1);   // clamped: loads stay inside the footprint
            const int row = t / QW, q = t % QW, x0 = (q & 1) * 4;
            const u32x2 sb = gld<u32x2>(rec + 16 + 8 * (sy * NBX + (q >> 1)));
            mxs[k] = (int)(int16_t)(sb[1] & 0xffff) * 64;
            const int wx = (int16_t)(sb[0] & 0xffff), wy = (int)sb[0] >> 16;   // the 8x8's source position
            const P *s = ref + (wy + row - 3) * rs + wx + x0 - 3;   // columns x0-3 .. x0+7
            if (clamp) {   // the 12 pixels gathered at clamped positions, already aligned
                const uint8_t *b = reinterpret_cast<const uint8_t *>(ref);
                const unsigned sbb = (unsigned)rs * sizeof(P);
                const int yy = wy + row - 3, xx = wx + x0 - 3;
                uint32_t w[6];
#pragma unroll
                for (int i = 0; i < (BPC == 8 ? 3 : 6); i++) {
                    uint32_t v = 0;
#pragma unroll
                    for (int j = 0; j < 4 / (int)sizeof(P); j++)
                        v |= clamped_px<P>(b, sbb, xx + (4 / (int)sizeof(P)) * i + j, yy, cw, ch) << (8 * sizeof(P) * j);
                    w[i] = v;
                }
                shs[k] = 0;
                if constexpr (BPC == 8) {
                    raw[k] = u32x4{w[0], w[1], w[2], 0};
                } else {
                    raw[k] = u32x4a2{w[0], w[1], w[2], w[3]};
                    raw2[k] = u32x2a2{w[4], w[5]};
                }
            } else if constexpr (BPC == 8) {
                shs[k] = (unsigned)reinterpret_cast<uintptr_t>(s) & 3u;
                raw[k] = gld<u32x4>(reinterpret_cast<const uint8_t *>(s) - shs[k]);
            } else {
                shs[k] = 0;
                raw[k] = gld<u32x4a2>(s);
                raw2[k] = gld<u32x2a2>(s + 8);
            }
        }
#pragma unroll
        for (int k = 0; k < KH; k++) {
            const int t = l + k * G;
            if (t < NHT) {
                const int row = t / QW, q = t % QW, x0 = (q & 1) * 4;
                const int mx = mxs[k];
                int m4[4];
                if constexpr (BPC == 8) {
                    const u32x4 d = raw[k];
                    const unsigned sh = shs[k];
                    const uint32_t w0 = alb(d[1], d[0], sh) ^ 0x80808080u, w1 = alb(d[2], d[1], sh) ^ 0x80808080u,
                                   w2 = alb(d[3], d[2], sh) ^ 0x80808080u;
                    const uint32_t lo[4] = {w0, alb(w1, w0, 1), alb(w1, w0, 2), alb(w1, w0, 3)};
                    const uint32_t hi[4] = {w1, alb(w2, w1, 1), alb(w2, w1, 2), alb(w2, w1, 3)};
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int pos = mx + row * a1 + (x0 + i) * a0;
                        const uint2 kt = wtab[64 + ((pos + 512) >> 10)];
                        // taps sum to 128 and p ^ 0x80 == p - 128: sum = acc + 128 * 128
                        m4[i] = (dot4(hi[i], kt.y, dot4(lo[i], kt.x, 16384 + hrnd))) >> hsh;
                    }
                } else {
                    const uint32_t e[6] = {raw[k].x, raw[k].y, raw[k].z, raw[k].w, raw2[k].x, raw2[k].y};
                    uint32_t o[5];
#pragma unroll
                    for (int i = 0; i < 5; i++) o[i] = alb(e[i + 1], e[i], 2);   // pairs (2m+1, 2m+2)
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int pos = mx + row * a1 + (x0 + i) * a0;
                        const uint2 kt = wtab[64 + ((pos + 512) >> 10)];
                        uint32_t tp[4];   // int8 taps -> int16 pairs
#pragma unroll
                        for (int m = 0; m < 4; m++) {
                            const uint32_t src = m < 2 ? kt.x : kt.y;
                            const int b0 = __builtin_amdgcn_sbfe((int)src, 16 * (m & 1), 8);
                            const int b1 = __builtin_amdgcn_sbfe((int)src, 16 * (m & 1) + 8, 8);
                            tp[m] = pack16(b0, b1);
                        }
                        const uint32_t *pp = (i & 1) ? o + (i >> 1) : e + (i >> 1);
                        const int acc = dot2(pp[3], tp[3], dot2(pp[2], tp[2], dot2(pp[1], tp[1], dot2(pp[0], tp[0], 0))));
                        m4[i] = (acc + hrnd) >> hsh;
                    }
                }
                uint2 ov;
                ov.x = pack16(m4[0], m4[1]);
                ov.y = pack16(m4[2], m4[3]);
                *reinterpret_cast<uint2 *>(mid + row * W + 4 * q) = ov;
            }
        }
        wave_sync();
#pragma unroll 1
        for (int k = 0; k < (NVT + G - 1) / G; k++) {   // vertical + emit: 4x2 tasks of the strip
            const int t = l + k * G;
            if (t < NVT) {
                const int j = t / QW, q = t % QW, x0 = (q & 1) * 4;
                const u32x2 sb = gld<u32x2>(rec + 16 + 8 * (sy * NBX + (q >> 1)));
                const int my = ((int)sb[1] >> 16) * 64;
                // the 8 outputs' vertical taps, then the 9 mid rows streamed
                // through the 8 accumulators (few live registers)
                u32x2 kv[2][4];
#pragma unroll
                for (int rr = 0; rr < 2; rr++)
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int pos = my + (2 * j + rr) * a3 + (x0 + i) * a2;
                        const uint2 t2 = wtab[64 + ((pos + 512) >> 10)];
                        kv[rr][i] = u32x2{t2.x, t2.y};
                    }
                int sum[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
                for (int r = 0; r < 9; r++) {
                    const uint2 v = *reinterpret_cast<const uint2 *>(mid + (2 * j + r) * W + 4 * q);
                    const int m[4] = {(int16_t)(v.x & 0xffff), (int)v.x >> 16, (int16_t)(v.y & 0xffff), (int)v.y >> 16};
#pragma unroll
                    for (int rr = 0; rr < 2; rr++) {
                        const int kk = r - rr;
                        if (kk < 0 || kk > 7) continue;
#pragma unroll
                        for (int i = 0; i < 4; i++)
                            sum[rr][i] += __builtin_amdgcn_sbfe((int)kv[rr][i][kk >> 2], 8 * (kk & 3), 8) * m[i];
                    }
                }
                int pv[8];
#pragma unroll
                for (int rr = 0; rr < 2; rr++)
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        pv[4 * rr + i] = clampi((sum[rr][i] + ((1 << (7 + ib)) >> 1)) >> (7 + ib), 0, bdmax);
                emit(4 * sy + j, q, pv);
            }
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------- kernel --

struct NoWait {
    __device__ __forceinline__ void operator()() const {}
};

// DGPU_LANE_OPAQUE (the superblock wavefront's TUs, recon_sb*.hip): the lane
// id from an asm the compiler cannot move, so nothing lane-derived is hoisted
// out of their task loops (hoisted across 19 class bodies it spills)
#ifndef DGPU_LANE_OPAQUE
#define DGPU_LANE_OPAQUE 0
#endif
__device__ __forceinline__ int unit_lane() {
    if constexpr (DGPU_LANE_OPAQUE) {
        int l;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
        return l;
    } else {
        return threadIdx.x & 63;
    }
}

template <int BPC, int TX, bool WARPK, bool GATHER = false, typename WaitT = NoWait>
__device__ __forceinline__ void recon_units(const ReconArgs<BPC> &a, const PlaneTab<BPC> &pt,
                                            const Dav1dGpuUnit &u_in, const Dav1dGpuIntraEdge &rec, int first,
                                            int count, uint8_t *wave_lds, int gw, int grp,
                                            const WaitT &wait = WaitT()) {
    using CL = Cls<TX>;
    using SL = Slot<BPC, TX>;
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    using TT = typename Tmp<BPC>::T;
    constexpr int W = CL::W, H = CL::H, SW = CL::SW, SH = CL::SH, G = CL::G, QW = CL::QW, NT = CL::NT;
    constexpr int TPL = CL::TPL;
    const int lane = unit_lane();
    const int g = lane / G, l = lane % G;
    if (g >= count) return;
    // DGPU_TRACE: timestamp phase i after draining this wave's memory ops
    auto mark = [&](int i) {
        if constexpr (DGPU_TRACE) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            // DGPU_TRACE_RT: the 100 MHz clock of the flow trace instead of the core clock
            const unsigned long long t = DGPU_TRACE_RT ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
            if (lane == 0) a.trace[((size_t)grp << 20) + (size_t)gw * 16 + i] = t;
        }
    };
    mark(0);

    Dav1dGpuUnit ug = u_in;   // GATHER: the edge stage rewrites its mode / angle
    const Dav1dGpuUnit &u = GATHER ? ug : u_in;
    mark(1);   // the descriptor was loaded by the kernel prologue (lane's unit = first + g)
    uint8_t *slot = wave_lds + g * (WARPK ? SL::BYTES_W : SL::BYTES);
    uint8_t *cfl = slot;                                           // staged coefs, then residual
    TT *res = reinterpret_cast<TT *>(slot);
    TT *tmp = reinterpret_cast<TT *>(slot + SL::CFR);
    uint8_t *src = slot + SL::CFR + SL::TMP;
    uint32_t *mid0 = reinterpret_cast<uint32_t *>(src);
    uint32_t *mid1 = reinterpret_cast<uint32_t *>(src + (CL::SEQREF ? 0 : SL::MID));
    int16_t *fe = reinterpret_cast<int16_t *>(src + SL::EB);
    int16_t *ptile = reinterpret_cast<int16_t *>(src + SL::EB);

    const int plane = u.plane;
    const int bdmax = a.bdmax;
    const int ib = Px<BPC>::ibits(bdmax);
    const int pred = u.pred;
    const bool comp = pred == DGPU_PRED_INTER_AVG || pred == DGPU_PRED_INTER_WAVG || pred == DGPU_PRED_INTER_MASK;
    // inter-intra: the second launch (staged edges) and the wavefront (GATHER:
    // its edges from the picture, for the recorder); never the main kernel
    const bool ii = (WARPK || GATHER) && pred == DGPU_PRED_INTER_INTRA;
    const bool inter = pred == DGPU_PRED_INTER || comp || ii;
    const int txtp = u.txtp;
    const bool nores = txtp == DGPU_NO_RESIDUAL;
    const int nzw = u.nzw, nzh = u.nzh;
    const bool dconly = !nores && nzw == 0;
    const bool haveres = !nores && !dconly;
    // WHT_WHT (lossless, 4x4 units only): one lane runs both passes below
    const bool wht = W == 4 && H == 4 && txtp == DGPU_WHT_WHT;
    P *dstp = pt.dst[plane] + u.dst_off;
    const int ds = pt.dst_stride[plane];

    // ---------------- P1: every global load of the unit, then the LDS commits --------------
    // (coefficients, intra edges and the first ref's footprint rows are in
    // flight together: one memory round trip after the descriptor)
    C *cf = a.coef + u.coef_off;
    const int ncoef = nores ? 0 : dconly ? 1 : nzw * nzh;
    Stage<CL::SW * CL::SH * (int)sizeof(C), G> cst;
    if (ncoef) cst.load(cf, ncoef * (int)sizeof(C), l);
    Stage<SL::EDGE * (int)sizeof(P), G> est;
    constexpr bool NW = !WARPK;   // the warp launch compiles only the WARP prediction
    const bool edged = NW && (pred == DGPU_PRED_INTRA || pred == DGPU_PRED_CFL);   // same edge_off in both views
    if (edged && !GATHER) est.load(a.edges + u.p.intra.edge_off - 2 * H, SL::EDGE * (int)sizeof(P), l);
    // read for every unit (only inter kinds use it; the bank math below stays
    // in range for any byte).  Selecting it on `inter` gave inter-intra units
    // Filter2d 0 in the second launch's kernel (measured on MI355X, cause
    // not isolated), so no select.
    const int f2d = u.p.inter.filter2d;
    const bool bil = f2d == DGPU_FILTER_2D_BILINEAR;
    // filter_type = type_h | type_v << 2 per Filter2d (src/mc_tmpl.c:376-384)
    const int ftype = bil ? 0 : (int)((0x951a62840ull >> (4 * f2d)) & 15);
    const int bw = u.bw4 * 4, bh = u.bh4 * 4;
    const int bank_h = mc_bank(ftype & 3, bil, bw), bank_v = mc_bank(ftype >> 2, bil, bh);
    const uint4 tv0 = inter ? reinterpret_cast<const uint4 *>(dspt_mc16)[bank_v * 16 + u.p.inter.my[0]]
                            : make_uint4(0, 0, 0, 0);
    const uint4 tv1 = comp ? reinterpret_cast<const uint4 *>(dspt_mc16)[bank_v * 16 + u.p.inter.my[1]]
                           : make_uint4(0, 0, 0, 0);
    using HP = HPass<BPC, TX, WARPK>;   // the second launch also runs DGPU_MX_CLAMP units
    auto hinit = [&](HP &hp, int k) {
        const int r = k ? u.p.inter.ref[1] : u.p.inter.ref[0];
        const int rs = pt.ref_stride[r * 3 + plane];
        if constexpr (WARPK) {
            const int mx = k ? u.p.inter.mx[1] : u.p.inter.mx[0];
            if (mx & DGPU_MX_CLAMP) {   // src_off = x | y << 16 (int16 each), the unit's top-left in the plane
                const int so = k ? u.p.inter.src_off[1] : u.p.inter.src_off[0];
                // the plane size by a lane-varying index straight from the
                // kernel-argument segment (indexing the by-value argument
                // would copy all of it to scratch); WARPK code runs only in
                // k_recon, whose argument `a` is
                int rw = 0, rh = 0;
#if defined(__HIP_DEVICE_COMPILE__)
                {
                    const __attribute__((address_space(4))) int *ka =
                        (const __attribute__((address_space(4))) int *)__builtin_amdgcn_kernarg_segment_ptr();
                    rw = ka[(offsetof(ReconArgs<BPC>, ref_w) >> 2) + r * 3 + plane];
                    rh = ka[(offsetof(ReconArgs<BPC>, ref_h) >> 2) + r * 3 + plane];
                }
#endif
                hp.init_clamp(pt.ref[r * 3 + plane], rs, rw, rh, (int)(int16_t)(so & 0xffff), so >> 16,
                              k ? mid1 : mid0, bank_h, mx & 15, l);
                return;
            }
        }
        const P *org = pt.ref[r * 3 + plane] + (k ? u.p.inter.src_off[1] : u.p.inter.src_off[0]) - 3 * rs - 3;
        hp.init(org, rs, k ? mid1 : mid0, bank_h, (k ? u.p.inter.mx[1] : u.p.inter.mx[0]) & (WARPK ? 15 : 255), l);
    };
    auto hpass = [&](int k) {   // the whole h-pass of ref k
        HP hp;
        hinit(hp, k);
        hp.load(0);
        hp.compute(0, ib);
        hp.rest(ib);
    };
    const bool do_mc = inter;   // (WARPK: inter-intra and DGPU_MX_CLAMP inter units)
    HP hp0;
    if (do_mc) {
        hinit(hp0, 0);
        hp0.load(0);
    }
    // INTER_MASK / PAL: the unit's aux_pool offset (mask / palette record)
    const bool auxed = pred == DGPU_PRED_INTER_MASK || pred == DGPU_PRED_PAL || pred == DGPU_PRED_WARP || ii;
    const int auxo = auxed ? bld(a.aux + first + g) : 0;
    int cfsk = 0;
    if (ncoef) cfsk = cst.commit(cfl, l);
    const P *tl = nullptr;
    if (edged) tl = GATHER ? reinterpret_cast<const P *>(src) + 2 * H
                           : reinterpret_cast<const P *>(src + est.commit(src, l)) + 2 * H;
    mark(2);

    // ---------------- P2: mc horizontal pass(es) ----------------
    if (do_mc) {
        hp0.compute(0, ib);
        hp0.rest(ib);
        if (!CL::SEQREF && comp) hpass(1);
    }
    wave_sync();
    mark(3);

    // coefficient zeroing (the reference's itx zeroes what it consumed,
    // src/itx_tmpl.c:55/89); loads above completed before the LDS writes
    if (a.zero_coefs && ncoef)
        for (int i = l; i < ncoef; i += G) bst<C>(cf + i, 0);

    // ---------------- P3: row transforms -> tmp [SH][W] ----------------
    int dcres = 0;
    if (dconly) {   // src/itx_tmpl.c:53-65
        int dc = reinterpret_cast<const C *>(cfl + cfsk)[0];
        if (CL::RECT2) dc = r8s(dc);
        dc = r8s(dc);
        dc = (dc + ((1 << CL::SHIFT) >> 1)) >> CL::SHIFT;
        dcres = (dc * 181 + 128 + 2048) >> 12;
    }
    const Clip rc = ItxClip<BPC>::row(bdmax), cc = ItxClip<BPC>::col(bdmax);
    if (haveres && !wht) {
        const C *cs = reinterpret_cast<const C *>(cfl + cfsk);
#pragma unroll
        for (int k = 0; k < (SH + G - 1) / G; k++) {
            const int r = l + k * G;
            if (r < SH) {
                TT *trow = tmp + r * W;
                if (r < nzh) {
                    int c[W];
#pragma unroll
                    for (int x = 0; x < W; x++) {
                        int v = 0;
                        if (x < SW) {
                            v = cs[x * nzh + r];
                            v = x < nzw ? v : 0;
                        }
                        c[x] = CL::RECT2 ? r8s(v) : v;
                    }
                    tx1d<W, 1, BPC == 8>(kind_h(txtp), c, rc);
                    constexpr int RND = (1 << CL::SHIFT) >> 1;
#pragma unroll
                    for (int x = 0; x < W; x++) c[x] = cc((c[x] + RND) >> CL::SHIFT);
                    if constexpr (BPC == 8) {
#pragma unroll
                        for (int x = 0; x < W; x += 4) {
                            uint2 o;
                            o.x = pack16(c[x], c[x + 1]);
                            o.y = pack16(c[x + 2], c[x + 3]);
                            *reinterpret_cast<uint2 *>(trow + x) = o;
                        }
                    } else {
#pragma unroll
                        for (int x = 0; x < W; x += 4)
                            *reinterpret_cast<int4 *>(trow + x) = make_int4(c[x], c[x + 1], c[x + 2], c[x + 3]);
                    }
                } else {
#pragma unroll
                    for (int x = 0; x < W * (int)sizeof(TT); x += 8)
                        *reinterpret_cast<uint2 *>(reinterpret_cast<uint8_t *>(trow) + x) = make_uint2(0, 0);
                }
            }
        }
    }
    wave_sync();

    mark(4);
    // ---------------- P4: column transforms -> residual [W][H] ----------------
    if constexpr (W == 4 && H == 4) {
        if (wht && l == 0) {   // the staged coefficients are read before the residual overwrites them
            int t[16];
            wht4x4(reinterpret_cast<const C *>(cfl + cfsk), nzw, nzh, t);
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 4; y++)
                    res[x * SL::RS + y] = (TT)(BPC == 8 ? clampi(t[4 * y + x], -32768, 32767) : t[4 * y + x]);
        }
    }
    if (haveres && !wht) {
#pragma unroll
        for (int k = 0; k < (W + G - 1) / G; k++) {
            const int x = l + k * G;
            if (x < W) {
                int col[H];
#pragma unroll
                for (int y = 0; y < H; y++) col[y] = y < SH ? (int)tmp[y * W + x] : 0;
                tx1d<H, 1, BPC == 8>(kind_v(txtp), col, cc);
                TT *rcol = res + x * SL::RS;
                if constexpr (BPC == 8) {
#pragma unroll
                    for (int y = 0; y < H; y += 4) {
                        uint2 o;
                        o.x = pack16((col[y] + 8) >> 4, (col[y + 1] + 8) >> 4);
                        o.y = pack16((col[y + 2] + 8) >> 4, (col[y + 3] + 8) >> 4);
                        *reinterpret_cast<uint2 *>(rcol + y) = o;
                    }
                } else {
#pragma unroll
                    for (int y = 0; y < H; y += 4)
                        *reinterpret_cast<int4 *>(rcol + y) =
                            make_int4((col[y] + 8) >> 4, (col[y + 1] + 8) >> 4, (col[y + 2] + 8) >> 4,
                                      (col[y + 3] + 8) >> 4);
                }
            }
        }
    }

    wave_sync();
    // GATHER: the edges come last, after the coefficient loads and both
    // transform passes, which need nothing from the neighbours; `wait` (the
    // persistent kernel's level wait) is the first point that does, so a
    // wave does all of that while the previous level finishes
    if constexpr (GATHER) {
        wait();
    }
    IeCtx<P> iec;
    if constexpr (GATHER) {   // dav1d_prepare_intra_edges, every entry straight into LDS
        if (edged) {
            const PlaneTabIE<BPC> &pti = static_cast<const PlaneTabIE<BPC> &>(pt);
            iec = ie_setup<P>(rec, pt.dst[plane], ds, pti.top[plane], pti.top_stride[plane], pti.sb_log2[plane],
                              W / 4, H / 4, bdmax);
            // every entry's load first (a fixed, unrolled count per lane, so
            // the loads go out together), then the LDS writes
            constexpr int NE = 2 * W + 2 * H + 1, EPL = (NE + G - 1) / G;
            P *tw_ = reinterpret_cast<P *>(src) + 2 * H;
            int ev[EPL];
#pragma unroll
            for (int k = 0; k < EPL; k++) {
                const int i = -2 * H + l + k * G;
                bool need;
                ev[k] = (i <= 2 * W && ie_need(iec, i)) ? ie_value<P>(iec, i, need) : -1;
            }
#pragma unroll
            for (int k = 0; k < EPL; k++)
                if (ev[k] >= 0) tw_[-2 * H + l + k * G] = (P)ev[k];
            ug.p.intra.mode = (uint8_t)iec.mode;   // CFL: its DC source, the same byte
            if (pred != DGPU_PRED_CFL) ug.p.intra.angle = ie_angle_field(rec, iec.angle);
            if (l == 0) {
                bst(&a.units_rw[first + g].p.intra.mode, ug.p.intra.mode);
                if (pred != DGPU_PRED_CFL) bst(&a.units_rw[first + g].p.intra.angle, ug.p.intra.angle);
            }
        }
    }

    if constexpr (GATHER) wave_sync();
    mark(5);

    // ---------------- P5/P6: prediction + residual -> picture ----------------
    // One loop per prediction kind, so values of one kind's path are not
    // live (register pressure) in another's.
    // GATHER: a unit whose bottom row ends a superblock row also copies it
    // to top_edge once stored (units never straddle superblock rows)
    P *bkrow = nullptr;
    if constexpr (GATHER) {
        const PlaneTabIE<BPC> &pti = static_cast<const PlaneTabIE<BPC> &>(pt);
        const int y1 = rec.y4 * 4 + H, sbl = pti.sb_log2[plane], sby = (y1 >> sbl) - 1;
        if (pti.top[plane] && (y1 & ((1 << sbl) - 1)) == 0 && sby < pti.top_rows[plane])
            bkrow = pti.top[plane] + (size_t)sby * pti.top_stride[plane] + rec.x4 * 4;
    }
    auto emit = [&](int j, int q, const int *pv) {   // + residual, clip, store 2 rows of 4
        int rv[8];
        if (haveres) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const TT *rp = res + (4 * q + i) * SL::RS + 2 * j;
                if constexpr (BPC == 8) {
                    const uint32_t v = *reinterpret_cast<const uint32_t *>(rp);
                    rv[i] = (int)(int16_t)(v & 0xffff);
                    rv[4 + i] = (int)v >> 16;
                } else {
                    const int2 v = *reinterpret_cast<const int2 *>(rp);
                    rv[i] = v.x;
                    rv[4 + i] = v.y;
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) rv[i] = dcres;
        }
#pragma unroll
        for (int rr = 0; rr < 2; rr++) {
            P *row = dstp + __mul24(2 * j + rr, ds) + 4 * q;   // 24-bit: strides < 2^23 px (full-rate multiply)
            const int o0 = clampi(pv[4 * rr + 0] + rv[4 * rr + 0], 0, bdmax);
            const int o1 = clampi(pv[4 * rr + 1] + rv[4 * rr + 1], 0, bdmax);
            const int o2 = clampi(pv[4 * rr + 2] + rv[4 * rr + 2], 0, bdmax);
            const int o3 = clampi(pv[4 * rr + 3] + rv[4 * rr + 3], 0, bdmax);
            if constexpr (BPC == 8) {
                gst<uint32_t>(row, (uint32_t)o0 | o1 << 8 | o2 << 16 | (uint32_t)o3 << 24);
            } else {
                gst<u32x2>(row, u32x2{(uint32_t)o0 | o1 << 16, (uint32_t)o2 | (uint32_t)o3 << 16});
            }
            // GATHER: a superblock-bottom unit's last row also goes to top_edge
            // (dav1d_backup_ipred_edge for its columns) straight from these
            // registers: reading it back from the picture after the stores
            // cost a store-to-load round trip on the wavefront's critical path
            if constexpr (GATHER) {
                if (bkrow && 2 * j + rr == H - 1) {
                    P *b = bkrow + 4 * q;
                    bst(b + 0, (P)o0);
                    bst(b + 1, (P)o1);
                    bst(b + 2, (P)o2);
                    bst(b + 3, (P)o3);
                }
            }
        }
    };

    if (inter && !ii) {   // (WARPK: DGPU_MX_CLAMP units)
        if (comp) {   // prep x2 (rnd_sh(t, 6) - PB) then avg_c, src/mc_tmpl.c:587-602
            constexpr int KP = kMidBias<BPC> + 32;
            int q0[CL::SEQREF ? TPL : 1][8];
            if constexpr (CL::SEQREF) {
                // first ref's prep values in registers while the second
                // ref's h-pass reuses the intermediate tile
#pragma unroll
                for (int k = 0; k < TPL; k++) {
                    const int t = l + k * G;
                    if (t < NT) {
                        mc_vtask<W>(mid0, t / QW, t % QW, tv0, KP, 6, q0[k]);
                    }
                }
                wave_sync();
                mark(6);
                hpass(1);
                wave_sync();
                mark(7);
            }
#pragma unroll
            for (int k = 0; k < TPL; k++) {
                const int t = l + k * G;
                if (t >= NT) break;
                const int j = t / QW, q = t % QW;
                int p0[8], t1[8], pv[8];
                if constexpr (CL::SEQREF) {
#pragma unroll
                    for (int i = 0; i < 8; i++) p0[i] = q0[k][i];
                } else {
                    mc_vtask<W>(mid0, j, q, tv0, KP, 6, p0);
                }
                mc_vtask<W>(mid1, j, q, tv1, KP, 6, t1);
                // p = prep + PREP_BIAS, so the reference's bias terms cancel:
                // avg_c / w_avg_c / mask_c (src/mc_tmpl.c:587-639)
                if (pred == DGPU_PRED_INTER_AVG) {
#pragma unroll
                    for (int i = 0; i < 8; i++)
                        pv[i] = clampi((p0[i] + t1[i] + (1 << ib)) >> (ib + 1), 0, bdmax);
                } else if (pred == DGPU_PRED_INTER_WAVG) {
                    const int wt = u.p.inter.weight;
#pragma unroll
                    for (int i = 0; i < 8; i++)
                        pv[i] = clampi((__mul24(p0[i], wt) + __mul24(t1[i], 16 - wt) + (8 << ib)) >> (ib + 4), 0, bdmax);
                } else {   // INTER_MASK: mask rows of the block (stride bw), 4 bytes per task row
                    const uint8_t *mk = a.aux_pool + auxo + __mul24(2 * j, bw) + 4 * q;
                    const uint32_t m0 = gld<uint32_t>(mk), m1 = gld<uint32_t>(mk + bw);
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const int m = (int)(((i < 4 ? m0 : m1) >> (8 * (i & 3))) & 0xff);
                        pv[i] = clampi((__mul24(p0[i], m) + __mul24(t1[i], 64 - m) + (32 << ib)) >> (ib + 6), 0, bdmax);
                    }
                }
                emit(j, q, pv);
            }
        } else {   // put: rnd_sh(t, 6 + ib)
            const int sh = 6 + ib, kp = kMidBias<BPC> + (1 << (sh - 1));
#pragma unroll
            for (int k = 0; k < TPL; k++) {
                const int t = l + k * G;
                if (t >= NT) break;
                const int j = t / QW, q = t % QW;
                int t0[8], pv[8];
                mc_vtask<W>(mid0, j, q, tv0, kp, sh, t0);
#pragma unroll
                for (int i = 0; i < 8; i++) pv[i] = clampi(t0[i], 0, bdmax);
                emit(j, q, pv);
            }
        }
    } else if (NW && pred == DGPU_PRED_INTRA) {
        const IntraState is = intra_prep<BPC, TX>(u, tl, fe, l, bdmax);
        wave_sync();
        if (is.mode == DGPU_FILTER_PRED) filter_intra<TX>(u, tl, ptile, l, bdmax);
        wave_sync();
#pragma unroll
        for (int k = 0; k < TPL; k++) {
            const int t = l + k * G;
            if (t >= NT) break;
            const int j = t / QW, q = t % QW;
            int pv[8];
            if (is.mode == DGPU_FILTER_PRED) {
#pragma unroll
                for (int i = 0; i < 8; i++) pv[i] = ptile[(2 * j + (i >> 2)) * W + 4 * q + (i & 3)];
            } else {
                intra_task<TX>(is, tl, fe, 4 * q, 2 * j, pv);
            }
            emit(j, q, pv);
        }
    } else if (ii) {   // inter-intra, second launch: put, intra_pred, blend_c (src/mc_tmpl.c:641-653)
        // 1. the inter (put) prediction of every task into registers
        const int sh = 6 + ib, kp = kMidBias<BPC> + (1 << (sh - 1));
        int ipv[TPL][8];
#pragma unroll
        for (int k = 0; k < TPL; k++) {
            const int t = l + k * G;
            if (t < NT) {
                int t0[8];
                mc_vtask<W>(mid0, t / QW, t % QW, tv0, kp, sh, t0);
#pragma unroll
                for (int i = 0; i < 8; i++) ipv[k][i] = clampi(t0[i], 0, bdmax);
            }
        }
        wave_sync();   // the intermediate tile is free: the edges go there
        // 2. the intra record, its edge array and the edge preparation
        const Dav1dGpuIntraEdge &rec_in = rec;   // (GATHER: the unit's edge record)
        const u32x4 rec = gld<u32x4>(a.aux_pool + auxo);
        Dav1dGpuUnit ui = u;
        ui.p.intra.edge_off = (int32_t)rec[0];
        ui.p.intra.mode = (uint8_t)(rec[1] & 0xff);
        ui.p.intra.angle = (uint16_t)(rec[1] >> 16);
        ui.p.intra.max_w = ui.p.intra.max_h = 0;
        const P *tl2;
        if constexpr (GATHER) {   // dav1d_prepare_intra_edges from the picture, as for INTRA units
            const PlaneTabIE<BPC> &pti = static_cast<const PlaneTabIE<BPC> &>(pt);
            IeCtx<P> ie = ie_setup<P>(rec_in, pt.dst[plane], ds, pti.top[plane], pti.top_stride[plane],
                                      pti.sb_log2[plane], W / 4, H / 4, bdmax);
            constexpr int NE = 2 * W + 2 * H + 1, EPL = (NE + G - 1) / G;
            P *tw_ = reinterpret_cast<P *>(src) + 2 * H;
            int ev[EPL];
#pragma unroll
            for (int k = 0; k < EPL; k++) {
                const int i = -2 * H + l + k * G;
                bool need;
                ev[k] = (i <= 2 * W && ie_need(ie, i)) ? ie_value<P>(ie, i, need) : -1;
            }
#pragma unroll
            for (int k = 0; k < EPL; k++)
                if (ev[k] >= 0) tw_[-2 * H + l + k * G] = (P)ev[k];
            ui.p.intra.mode = (uint8_t)ie.mode;
            ui.p.intra.angle = ie_angle_field(rec_in, ie.angle);
            tl2 = tw_;
        } else {
            Stage<SL::EDGE * (int)sizeof(P), G> est2;
            est2.load(a.edges + (int)rec[0] - 2 * H, SL::EDGE * (int)sizeof(P), l);
            tl2 = reinterpret_cast<const P *>(src + est2.commit(src, l)) + 2 * H;
        }
        wave_sync();
        const IntraState is = intra_prep<BPC, TX>(ui, tl2, fe, l, bdmax);
        wave_sync();
        if (is.mode == DGPU_FILTER_PRED) filter_intra<TX>(ui, tl2, ptile, l, bdmax);
        wave_sync();
        const uint8_t *mkb = a.aux_pool + rec[2];
        // 3. per task: intra prediction, the mask, blend, residual
#pragma unroll
        for (int k = 0; k < TPL; k++) {
            const int t = l + k * G;
            if (t >= NT) break;
            const int j = t / QW, q = t % QW;
            int pvi[8], pv[8];
            if (is.mode == DGPU_FILTER_PRED) {
#pragma unroll
                for (int i = 0; i < 8; i++) pvi[i] = ptile[(2 * j + (i >> 2)) * W + 4 * q + (i & 3)];
            } else {
                intra_task<TX>(is, tl2, fe, 4 * q, 2 * j, pvi);
            }
            const uint8_t *mk = mkb + __mul24(2 * j, bw) + 4 * q;
            const uint32_t m0 = gld<uint32_t>(mk), m1 = gld<uint32_t>(mk + bw);
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int m = (int)(((i < 4 ? m0 : m1) >> (8 * (i & 3))) & 0xff);
                pv[i] = (__mul24(ipv[k][i], 64 - m) + __mul24(pvi[i], m) + 32) >> 6;
            }
            emit(j, q, pv);
        }
    } else if (pred == DGPU_PRED_WARP) {   // only in the warp launch (its own register budget)
        if constexpr (WARPK && W >= 8 && H >= 8)
            warp_unit<BPC, TX, P>(a, pt, u, auxo, reinterpret_cast<int16_t *>(mid0),
                                  reinterpret_cast<const uint2 *>(wave_lds + kWarpTabOff<BPC>), l, bdmax, emit);
    } else if (NW && pred == DGPU_PRED_PAL) {   // pal_pred (src/ipred_tmpl.c:717-730)
        const uint8_t *rec = a.aux_pool + auxo;
        const u32x4 pal = gld<u32x4>(rec);   // 8 entries (u8 x 8 or u16 x 8)
#pragma unroll
        for (int k = 0; k < TPL; k++) {
            const int t = l + k * G;
            if (t >= NT) break;
            const int j = t / QW, q = t % QW;
            int pv[8];
#pragma unroll
            for (int rr = 0; rr < 2; rr++) {
                const uint32_t ix = gld<uint16_t>(rec + 16 + (2 * j + rr) * (W / 2) + 2 * q);
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int e = (int)((ix >> (4 * i)) & 7);
                    if constexpr (BPC == 8)
                        pv[4 * rr + i] = (int)(((e < 4 ? pal[0] : pal[1]) >> (8 * (e & 3))) & 0xff);
                    else
                        pv[4 * rr + i] = (int)(((e < 2 ? pal[0] : e < 4 ? pal[1] : e < 6 ? pal[2] : pal[3]) >>
                                                (16 * (e & 1))) & 0xffff);
                }
            }
            emit(j, q, pv);
        }
    } else if (NW && pred == DGPU_PRED_CFL) {
        if constexpr (W == H && W <= 32) cfl_units<BPC, TX>(a, u, tl, fe, l, bdmax, emit);
    } else if (NW) {   // PRED_NONE: the residual goes onto the picture
#pragma unroll
        for (int k = 0; k < TPL; k++) {
            const int t = l + k * G;
            if (t >= NT) break;
            const int j = t / QW, q = t % QW;
            int pv[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                pv[i] = gld<P>(dstp + __mul24(2 * j + (i >> 2), ds) + 4 * q + (i & 3));
            }
            emit(j, q, pv);
        }
    }
    mark(8);
}


// ------------------------------------------------- the second launch's kinds --
// INTER_WMASK, INTER_OBMC and INTER_SCALED units (include/dav1d_gpu.h): run
// by the WARP group's kernel beside warp / inter-intra, in a function of
// their own so that the main kernel's code (recon_units above, which sits at
// the edge of its 5-wave register budget) is not perturbed by them.  Same
// phases as recon_units: staged coefficients, both transform passes into the
// LDS residual, then the prediction + residual per 4x2 task.
template <int BPC, int TX>
__device__ __forceinline__ void recon_units_ext(const ReconArgs<BPC> &a, const PlaneTab<BPC> &pt,
                                                const Dav1dGpuUnit &u, int first, int count, uint8_t *wave_lds) {
    using CL = Cls<TX>;
    using SL = Slot<BPC, TX>;
    using P = typename Px<BPC>::pixel;
    using C = typename Px<BPC>::coef;
    using TT = typename Tmp<BPC>::T;
    constexpr int W = CL::W, H = CL::H, SW = CL::SW, SH = CL::SH, G = CL::G, QW = CL::QW, NT = CL::NT;
    constexpr int TPL = CL::TPL;
    const int lane = unit_lane();
    const int g = lane / G, l = lane % G;
    if (g >= count) return;
    uint8_t *slot = wave_lds + g * SL::BYTES_W;
    uint8_t *cfl = slot;
    TT *res = reinterpret_cast<TT *>(slot);
    TT *tmp = reinterpret_cast<TT *>(slot + SL::CFR);
    uint8_t *src = slot + SL::CFR + SL::TMP;
    uint32_t *mid0 = reinterpret_cast<uint32_t *>(src);
    uint32_t *mid1 = reinterpret_cast<uint32_t *>(src + (CL::SEQREF ? 0 : SL::MID));

    const int plane = u.plane;
    const int bdmax = a.bdmax;
    const int ib = Px<BPC>::ibits(bdmax);
    const int pred = u.pred;
    const bool wm = pred == DGPU_PRED_INTER_WMASK, ob = pred == DGPU_PRED_INTER_OBMC;
    const bool sc = pred == DGPU_PRED_INTER_SCALED;
    const int txtp = u.txtp;
    const bool nores = txtp == DGPU_NO_RESIDUAL;
    const int nzw = u.nzw, nzh = u.nzh;
    const bool dconly = !nores && nzw == 0;
    const bool haveres = !nores && !dconly;
    const bool wht = W == 4 && H == 4 && txtp == DGPU_WHT_WHT;   // lossless: one lane, both passes
    P *dstp = pt.dst[plane] + u.dst_off;
    const int ds = pt.dst_stride[plane];
    const int auxo = bld(a.aux + first + g);

    // ---- loads: coefficients and the first reference's footprint rows
    C *cf = a.coef + u.coef_off;
    const int ncoef = nores ? 0 : dconly ? 1 : nzw * nzh;
    Stage<CL::SW * CL::SH * (int)sizeof(C), G> cst;
    if (ncoef) cst.load(cf, ncoef * (int)sizeof(C), l);
    const int f2d = u.p.inter.filter2d;
    const bool bil = f2d == DGPU_FILTER_2D_BILINEAR;
    const int ftype = bil ? 0 : (int)((0x951a62840ull >> (4 * f2d)) & 15);   // type_h | type_v << 2
    const int bw = u.bw4 * 4, bh = u.bh4 * 4;
    const int bank_h = mc_bank(ftype & 3, bil, bw), bank_v = mc_bank(ftype >> 2, bil, bh);
    const uint4 tv0 = reinterpret_cast<const uint4 *>(dspt_mc16)[bank_v * 16 + u.p.inter.my[0]];
    const uint4 tv1 = reinterpret_cast<const uint4 *>(dspt_mc16)[bank_v * 16 + u.p.inter.my[1]];
    // DGPU_MX_CLAMP (round 6, as the first launch's inter units): src_off[k]
    // = x | y << 16 and every footprint pixel clamped to the plane
    using HPC = HPass<BPC, TX, true>;
    auto hinit = [&](HPC &hp, int k) {
        const int r = u.p.inter.ref[k];
        const int rs = pt.ref_stride[r * 3 + plane];
        const int mx = u.p.inter.mx[k];
        if (mx & DGPU_MX_CLAMP) {
            int rw, rh;
            ref_plane_wh<BPC>(r, plane, rw, rh);
            const int so = u.p.inter.src_off[k];
            hp.init_clamp(pt.ref[r * 3 + plane], rs, rw, rh, (int)(int16_t)(so & 0xffff), so >> 16, k ? mid1 : mid0,
                          bank_h, mx & 15, l);
            return;
        }
        const P *org = pt.ref[r * 3 + plane] + u.p.inter.src_off[k] - 3 * rs - 3;
        hp.init(org, rs, k ? mid1 : mid0, bank_h, mx, l);
    };
    HPC hp0;
    if (wm || ob) {
        hinit(hp0, 0);
        hp0.load(0);
    }
    int cfsk = 0;
    if (ncoef) cfsk = cst.commit(cfl, l);
    if (wm || ob) {
        hp0.compute(0, ib);
        hp0.rest(ib);
        if (!CL::SEQREF && wm) {
            HPC hp1;
            hinit(hp1, 1);
            hp1.load(0);
            hp1.compute(0, ib);
            hp1.rest(ib);
        }
    }
    wave_sync();
    if (a.zero_coefs && ncoef)
        for (int i = l; i < ncoef; i += G) bst<C>(cf + i, 0);

    // ---- row, then column transforms into the residual (as recon_units)
    int dcres = 0;
    if (dconly) {   // src/itx_tmpl.c:53-65
        int dc = reinterpret_cast<const C *>(cfl + cfsk)[0];
        if (CL::RECT2) dc = r8s(dc);
        dc = r8s(dc);
        dc = (dc + ((1 << CL::SHIFT) >> 1)) >> CL::SHIFT;
        dcres = (dc * 181 + 128 + 2048) >> 12;
    }
    const Clip rc = ItxClip<BPC>::row(bdmax), cc = ItxClip<BPC>::col(bdmax);
    if (haveres && !wht) {
        const C *cs = reinterpret_cast<const C *>(cfl + cfsk);
#pragma unroll
        for (int k = 0; k < (SH + G - 1) / G; k++) {
            const int r = l + k * G;
            if (r < SH) {
                TT *trow = tmp + r * W;
                int c[W];
#pragma unroll
                for (int x = 0; x < W; x++) {
                    int v = 0;
                    if (x < SW && r < nzh) {
                        v = cs[x * nzh + r];
                        v = x < nzw ? v : 0;
                    }
                    c[x] = CL::RECT2 ? r8s(v) : v;
                }
                if (r < nzh) tx1d<W, 1, BPC == 8>(kind_h(txtp), c, rc);
                constexpr int RND = (1 << CL::SHIFT) >> 1;
#pragma unroll
                for (int x = 0; x < W; x++) trow[x] = (TT)cc((c[x] + RND) >> CL::SHIFT);
            }
        }
    }
    wave_sync();
    if constexpr (W == 4 && H == 4) {
        if (wht && l == 0) {
            int t[16];
            wht4x4(reinterpret_cast<const C *>(cfl + cfsk), nzw, nzh, t);
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 4; y++)
                    res[x * SL::RS + y] = (TT)(BPC == 8 ? clampi(t[4 * y + x], -32768, 32767) : t[4 * y + x]);
        }
    }
    if (haveres && !wht) {
#pragma unroll
        for (int k = 0; k < (W + G - 1) / G; k++) {
            const int x = l + k * G;
            if (x < W) {
                int col[H];
#pragma unroll
                for (int y = 0; y < H; y++) col[y] = y < SH ? (int)tmp[y * W + x] : 0;
                tx1d<H, 1, BPC == 8>(kind_v(txtp), col, cc);
                TT *rcol = res + x * SL::RS;
#pragma unroll
                for (int y = 0; y < H; y++) rcol[y] = (TT)((col[y] + 8) >> 4);
            }
        }
    }
    wave_sync();

    auto emit = [&](int j, int q, const int *pv) {   // + residual, clip, store 2 rows of 4
#pragma unroll
        for (int rr = 0; rr < 2; rr++) {
            int o[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int rv = haveres ? (int)res[(4 * q + i) * SL::RS + 2 * j + rr] : dcres;
                o[i] = clampi(pv[4 * rr + i] + rv, 0, bdmax);
            }
            P *row = dstp + __mul24(2 * j + rr, ds) + 4 * q;   // 24-bit: strides < 2^23 px (full-rate multiply)
            if constexpr (BPC == 8)
                gst<uint32_t>(row, (uint32_t)o[0] | o[1] << 8 | o[2] << 16 | (uint32_t)o[3] << 24);
            else
                gst<u32x2>(row, u32x2{(uint32_t)o[0] | o[1] << 16, (uint32_t)o[2] | (uint32_t)o[3] << 16});
        }
    };
    const int psh = 6 + ib, pkp = kMidBias<BPC> + (1 << (psh - 1));   // put rounding

    if (wm) {   // COMP_INTER_SEG luma: mct x2, w_mask_c (src/mc_tmpl.c:683-726)
        constexpr int KP = kMidBias<BPC> + 32;
        int q0[CL::SEQREF ? TPL : 1][8];
        if constexpr (CL::SEQREF) {   // the first ref's prep values held while the second's h-pass reuses the tile
#pragma unroll
            for (int k = 0; k < TPL; k++) {
                const int t = l + k * G;
                if (t < NT) mc_vtask<W>(mid0, t / QW, t % QW, tv0, KP, 6, q0[k]);
            }
            wave_sync();
            HPC hp1;
            hinit(hp1, 1);
            hp1.load(0);
            hp1.compute(0, ib);
            hp1.rest(ib);
            wave_sync();
        }
        const int sign = u.p.inter.weight;
        const int msh = bits_of(bdmax) + ib - 4, mrnd = 1 << (msh - 5);
        // the mask at the chroma layout's resolution (cfl_ss), row stride
        // bw >> ss_hor; aux = the unit's top-left value in it
        uint8_t *mo = const_cast<uint8_t *>(a.aux_pool) + auxo;
        const int ssh = a.cfl_ss & 1, ssv = (a.cfl_ss >> 1) & 1, ms = bw >> ssh;
#pragma unroll
        for (int k = 0; k < TPL; k++) {
            const int t = l + k * G;
            if (t >= NT) break;
            const int j = t / QW, q = t % QW;
            int p0[8], p1[8], pv[8], mm[8];
            if constexpr (CL::SEQREF) {
#pragma unroll
                for (int i = 0; i < 8; i++) p0[i] = q0[k][i];
            } else {
                mc_vtask<W>(mid0, j, q, tv0, KP, 6, p0);
            }
            mc_vtask<W>(mid1, j, q, tv1, KP, 6, p1);
#pragma unroll
            for (int i = 0; i < 8; i++) {   // p = prep + PREP_BIAS: the bias terms cancel
                const int m = min(38 + ((abs(p0[i] - p1[i]) + mrnd) >> msh), 64);
                mm[i] = m;
                pv[i] = clampi((__mul24(p0[i], m) + __mul24(p1[i], 64 - m) + (32 << ib)) >> (ib + 6), 0, bdmax);
            }
            if (!ssh) {
#pragma unroll
                for (int rr = 0; rr < 2; rr++)
                    gst<uint32_t>(mo + (2 * j + rr) * ms + 4 * q, (uint32_t)mm[4 * rr] | mm[4 * rr + 1] << 8 |
                                                                      mm[4 * rr + 2] << 16 |
                                                                      (uint32_t)mm[4 * rr + 3] << 24);
            } else if (!ssv) {
#pragma unroll
                for (int rr = 0; rr < 2; rr++) {
                    const int v0 = (mm[4 * rr] + mm[4 * rr + 1] + 1 - sign) >> 1;
                    const int v1 = (mm[4 * rr + 2] + mm[4 * rr + 3] + 1 - sign) >> 1;
                    gst<uint16_t>(mo + (2 * j + rr) * ms + 2 * q, (uint16_t)(v0 | v1 << 8));
                }
            } else {
                const int v0 = (mm[0] + mm[1] + mm[4] + mm[5] + 2 - sign) >> 2;
                const int v1 = (mm[2] + mm[3] + mm[6] + mm[7] + 2 - sign) >> 2;
                gst<uint16_t>(mo + j * ms + 2 * q, (uint16_t)(v0 | v1 << 8));
            }
            emit(j, q, pv);
        }
    } else if (ob) {
        // the block's own put prediction, then the neighbours' predictions
        // over the unit's overlap regions (the lap calls), blended in the
        // reference's order: every blend_h (above) before every blend_v (left)
        const int sh = psh, kp = pkp;
        int ipv[TPL][8];
#pragma unroll
        for (int k = 0; k < TPL; k++) {
            const int t = l + k * G;
            if (t < NT) {
                int t0[8];
                mc_vtask<W>(mid0, t / QW, t % QW, tv0, kp, sh, t0);
#pragma unroll
                for (int i = 0; i < 8; i++) ipv[k][i] = clampi(t0[i], 0, bdmax);
            }
        }
        const uint8_t *rec = a.aux_pool + auxo;
        const int ne = gld<int>(rec);
        int nmax = ne;   // the loop runs to the most entries of the wave's units
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) nmax = max(nmax, __shfl_xor(nmax, off, 64));
#pragma unroll 1
        for (int e = 0; e < nmax; e++) {
            wave_sync();   // the intermediate tile is free
            const bool has = e < ne;
            const u32x4 er = has ? gld<u32x4>(rec + 16 + 16 * e) : u32x4{0, 0, 0, 0};
            const int ef2d = (er[1] >> 16) & 0xff, eref = er[1] >> 24;
            const bool ebil = ef2d == DGPU_FILTER_2D_BILINEAR;
            const int eft = ebil ? 0 : (int)((0x951a62840ull >> (4 * ef2d)) & 15);
            const int ebh = mc_bank(eft & 3, ebil, (int)(er[3] & 0xff) * 4);
            const int ebv = mc_bank(eft >> 2, ebil, (int)((er[3] >> 8) & 0xff) * 4);
            if (has) {
                HPC hp;
                const int rs = pt.ref_stride[eref * 3 + plane];
                const int emx = (int)(er[1] & 0xff);
                if (emx & DGPU_MX_CLAMP) {   // this lap's footprint clamped: er[0] = x | y << 16
                    int rw, rh;
                    ref_plane_wh<BPC>(eref, plane, rw, rh);
                    hp.init_clamp(pt.ref[eref * 3 + plane], rs, rw, rh, (int)(int16_t)(er[0] & 0xffff),
                                  (int)er[0] >> 16, mid0, ebh, emx & 15, l);
                } else {
                    const P *org = pt.ref[eref * 3 + plane] + (int)er[0] - 3 * rs - 3;
                    hp.init(org, rs, mid0, ebh, emx, l);
                }
                hp.load(0);
                hp.compute(0, ib);
                hp.rest(ib);
            }
            wave_sync();
            const uint4 etv = reinterpret_cast<const uint4 *>(dspt_mc16)[ebv * 16 + ((er[1] >> 8) & 0xff)];
            const int x0 = er[2] & 0xff, y0 = (er[2] >> 8) & 0xff, x1 = (er[2] >> 16) & 0xff, y1 = er[2] >> 24;
            const int dir = (er[3] >> 16) & 0xff, moff = er[3] >> 24;
#pragma unroll
            for (int k = 0; k < TPL; k++) {
                const int t = l + k * G;
                const int j = t / QW, q = t % QW;
                if (has && t < NT && 2 * j + 1 >= y0 && 2 * j < y1 && 4 * q + 3 >= x0 && 4 * q < x1) {
                    int lap[8];
                    mc_vtask<W>(mid0, j, q, etv, kp, sh, lap);
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const int x = 4 * q + (i & 3), y = 2 * j + (i >> 2);
                        if (x >= x0 && x < x1 && y >= y0 && y < y1) {   // blend_px, src/mc_tmpl.c:640
                            const int m = dspt_obmc[moff + (dir ? x : y)];
                            ipv[k][i] = (__mul24(ipv[k][i], 64 - m) + __mul24(clampi(lap[i], 0, bdmax), m) + 32) >> 6;
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < TPL; k++) {
            const int t = l + k * G;
            if (t < NT) emit(t / QW, t % QW, ipv[k]);
        }
    } else if (sc) {   // scaled references, second launch: put_8tap_scaled, or
        // prep_8tap_scaled x2 + avg / w_avg (src/mc_tmpl.c:173-328; bilinear
        // :452-585 as the (64 - 4m, 4m) bank, m = 0 the identity)
        const uint8_t *rec = a.aux_pool + auxo;
        const int nref = gld<int>(rec) & 3;
        int16_t *mids = reinterpret_cast<int16_t *>(mid0);
        const int fb_h = mc_bank(ftype & 3, bil, bw), fb_v = mc_bank(ftype >> 2, bil, bh);
        int q0[TPL][8];
#pragma unroll 1
        for (int k = 0; k < 2; k++) {
            wave_sync();
            const bool act = k < nref;
            const u32x4 rr = act ? gld<u32x4>(rec + 16 + 16 * k) : u32x4{0, 0, 0, 0};
            // bit 15 of the x phase: this reference's footprint clamped to the
            // plane (round 6), rr[0] = x | y << 16 of the integer origin
            const bool scl = rr[1] & 0x8000u;
            const int smx = (int)(rr[1] & 0x7fff), smy = (int)(rr[1] >> 16);
            const int sdx = (int)(rr[2] & 0xffff), sdy = (int)(rr[2] >> 16);
            const int r = u.p.inter.ref[k];
            const int rs = pt.ref_stride[r * 3 + plane];
            const P *org = pt.ref[r * 3 + plane] + (scl ? 0 : (int)rr[0] - 3 * rs - 3);
            int cw = 1, chh = 1;
            if (scl) ref_plane_wh<BPC>(r, plane, cw, chh);
            const int cx0 = (int)(int16_t)(rr[0] & 0xffff) - 3, cy0 = ((int)rr[0] >> 16) - 3;
            const int rows = min((((H - 1) * sdy + smy) >> 10) + 8, 2 * H + 8);   // (bound: the LDS area)
            const int hsh = 6 - ib, hrnd = (1 << hsh) >> 1;
            if (act) {
#pragma unroll 1
                for (int it = l; it < rows * W; it += G) {
                    const int row = it / W, x = it - row * W;
                    const int pos = smx + x * sdx;
                    const P *sp = org + row * rs + (pos >> 10);
                    const uint2 tp = reinterpret_cast<const uint2 *>(dspt_mc8)[fb_h * 16 + ((pos & 1023) >> 6)];
                    int acc = 0;
                    if (scl) {
#pragma unroll
                        for (int i = 0; i < 8; i++)
                            acc += __builtin_amdgcn_sbfe((int)(i < 4 ? tp.x : tp.y), 8 * (i & 3), 8) *
                                   (int)clamped_px<P>(reinterpret_cast<const uint8_t *>(org), (unsigned)rs * sizeof(P),
                                                      cx0 + (pos >> 10) + i, cy0 + row, cw, chh);
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; i++)
                            acc += __builtin_amdgcn_sbfe((int)(i < 4 ? tp.x : tp.y), 8 * (i & 3), 8) * (int)gld<P>(sp + i);
                    }
                    mids[row * W + x] = (int16_t)((acc + hrnd) >> hsh);
                }
            }
            wave_sync();
#pragma unroll
            for (int kt = 0; kt < TPL; kt++) {
                const int t = l + kt * G;
                if (!act || t >= NT) continue;
                const int j = t / QW, qq = t % QW;
                int pv[8];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int x = 4 * qq + (i & 3), y = 2 * j + (i >> 2);
                    const int pos = smy + y * sdy;
                    const uint2 tp = reinterpret_cast<const uint2 *>(dspt_mc8)[fb_v * 16 + ((pos & 1023) >> 6)];
                    const int16_t *mc_ = mids + (pos >> 10) * W + x;
                    int acc = 0;
#pragma unroll
                    for (int tt = 0; tt < 8; tt++)
                        acc += __builtin_amdgcn_sbfe((int)(tt < 4 ? tp.x : tp.y), 8 * (tt & 3), 8) * (int)mc_[tt * W];
                    pv[i] = acc;
                }
                if (nref == 1) {   // put: (sum + (32 << ib)) >> (6 + ib), clipped
#pragma unroll
                    for (int i = 0; i < 8; i++) pv[i] = clampi((pv[i] + (32 << ib)) >> (6 + ib), 0, bdmax);
                    emit(j, qq, pv);
                } else if (k == 0) {   // prep + PREP_BIAS of the first reference, kept
#pragma unroll
                    for (int i = 0; i < 8; i++) q0[kt][i] = (pv[i] + 32) >> 6;
                } else {
                    const int wt = u.p.inter.weight;   // 0: avg_c, 1..15: w_avg_c (src/mc_tmpl.c:587-620)
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const int p1 = (pv[i] + 32) >> 6;
                        pv[i] = wt ? clampi((__mul24(q0[kt][i], wt) + __mul24(p1, 16 - wt) + (8 << ib)) >> (ib + 4), 0, bdmax)
                                   : clampi((q0[kt][i] + p1 + (1 << ib)) >> (ib + 1), 0, bdmax);
                    }
                    emit(j, qq, pv);
                }
            }
        }
    }
}

}  // namespace dgpu
