// intra_edge_dev.hpp -- device form of bytefn(dav1d_prepare_intra_edges)
// (src/ipred_prepare_tmpl.c:76-204) per record, shared by the standalone
// edge stage (edges.hip) and the intra wavefront's reconstruction kernels
// (recon_kernel.hpp, GATHER).  ie_setup derives the implementation mode (the
// remap of :83-104) and the extents; ie_value computes one entry
// topleft[i], i in [-2*4*th, 2*4*tw], straight from the picture with the
// reference's extension rules, so entries are independent of each other
// (the Z2 top-left filter of :197-200 recomputes topleft[-1] and topleft[1]).
#pragma once
#include <hip/hip_runtime.h>

#include "dav1d_gpu.h"

namespace dgpu {

// needs per implementation mode: bit0 left, 1 top, 2 top-left, 3 top-right,
// 4 bottom-left (av1_intra_prediction_edges, src/ipred_prepare_tmpl.c:50-75)
__device__ __forceinline__ int ie_needs(int m) {
    constexpr uint64_t t = (3ull << 0) | (2ull << 5) | (1ull << 10) | (1ull << 15) | (2ull << 20) | (0ull << 25) |
                           (14ull << 30) | (7ull << 35) | (21ull << 40) | (3ull << 45) | (3ull << 50) |
                           (3ull << 55) | (7ull << 60);
    return m == DGPU_FILTER_PRED ? 7 : (int)((t >> (5 * m)) & 31);
}

template <typename P> struct IeCtx {
    const P *dst;    // the block's top-left pixel
    const P *top;    // the row above (picture or top_edge row)
    int ps;          // picture stride, pixels
    int mode, angle, nd;
    int hl, ht, hbl, htr;
    int szl, szt, nl, nt, nbl, ntr;
    int half, z2f;
};

// dst: picture plane, ps its stride; top_row: top_edge row base of the
// plane (used when the record has DGPU_IE_TOP_SB_EDGE), ts its stride;
// tw4 / th4: the transform size in 4-px units
template <typename P>
__device__ __forceinline__ IeCtx<P> ie_setup(const Dav1dGpuIntraEdge &r, const P *pic, int ps, const P *top_edge,
                                             int ts, int sb_log2, int tw4, int th4, int bdmax) {
    IeCtx<P> c;
    c.ps = ps;
    c.dst = pic + (size_t)(r.y4 * 4) * ps + r.x4 * 4;
    c.hl = r.flags & DGPU_IE_HAVE_LEFT;
    c.ht = r.flags & DGPU_IE_HAVE_TOP;
    int angle = r.angle, mode = r.mode;
    if (mode >= 1 && mode <= 8) {
        // base angles of modes 1..8: 90 180 45 135 113 157 203 67
        angle = (int)((0x43cb9d71872db45aull >> (8 * (mode - 1))) & 0xff) + 3 * angle;
        mode = angle <= 90 ? (angle < 90 && c.ht ? DGPU_Z1_PRED : DGPU_VERT_PRED)
             : angle < 180 ? DGPU_Z2_PRED
                           : (angle > 180 && c.hl ? DGPU_Z3_PRED : DGPU_HOR_PRED);
    } else if (mode == 0) {
        mode = c.hl ? (c.ht ? DGPU_DC_PRED : DGPU_LEFT_DC_PRED) : (c.ht ? DGPU_TOP_DC_PRED : DGPU_DC_128_PRED);
    } else if (mode == 12) {
        mode = c.hl ? (c.ht ? DGPU_PAETH_PRED : DGPU_HOR_PRED) : (c.ht ? DGPU_VERT_PRED : DGPU_DC_128_PRED);
    }
    c.mode = mode;
    c.angle = angle;
    c.nd = ie_needs(mode);
    c.half = (bdmax + 1) >> 1;
    c.top = (r.flags & DGPU_IE_TOP_SB_EDGE)
                ? top_edge + (size_t)(((r.y4 * 4) >> sb_log2) - 1) * ts + r.x4 * 4
                : c.dst - ps;
    c.szl = th4 * 4;
    c.szt = tw4 * 4;
    c.nl = min(c.szl, (r.h4 - r.y4) * 4);
    c.nt = min(c.szt, (r.w4 - r.x4) * 4);
    c.hbl = c.hl && r.y4 + th4 < r.h4 && (r.flags & DGPU_IE_LEFT_HAS_BOTTOM);
    c.htr = c.ht && r.x4 + tw4 < r.w4 && (r.flags & DGPU_IE_TOP_HAS_RIGHT);
    c.nbl = c.hbl ? min(c.szl, (r.h4 - r.y4 - th4) * 4) : 1;
    c.ntr = c.htr ? min(c.szt, (r.w4 - r.x4 - tw4) * 4) : 1;
    c.z2f = mode == DGPU_Z2_PRED && tw4 + th4 >= 6 && (r.flags & DGPU_IE_FILTER_EDGE);
    return c;
}

// One pixel of the picture / top_edge (checked in the bounds build).
#if DGPU_BOUNDS
__device__ __noinline__ bool bnd_ok(const void *p, int n, int line);
#endif
template <typename P> __device__ __forceinline__ int ie_px(const P *p
#if DGPU_BOUNDS
                                                                    , int line = __builtin_LINE()
#endif
) {
#if DGPU_BOUNDS
    if (!bnd_ok(p, (int)sizeof(P), line)) return 0;
#endif
    return (int)*p;
}
template <typename P> __device__ __forceinline__ int ie_left(const IeCtx<P> &c, int k) {
    return c.hl ? ie_px(c.dst + (size_t)min(k, c.nl - 1) * c.ps - 1) : c.ht ? ie_px(c.top) : c.half + 1;
}
template <typename P> __device__ __forceinline__ int ie_top(const IeCtx<P> &c, int k) {
    return c.ht ? ie_px(c.top + min(k, c.nt - 1)) : c.hl ? ie_px(c.dst - 1) : c.half - 1;
}

// whether the remapped mode reads topleft[i]
template <typename P> __device__ __forceinline__ bool ie_need(const IeCtx<P> &c, int i) {
    const int bit = i < -c.szl ? 16 : i < 0 ? 1 : i == 0 ? 4 : i <= c.szt ? 2 : 8;
    return c.nd & bit;
}

// topleft[i]; `needed` false for entries the remapped mode does not read
template <typename P> __device__ __forceinline__ int ie_value(const IeCtx<P> &c, int i, bool &needed) {
    if (i < -c.szl) {           // bottom-left (:135-154)
        needed = c.nd & 16;
        const int k = -i - c.szl - 1;
        return c.hbl ? ie_px(c.dst + (size_t)(c.szl + min(k, c.nbl - 1)) * c.ps - 1) : ie_left<P>(c, c.szl - 1);
    }
    if (i < 0) {                // left (:124-133)
        needed = c.nd & 1;
        return ie_left<P>(c, -i - 1);
    }
    if (i == 0) {               // top-left (:187-201)
        needed = c.nd & 4;
        int v = c.hl ? (c.ht ? ie_px(c.top - 1) : ie_px(c.dst - 1)) : (c.ht ? ie_px(c.top) : c.half);
        if (c.z2f) v = ((ie_left<P>(c, 0) + ie_top<P>(c, 0)) * 5 + v * 6 + 8) >> 4;
        return v;
    }
    if (i <= c.szt) {           // top (:156-166)
        needed = c.nd & 2;
        return ie_top<P>(c, i - 1);
    }
    needed = c.nd & 8;          // top-right (:168-185)
    const int k = i - c.szt - 1;
    return c.htr ? ie_px(c.top + c.szt + min(k, c.ntr - 1)) : ie_top<P>(c, c.szt - 1);
}

// the unit's rewritten angle field: angle | smooth << 9 | edge filter << 10
__device__ __forceinline__ uint16_t ie_angle_field(const Dav1dGpuIntraEdge &r, int angle) {
    return (uint16_t)((angle & 511) | ((r.flags & DGPU_IE_SMOOTH) ? 512 : 0) |
                      ((r.flags & DGPU_IE_FILTER_EDGE) ? 1024 : 0));
}

}  // namespace dgpu
