// recon_persist.hpp -- the batch tier's main group as resident waves
// (round-5 experiment, DGPU_PERSIST builds only: tools/build_variants.sh
// persist / persist2 / persist3).  Included by recon_impl.hpp when
// DGPU_PERSIST is set; product builds never compile it.
#pragma once
#include "recon_impl.hpp"

namespace dgpu {

// ---------------------------------------------------- resident-wave form ---
// DGPU_PERSIST (round 5): the main group as resident waves.
// The grid holds only as many workgroups as the chip keeps resident; each
// wave walks the same (segment, class) wave schedule k_recon's grid covers
// (its XCD's contiguous eighth of it, in the order the dispatcher would have
// handed it out), so the plane table is built once per wave and, with
// DGPU_PERSIST >= 2, the next work item's unit descriptor is loaded while the
// current one computes.  The loop re-reads the launch arguments through a
// laundered kernarg pointer and takes its lane id from an opaque asm (the
// superblock wavefront's recipe, flow_impl.hpp), so nothing is hoisted out of
// the 19 inlined class bodies.
template <int BPC> struct ItemSched {
    int cls, first, count;
};
// (segment, class) schedule position of wave item gw: as k_recon's prologue
template <int BPC, int GRP>
__device__ __forceinline__ ItemSched<BPC> item_sched(const ReconArgs<BPC> *ka, int gw) {
    constexpr int NC = DGPU_N_RECT_TX_SIZES;
    constexpr int SL = kSegInner;
    int wpre[NC + 1];
#pragma unroll
    for (int c = 0; c <= NC; c++) wpre[c] = ka->wpre[c];
    const int wgrp = wpre[NC] * SL;
    const int sg = gw / wgrp, r = gw - sg * wgrp;
    int pos = 0, wpre_p = 0;
#pragma unroll
    for (int c = 1; c < NC; c++) {
        const bool ge = r >= wpre[c] * SL;
        pos = ge ? c : pos;
        wpre_p = ge ? wpre[c] : wpre_p;
    }
    ItemSched<BPC> s;
    s.cls = order_class(pos);
    const int wp = ka->wps[pos], cs0 = ka->class_start[s.cls], cs1 = ka->class_end[s.cls];
    const int lg = (int)((kLog2Lanes >> (3 * s.cls)) & 7);
    const int U = 64 >> lg;
    const int r2 = r - wpre_p * SL;
    const int sl = SL == 1 ? 0 : r2 / wp;
    const int seg = sg * SL + sl;
    s.first = cs0 + (seg * wp + r2 - sl * wp) * U;
    s.count = min(U, cs1 - s.first);
    return s;
}

#if DGPU_PERSIST >= 3
// [0..7] per-XCD tickets (3), [8] finished waves, [16 + 16 * shard + xcd]
// sharded tickets (4: 16 shards per XCD, each on its own 64-B line)
static __device__ int g_persist_ctr[16 + 16 * 16 * 8];
#endif
#ifndef DGPU_PERSIST_WPE
#define DGPU_PERSIST_WPE 5
#endif
template <int BPC, int GRP>
__global__ __launch_bounds__((64 * waves_per_block<BPC, GRP>()))
__attribute__((amdgpu_waves_per_eu(DGPU_PERSIST_WPE))) void k_recon_p(ReconArgs<BPC> a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int WL = wave_lds<BPC, GRP>();
    constexpr int WPB = waves_per_block<BPC, GRP>();
    using P = typename Px<BPC>::pixel;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwaves = a.nwaves;
    // the item blocks k_recon's grid would have had, per XCD
    const int NB = ((nwaves + WPB - 1) / WPB + 7) & ~7;
    const int NBX = NB >> 3, NLX = gridDim.x >> 3;
    const int x = blockIdx.x & 7, k0 = blockIdx.x >> 3;
    using PT = PlaneTab<BPC>;
    __shared__ PT ptab[WPB];
    PT &pt = ptab[wave];
    {
        const int t = threadIdx.x & 63;
        const int tr = min(t, DGPU_MAX_REFS * 3 - 1), td = min(t, 2);
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
    }
    wave_sync();
    uint8_t *wl = lds + wave * WL;
    const Dav1dGpuIntraEdge rec{};
#if defined(__HIP_DEVICE_COMPILE__)
    const __attribute__((address_space(4))) ReconArgs<BPC> *ka40 =
        (const __attribute__((address_space(4))) ReconArgs<BPC> *)__builtin_amdgcn_kernarg_segment_ptr();
#endif
    if constexpr (DGPU_PERSIST == 4) {
        // sharded tickets: the waves of launched block b take the items of
        // XCD x that are congruent to shard (b >> 3) % 16 (a uniform sample
        // of the XCD's schedule), one counter per (shard, XCD) on its own line
        const int items = NBX * WPB, base = x * items;
        const int sh = k0 & 15;
        int *ctr = &g_persist_ctr[16 + (sh * 8 + x) * 16];
        const int lane = unit_lane();
        int t = 0;
        if (lane == 0) t = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = __builtin_amdgcn_readfirstlane(t);
#pragma unroll 1
        while (sh + 16 * t < items && base + sh + 16 * t < nwaves) {
            asm volatile("" ::: "memory");
            int tn = 0;
            if (lane == 0) tn = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if defined(__HIP_DEVICE_COMPILE__)
            const __attribute__((address_space(4))) ReconArgs<BPC> *ka4 = ka40;
            asm volatile("" : "+s"(ka4));
            const ReconArgs<BPC> *ka = (const ReconArgs<BPC> *)ka4;
#else
            const ReconArgs<BPC> *ka = &a;
#endif
            const int gw = base + sh + 16 * t;
            const ItemSched<BPC> s = item_sched<BPC, GRP>(ka, gw);
            if (s.count > 0) {
                const Dav1dGpuUnit u =
                    bld(ka->units + s.first + min(lane >> (int)((kLog2Lanes >> (3 * s.cls)) & 7), s.count - 1));
                dispatch<BPC, GRP>(*ka, pt, u, rec, s.cls, s.first, s.count, wl, gw);
            }
            t = __builtin_amdgcn_readfirstlane(tn);
        }
        if (lane == 0) {
            const int total = (int)gridDim.x * WPB;
            if (__hip_atomic_fetch_add(&g_persist_ctr[8], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == total - 1) {
                for (int i = 0; i < 16 * 8; i++)
                    __hip_atomic_store(&g_persist_ctr[16 + i * 16], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&g_persist_ctr[8], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    } else if constexpr (DGPU_PERSIST == 3) {
        // dynamic: the waves of an XCD take that XCD's wave items in schedule
        // order from a ticket counter (the next ticket is fetched before the
        // current item's class code runs); the last wave to finish resets the
        // counters for the next launch on the stream (experiment only: two
        // launches in flight on different streams would share them)
        const int items = NBX * WPB, base = x * items;
        const int lane = unit_lane();
        int t = 0;
        if (lane == 0) t = __hip_atomic_fetch_add(&g_persist_ctr[x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = __builtin_amdgcn_readfirstlane(t);
#pragma unroll 1
        while (t < items && base + t < nwaves) {
            asm volatile("" ::: "memory");
            int tn = 0;
            if (lane == 0) tn = __hip_atomic_fetch_add(&g_persist_ctr[x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if defined(__HIP_DEVICE_COMPILE__)
            const __attribute__((address_space(4))) ReconArgs<BPC> *ka4 = ka40;
            asm volatile("" : "+s"(ka4));
            const ReconArgs<BPC> *ka = (const ReconArgs<BPC> *)ka4;
#else
            const ReconArgs<BPC> *ka = &a;
#endif
            const int gw = base + t;
            const ItemSched<BPC> s = item_sched<BPC, GRP>(ka, gw);
            if (s.count > 0) {
                const Dav1dGpuUnit u =
                    bld(ka->units + s.first + min(lane >> (int)((kLog2Lanes >> (3 * s.cls)) & 7), s.count - 1));
                dispatch<BPC, GRP>(*ka, pt, u, rec, s.cls, s.first, s.count, wl, gw);
            }
            t = __builtin_amdgcn_readfirstlane(tn);
        }
        if (lane == 0) {
            const int total = (int)gridDim.x * WPB;
            if (__hip_atomic_fetch_add(&g_persist_ctr[8], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == total - 1)
                for (int i = 0; i < 9; i++) __hip_atomic_store(&g_persist_ctr[i], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if constexpr (DGPU_PERSIST >= 2) {
        // the next item's schedule and descriptor are loaded before the
        // current item's class code runs
        int k = k0, gw = (x * NBX + k) * WPB + wave;
        if (k >= NBX || gw >= nwaves) return;
        ItemSched<BPC> s = item_sched<BPC, GRP>(&a, gw);
        Dav1dGpuUnit un{};
        if (s.count > 0) un = bld(a.units + s.first + min(unit_lane() >> (int)((kLog2Lanes >> (3 * s.cls)) & 7), s.count - 1));
#pragma unroll 1
        for (;;) {
            asm volatile("" ::: "memory");
#if defined(__HIP_DEVICE_COMPILE__)
            const __attribute__((address_space(4))) ReconArgs<BPC> *ka4 = ka40;
            asm volatile("" : "+s"(ka4));
            const ReconArgs<BPC> *ka = (const ReconArgs<BPC> *)ka4;
#else
            const ReconArgs<BPC> *ka = &a;
#endif
            const ItemSched<BPC> cur = s;
            const Dav1dGpuUnit u = un;
            k += NLX;
            gw = (x * NBX + k) * WPB + wave;
            const bool more = k < NBX && gw < nwaves;
            if (more) {
                s = item_sched<BPC, GRP>(ka, gw);
                if (s.count > 0)
                    un = bld(ka->units + s.first + min(unit_lane() >> (int)((kLog2Lanes >> (3 * s.cls)) & 7), s.count - 1));
            }
            if (cur.count > 0) dispatch<BPC, GRP>(*ka, pt, u, rec, cur.cls, cur.first, cur.count, wl, gw);
            if (!more) break;
        }
    } else {
        // one item at a time: only the loop counter crosses the class code
#pragma unroll 1
        for (int k = k0; k < NBX; k += NLX) {
            asm volatile("" ::: "memory");
            const int gw = (x * NBX + k) * WPB + wave;
            if (gw >= nwaves) break;
#if defined(__HIP_DEVICE_COMPILE__)
            const __attribute__((address_space(4))) ReconArgs<BPC> *ka4 = ka40;
            asm volatile("" : "+s"(ka4));
            const ReconArgs<BPC> *ka = (const ReconArgs<BPC> *)ka4;
#else
            const ReconArgs<BPC> *ka = &a;
#endif
            const ItemSched<BPC> s = item_sched<BPC, GRP>(ka, gw);
            if (s.count <= 0) continue;
            const Dav1dGpuUnit u =
                bld(ka->units + s.first + min(unit_lane() >> (int)((kLog2Lanes >> (3 * s.cls)) & 7), s.count - 1));
            dispatch<BPC, GRP>(*ka, pt, u, rec, s.cls, s.first, s.count, wl, gw);
        }
    }
}

// resident workgroups of k_recon_p on this device (cached per device)
template <int BPC, int GRP> static int persist_blocks(int lds) {
    static int cached[16] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
    if (!cached[dev]) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)k_recon_p<BPC, GRP>,
                                                         64 * waves_per_block<BPC, GRP>(), lds) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 0;
        cached[dev] = ((per_cu * cus) & ~7);
    }
    return cached[dev];
}

}  // namespace dgpu
