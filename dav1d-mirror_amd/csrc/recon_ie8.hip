// recon_ie8.hip -- 8bpc instantiation of the intra wavefront's fused
// reconstruction launch (recon_ie.hpp); its own TU so it compiles in
// parallel with the unit batch and leaves that code unchanged.
// 8 lanes per 4x4 / 4x8 / 8x4 unit in the wavefront (round 5, measured:
// 4K one-tile intra frame 17.9 -> 17.1 ms, 2x2 tiles 10.9 -> 10.6 ms,
// bit-exact; 16 lanes 18.2 / 12.3 ms; profiles/r5/r5k_intra_lanes_ab.json).
// Only these TUs: the unit batch's classes keep their lanes.
#ifndef DGPU_IE_SMALL_LANES
#define DGPU_IE_SMALL_LANES 8
#endif
// Round 6: every other class one 4x2 output task per lane (W*H/8, at most
// 64) instead of the unit batch's LDS-bound counts: the flow trace had the
// tall classes (4x16: 4 lanes, 8x16: 8) as most levels' slowest task; 4K
// one-tile intra frame 16.95 -> 15.55 ms, 2x2 tiles 10.42 -> 9.52 ms,
// bit-exact (profiles/r6/r6e_intra_lanes_ab.json).
#ifndef DGPU_IE_WIDE_LANES
#define DGPU_IE_WIDE_LANES 1
#endif
#include "recon_ie.hpp"

int dgpu_recon_ie_8bpc(const Dav1dGpuFrameBatch *b, const Dav1dGpuIntraEdgeBatch *e, void *stream) {
    return dgpu::launch_ie<8>(b, e, (hipStream_t)stream);
}

int dgpu_recon_flow_8bpc(const Dav1dGpuFrameBatch *b, const Dav1dGpuIntraEdgeBatch *e, const Dav1dGpuIntraSchedule *s,
                          void *stream) {
    return dgpu::launch_flow<8>(b, e, s, (hipStream_t)stream);
}

int64_t dgpu_flow_workspace_bytes_8bpc(const Dav1dGpuIntraSchedule *s, int n_units) {
    return dgpu::flow_workspace_bytes<8>(s, n_units);
}
