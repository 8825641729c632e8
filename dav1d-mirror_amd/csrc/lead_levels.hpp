// lead_levels.hpp -- DGPU_IS_LEVEL0_BATCH (include/dav1d_gpu.h): how many
// leading levels of a persistent schedule run as ordinary fused launches
// ahead of the persistent kernel (edges.hip launches them, flow_impl.hpp
// leaves them out of its task list).  Level 0 always; then each following
// level while it holds at least kLeadLevelUnits units: there the launch's
// full-occupancy throughput beats the persistent kernel's per-task ticket
// and agent-scope release, and its one dependency step costs a launch
// boundary (the 4K mixed frame: 170.6k units at level 0, 15.3k, 11.0k, 8.4k,
// 6.8k, ... 2.0k at level 10, then a tail of 35 levels with 9.1k units).
#pragma once
#include <stdlib.h>

#include "dav1d_gpu.h"

namespace dgpu {

constexpr int kLeadLevelUnits = 2048;
inline int lead_level_units() {   // DAV1D_GPU_LEAD_UNITS (tuning): the threshold
    static const int v = [] {
        const char *e = getenv("DAV1D_GPU_LEAD_UNITS");
        return e ? atoi(e) : kLeadLevelUnits;
    }();
    return v;
}

inline int lead_levels(const Dav1dGpuIntraSchedule *s) {
    if (!(s->flags & DGPU_IS_LEVEL0_BATCH) || s->n_levels <= 0) return 0;
    const int t = lead_level_units();
    int k = 1;
    while (k < s->n_levels && s->unit_start[k + 1] - s->unit_start[k] >= t) k++;
    return k;
}

}  // namespace dgpu
