// recon_sb16.hip -- 16bpc instantiation of the intra wavefront's
// superblock launch (DGPU_IS_SB, k_flow_sb in flow_impl.hpp); its own TU so
// its class code compiles in parallel with recon_ie16.hip.
#define DGPU_LANE_OPAQUE 1   // (recon_kernel.hpp: no lane-derived value hoisted out of the task loops)
#include "recon_ie.hpp"

namespace dgpu {
int flow_sb_launch16(const Dav1dGpuFrameBatch *b, const Dav1dGpuIntraEdgeBatch *e, const Dav1dGpuIntraSchedule *s,
                   const std::vector<FlowTask> &tasks, hipStream_t stream) {
    return launch_flow_sb<16>(b, e, s, tasks, stream);
}
}  // namespace dgpu
