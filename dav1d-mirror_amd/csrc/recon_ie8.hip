// recon_ie8.hip -- 8bpc instantiation of the intra wavefront's fused
// reconstruction launch (recon_ie.hpp); its own TU so it compiles in
// parallel with the unit batch and leaves that code unchanged.
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
