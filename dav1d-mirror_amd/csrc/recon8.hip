// recon8.hip -- 8bpc batch tier entry point (include/dav1d_gpu.h)
#include "recon_impl.hpp"

extern "C" int dav1d_gpu_recon_8bpc(const Dav1dGpuFrameBatch *b, void *stream) {
    return dgpu::launch<8>(b, (hipStream_t)stream);
}

// LDS bytes per 256-thread workgroup of each launch (roofline notes)
extern "C" int dav1d_gpu_recon_lds_bytes(int bpc, int big) {
    if (bpc == 8) return 4 * (big ? dgpu::ClassSet<true>::wave_lds<8>() : dgpu::ClassSet<false>::wave_lds<8>());
    return 4 * (big ? dgpu::ClassSet<true>::wave_lds<16>() : dgpu::ClassSet<false>::wave_lds<16>());
}
