// recon8.hip -- 8bpc batch tier entry point (include/dav1d_gpu.h)
#include "recon_impl.hpp"

extern "C" int dav1d_gpu_recon_8bpc(const Dav1dGpuFrameBatch *b, void *stream) {
    return dgpu::launch<8>(b, (hipStream_t)stream);
}

// LDS bytes per workgroup of one kernel (group 0 small, 1 large
// -- up to 32x32 --, 2 huge -- a 64-point side); `big` != 0 selects group 2
// for compatibility.  Diagnostics only.
extern "C" int dav1d_gpu_recon_lds_bytes(int bpc, int group) {
    using namespace dgpu;
    if (bpc == 8)
        return group == 0 ? waves_per_block<8, 0>() * wave_lds<8, 0>()
             : group == 1 ? waves_per_block<8, 1>() * wave_lds<8, 1>()
                          : waves_per_block<8, 2>() * wave_lds<8, 2>();
    return group == 0 ? waves_per_block<16, 0>() * wave_lds<16, 0>()
         : group == 1 ? waves_per_block<16, 1>() * wave_lds<16, 1>()
                      : waves_per_block<16, 2>() * wave_lds<16, 2>();
}
