// recon8.hip -- 8bpc batch tier entry point (include/dav1d_gpu.h)
#include "recon_impl.hpp"

extern "C" int dav1d_gpu_recon_8bpc(const Dav1dGpuFrameBatch *b, void *stream) {
    return dgpu::launch<8>(b, (hipStream_t)stream);
}

// LDS bytes per workgroup of one kernel (group 0 small + large -- up to
// 32x32 --, 1 large when the groups are split, 2 huge -- a 64-point side --,
// 3 warp).  Diagnostics only.
template <int BPC> static int lds_bytes(int group) {
    using namespace dgpu;
    switch (group) {
    case 0: return waves_per_block<BPC, 0>() * wave_lds<BPC, 0>();
    case 1: return waves_per_block<BPC, 1>() * wave_lds<BPC, 1>();
    case 2: return waves_per_block<BPC, 2>() * wave_lds<BPC, 2>();
    case 3: return waves_per_block<BPC, 3>() * wave_lds<BPC, 3>();
    default: return -1;
    }
}
extern "C" int dav1d_gpu_recon_lds_bytes(int bpc, int group) {
    return bpc == 8 ? lds_bytes<8>(group) : lds_bytes<16>(group);
}
