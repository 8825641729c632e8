// recon16.hip -- 16bpc (10/12-bit) batch tier entry point (include/dav1d_gpu.h)
#include "recon_impl.hpp"

extern "C" int dav1d_gpu_recon_16bpc(const Dav1dGpuFrameBatch *b, void *stream) {
    return dgpu::launch<16>(b, (hipStream_t)stream);
}
