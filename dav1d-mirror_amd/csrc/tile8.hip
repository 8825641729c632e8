// tile8.hip -- 8bpc superblock-tile batch entry point (include/dav1d_gpu.h)
#include "tile_impl.hpp"

extern "C" int dav1d_gpu_recon_tiles_8bpc(const Dav1dGpuTileBatch *b, void *stream) {
    return dgpu::launch_tiles<8>(b, (hipStream_t)stream);
}
