// bounds.hpp -- the DGPU_BOUNDS diagnostics build's host-side buffer
// registry (recon_kernel.hpp: bnd_ok).  A caller that owns the device
// buffers of a batch (the recorder) lists each with its exact byte size
// before it launches; the batch launchers of a DGPU_BOUNDS build copy the
// list into the device range table, and every access outside all listed
// buffers and planes is then reported.  Product builds never read it.
#pragma once
#include <stddef.h>

#include <vector>

namespace dgpu {

// ids printed with the range table
enum BndId {
    BND_DST = 0, BND_REF = 1, BND_TOP = 2, BND_CFL = 3,
    BND_UNITS = 10, BND_RECS = 11, BND_COEF = 12, BND_EDGES = 13, BND_AUX = 14, BND_AUXPOOL = 15,
    BND_WORK = 16, BND_EMU = 17, BND_EMUJOBS = 18, BND_XUNITS = 19, BND_XAUX = 20,
    BND_TILES = 21, BND_PREDS = 22, BND_TXS = 23,   // the tile batch (dav1d_gpu_debug_register_buffer)
};
struct BndRange {
    const void *p;
    size_t bytes;
    int id;
};
std::vector<BndRange> &bnd_extra();   // the calling thread's list (runtime.hip)

}  // namespace dgpu
