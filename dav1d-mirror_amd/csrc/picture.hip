// picture.hip -- a Dav1dPicAllocator whose pictures live in HBM (SURVEY 8(f)
// row 2; include/dav1d_gpu.h, Dav1dGpuPicAllocator).
//
// dav1d calls alloc_picture_callback on its main thread and
// release_picture_callback from any frame thread (include/dav1d/picture.h:
// 110-145).  Geometry follows dav1d_default_picture_alloc (src/picture.c:
// 46-83) so every DSP and frame-tier entry sees the strides, alignment and
// over-read padding it would see with dav1d's own allocator.  Buffers are
// pooled per size (a decoder cycles through a handful of pictures of one
// size), so steady-state decoding allocates nothing.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <mutex>
#include <unordered_map>
#include <vector>

#include "dav1d_gpu.h"

static_assert(sizeof(Dav1dGpuPicture) == 272, "Dav1dPicture layout");
static_assert(offsetof(Dav1dGpuPicture, data) == 16 && offsetof(Dav1dGpuPicture, stride) == 40 &&
                  offsetof(Dav1dGpuPicture, p) == 56 && offsetof(Dav1dGpuPicture, allocator_data) == 264,
              "Dav1dPicture field offsets");

namespace {

constexpr size_t kAlign = 64;   // DAV1D_PICTURE_ALIGNMENT

struct Buf {
    void *base;
    size_t size;
};

struct Pool {
    int device, flags;
    std::mutex mu;
    std::unordered_map<size_t, std::vector<void *>> free_;
    long outstanding = 0;

    void *get(size_t size) {
        {
            std::lock_guard<std::mutex> lk(mu);
            auto it = free_.find(size);
            if (it != free_.end() && !it->second.empty()) {
                void *p = it->second.back();
                it->second.pop_back();
                outstanding++;
                return p;
            }
        }
        int prev = 0;
        (void)hipGetDevice(&prev);
        if (hipSetDevice(device) != hipSuccess) return nullptr;
        void *p = nullptr;
        hipError_t e = flags == DGPU_PIC_HOST_MAPPED ? hipHostMalloc(&p, size, hipHostMallocMapped)
                                                     : hipMalloc(&p, size);
        (void)hipSetDevice(prev);
        if (e != hipSuccess) return nullptr;
        std::lock_guard<std::mutex> lk(mu);
        outstanding++;
        return p;
    }
    void put(void *p, size_t size) {
        std::lock_guard<std::mutex> lk(mu);
        free_[size].push_back(p);
        outstanding--;
    }
};

struct Alloc {   // allocator_data: the buffer and its size class
    void *base;
    size_t size;
};

int pic_alloc(Dav1dGpuPicture *p, void *cookie) {
    Pool *pool = (Pool *)cookie;
    const int hbd = p->p.bpc > 8;
    const int aligned_w = (p->p.w + 127) & ~127, aligned_h = (p->p.h + 127) & ~127;
    const int has_chroma = p->p.layout != 0;
    const int ss_ver = p->p.layout == 1, ss_hor = p->p.layout != 3;
    ptrdiff_t y_stride = (ptrdiff_t)aligned_w << hbd;
    ptrdiff_t uv_stride = has_chroma ? y_stride >> ss_hor : 0;
    if (!(y_stride & 1023)) y_stride += kAlign;   // the default allocator's set-conflict padding
    if (!(uv_stride & 1023) && has_chroma) uv_stride += kAlign;
    const size_t y_sz = (size_t)y_stride * aligned_h;
    const size_t uv_sz = (size_t)uv_stride * (aligned_h >> ss_ver);
    const size_t size = y_sz + 2 * uv_sz + kAlign;
    Alloc *a = new (std::nothrow) Alloc{nullptr, size};
    if (!a) return -ENOMEM;
    a->base = pool->get(size);
    if (!a->base) {
        delete a;
        return -ENOMEM;
    }
    uint8_t *d = (uint8_t *)a->base;   // hipMalloc / hipHostMalloc: >= 256-byte aligned
    p->stride[0] = y_stride;
    p->stride[1] = uv_stride;
    p->data[0] = d;
    p->data[1] = has_chroma ? d + y_sz : nullptr;
    p->data[2] = has_chroma ? d + y_sz + uv_sz : nullptr;
    p->allocator_data = a;
    return 0;
}

void pic_release(Dav1dGpuPicture *p, void *cookie) {
    Pool *pool = (Pool *)cookie;
    Alloc *a = (Alloc *)p->allocator_data;
    if (!a) return;
    pool->put(a->base, a->size);
    delete a;
    p->allocator_data = nullptr;
}

}  // namespace

extern "C" int dav1d_gpu_pic_allocator_init(Dav1dGpuPicAllocator *a, int device, int flags) {
    if (!a || (flags != DGPU_PIC_DEVICE && flags != DGPU_PIC_HOST_MAPPED) || device < 0) return -1;
    Pool *pool = new (std::nothrow) Pool();
    if (!pool) return -1;
    pool->device = device;
    pool->flags = flags;
    a->cookie = pool;
    a->alloc_picture_callback = pic_alloc;
    a->release_picture_callback = pic_release;
    return 0;
}

extern "C" int dav1d_gpu_pic_allocator_close(Dav1dGpuPicAllocator *a) {
    if (!a || !a->cookie) return -1;
    Pool *pool = (Pool *)a->cookie;
    long left;
    {
        std::lock_guard<std::mutex> lk(pool->mu);
        left = pool->outstanding;
        for (auto &kv : pool->free_)
            for (void *p : kv.second) {
                if (pool->flags == DGPU_PIC_HOST_MAPPED) (void)hipHostFree(p);
                else (void)hipFree(p);
            }
        pool->free_.clear();
    }
    if (left == 0) {
        delete pool;
        a->cookie = nullptr;
    }
    return (int)left;
}

extern "C" int dav1d_gpu_picture_plane(const Dav1dGpuPicture *pic, int plane, Dav1dGpuPlane *out) {
    if (!pic || !out || plane < 0 || plane > 2 || !pic->data[plane]) return -1;
    const int ss_hor = plane && pic->p.layout != 3, ss_ver = plane && pic->p.layout == 1;
    out->data = pic->data[plane];
    out->stride = pic->stride[plane ? 1 : 0];
    out->w = (pic->p.w + ss_hor) >> ss_hor;
    out->h = (pic->p.h + ss_ver) >> ss_ver;
    return 0;
}
