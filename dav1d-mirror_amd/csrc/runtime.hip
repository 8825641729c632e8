// runtime.hip -- per-call staging runtime + library-level C entry points.
#include "runtime.hpp"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>

#include "bounds.hpp"
#include "dav1d_gpu.h"

namespace dgpu {

std::mutex &fallback_mutex() {
    static std::mutex m;
    return m;
}

// DGPU_BOUNDS builds: the calling thread's registered device buffers
std::vector<BndRange> &bnd_extra() {
    static thread_local std::vector<BndRange> v;
    return v;
}

// ---- sticky error ------------------------------------------
static std::atomic<int> g_error{0};        // first latched error, 0 = none
static std::atomic<long> g_fail_after{-2}; // DAV1D_GPU_FAIL_AFTER: -2 unread, -1 off

// Test hook: DAV1D_GPU_FAIL_AFTER=n makes the (n+1)-th HIP call of the
// per-call tier fail as if the runtime had returned an error.
static bool injected_failure() {
    long n = g_fail_after.load(std::memory_order_relaxed);
    if (n == -2) {
        const char *e = getenv("DAV1D_GPU_FAIL_AFTER");
        n = e ? strtol(e, nullptr, 0) : -1;
        g_fail_after.store(n);
    }
    if (n < 0) return false;
    return g_fail_after.fetch_sub(1) == 0;
}

void latch_error(int code, const char *what) {
    int expect = 0;
    if (g_error.compare_exchange_strong(expect, code))
        fprintf(stderr, "dav1d-gpu: %s failed (error %d); GPU DSP entries disabled until "
                        "dav1d_gpu_clear_error()\n", what, code);
}

bool gpu_usable() { return g_error.load(std::memory_order_relaxed) == 0; }

bool hip_ok(hipError_t e, const char *what) {
    if (e == hipSuccess && injected_failure()) e = hipErrorUnknown;
    if (e == hipSuccess) return true;
    latch_error((int)e, what);
    return false;
}

static thread_local int tls_device_req = 0;
static thread_local ThreadCtx tls_ctx;

bool ThreadCtx::reserve(size_t bytes) {
    if (bytes <= cap) return true;
    size_t n = cap ? cap : (size_t)1 << 20;
    while (n < bytes) n <<= 1;
    if (host) (void)hipHostFree(host);
    if (dev) (void)hipFree(dev);
    host = dev = nullptr;
    cap = 0;
    if (!hip_ok(hipHostMalloc((void **)&host, n, hipHostMallocDefault), "hipHostMalloc")) {
        host = nullptr;
        return false;
    }
    if (!hip_ok(hipMalloc((void **)&dev, n), "hipMalloc")) {
        dev = nullptr;
        return false;
    }
    cap = n;
    return true;
}

ThreadCtx::~ThreadCtx() {
    // errors ignored: at process exit the HIP runtime may already be gone
    if (device < 0 && !host && !dev) return;
    if (device >= 0) (void)hipSetDevice(device);
    if (stream) (void)hipStreamDestroy(stream);
    if (host) (void)hipHostFree(host);
    if (dev) (void)hipFree(dev);
    stream = nullptr;
    host = dev = nullptr;
    cap = 0;
}

ThreadCtx *thread_ctx() {
    ThreadCtx &c = tls_ctx;
    if (c.device != tls_device_req || !c.stream) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
            latch_error(-1, "device lookup (no HIP device)");
            return nullptr;
        }
        if (!hip_ok(hipSetDevice(tls_device_req), "hipSetDevice")) return nullptr;
        if (c.stream) (void)hipStreamDestroy(c.stream);
        if (c.host) (void)hipHostFree(c.host);
        if (c.dev) (void)hipFree(c.dev);
        c.stream = nullptr;
        c.host = c.dev = nullptr;
        c.cap = 0;
        c.device = -1;
        if (!hip_ok(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking), "hipStreamCreate")) {
            c.stream = nullptr;
            return nullptr;
        }
        c.device = tls_device_req;
    } else if (!hip_ok(hipSetDevice(c.device), "hipSetDevice")) {
        return nullptr;
    }
    return &c;
}

int Stager::add(const void *base, ptrdiff_t stride, long bx0, long bx1, long y0, long y1, int dir) {
    Rect r;
    r.base = (const uint8_t *)base;
    r.stride = stride;
    r.bx0 = bx0; r.bx1 = bx1; r.y0 = y0; r.y1 = y1;
    r.dir = dir;
    r.pitch = ((size_t)(bx1 - bx0) + 15) & ~(size_t)15;
    if (r.pitch == 0) r.pitch = 16;
    r.off = 0;
    rects_.push_back(r);
    return (int)rects_.size() - 1;
}

bool Stager::upload() {
    ctx_ = nullptr;
    if (!gpu_usable()) return false;
    ThreadCtx *c = thread_ctx();
    if (!c) return false;
    ctx_ = c;
    // inputs, then in/out, then outputs: H2D covers [0, in_end_), D2H covers
    // the in/out + output tail.
    size_t off = 0;
    for (int pass = 1; pass <= 3; pass++) {
        const int want = pass == 1 ? 1 : pass == 2 ? 3 : 2;
        for (auto &r : rects_)
            if (r.dir == want) {
                r.off = off;
                off += r.pitch * (size_t)(r.y1 - r.y0);
                off = (off + 255) & ~(size_t)255;
            }
        if (pass == 2) in_end_ = off;
    }
    total_ = off ? off : 256;
    if (!ctx_->reserve(total_)) return false;
    size_t out_begin = in_end_;
    for (auto &r : rects_)
        if (r.dir == 3 && r.off < out_begin) out_begin = r.off;
    for (auto &r : rects_) {
        if (!(r.dir & 1)) continue;
        const long rb = r.bx1 - r.bx0;
        for (long y = r.y0; y < r.y1; y++)
            memcpy(ctx_->host + r.off + (y - r.y0) * r.pitch, r.base + y * r.stride + r.bx0, rb);
    }
    if (in_end_ &&
        !hip_ok(hipMemcpyAsync(ctx_->dev, ctx_->host, in_end_, hipMemcpyHostToDevice, ctx_->stream), "H2D"))
        return false;
    return true;
}

bool Stager::finish() {
    if (!ctx_) return false;
    // every step must succeed before the first output byte is scattered back
    bool ok = hip_ok(hipGetLastError(), "kernel launch");
    size_t lo = total_;
    for (auto &r : rects_)
        if ((r.dir & 2) && r.off < lo) lo = r.off;
    if (ok && lo < total_)
        ok = hip_ok(hipMemcpyAsync(ctx_->host + lo, ctx_->dev + lo, total_ - lo, hipMemcpyDeviceToHost,
                                   ctx_->stream), "D2H");
    // drain the stream even after a failure: the staging buffer is reused
    const hipError_t se = hipStreamSynchronize(ctx_->stream);
    ok = ok && hip_ok(se, "hipStreamSynchronize");
    if (!ok) return false;
    for (auto &r : rects_) {
        if (!(r.dir & 2)) continue;
        const long rb = r.bx1 - r.bx0;
        uint8_t *b = const_cast<uint8_t *>(r.base);
        for (long y = r.y0; y < r.y1; y++)
            memcpy(b + y * r.stride + r.bx0, ctx_->host + r.off + (y - r.y0) * r.pitch, rb);
    }
    return true;
}

}  // namespace dgpu

extern "C" int dav1d_gpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int dav1d_gpu_set_device(int device) {
    int n = dav1d_gpu_device_count();
    if (device < 0 || device >= n) return -1;
    dgpu::tls_device_req = device;
    return 0;
}

extern "C" const char *dav1d_gpu_version(void) { return "dav1d-gpu gfx950 r6"; }

extern "C" int dav1d_gpu_get_error(void) { return dgpu::g_error.load(); }

extern "C" int dav1d_gpu_clear_error(void) { return dgpu::g_error.exchange(0); }

extern "C" int dav1d_gpu_debug_register_buffer(const void *p, size_t bytes, int id) {
    if (!p) dgpu::bnd_extra().clear();
    else if (bytes) dgpu::bnd_extra().push_back(dgpu::BndRange{p, bytes, id});
    return 0;
}
