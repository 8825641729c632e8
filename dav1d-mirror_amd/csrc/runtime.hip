// runtime.hip -- per-call staging runtime + library-level C entry points.
#include "runtime.hpp"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dav1d_gpu.h"

namespace dgpu {

[[noreturn]] void fatal(const char *what, hipError_t e) {
    fprintf(stderr, "dav1d-gpu: fatal HIP error in %s: %s (%d)\n", what,
            hipGetErrorString(e), (int)e);
    abort();
}

static thread_local int tls_device_req = 0;
static thread_local ThreadCtx tls_ctx;

void ThreadCtx::reserve(size_t bytes) {
    if (bytes <= cap) return;
    size_t n = cap ? cap : (size_t)1 << 20;
    while (n < bytes) n <<= 1;
    if (host) hip_check(hipHostFree(host), "hipHostFree");
    if (dev) hip_check(hipFree(dev), "hipFree");
    hip_check(hipHostMalloc((void **)&host, n, hipHostMallocDefault), "hipHostMalloc");
    hip_check(hipMalloc((void **)&dev, n), "hipMalloc");
    cap = n;
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

ThreadCtx &thread_ctx() {
    ThreadCtx &c = tls_ctx;
    if (c.device != tls_device_req || !c.stream) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
            fprintf(stderr, "dav1d-gpu: no HIP device available; the GPU DSP tables "
                            "cannot run (no CPU fallback by design)\n");
            abort();
        }
        hip_check(hipSetDevice(tls_device_req), "hipSetDevice");
        if (c.stream) hip_check(hipStreamDestroy(c.stream), "hipStreamDestroy");
        if (c.host) hip_check(hipHostFree(c.host), "hipHostFree");
        if (c.dev) hip_check(hipFree(c.dev), "hipFree");
        c.host = c.dev = nullptr;
        c.cap = 0;
        hip_check(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking), "hipStreamCreate");
        c.device = tls_device_req;
    } else {
        hip_check(hipSetDevice(c.device), "hipSetDevice");
    }
    return c;
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

void Stager::upload() {
    ctx_ = &thread_ctx();
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
    ctx_->reserve(total_);
    size_t out_begin = in_end_;
    for (auto &r : rects_)
        if (r.dir == 3 && r.off < out_begin) out_begin = r.off;
    for (auto &r : rects_) {
        if (!(r.dir & 1)) continue;
        const long rb = r.bx1 - r.bx0;
        for (long y = r.y0; y < r.y1; y++)
            memcpy(ctx_->host + r.off + (y - r.y0) * r.pitch, r.base + y * r.stride + r.bx0, rb);
    }
    if (in_end_)
        hip_check(hipMemcpyAsync(ctx_->dev, ctx_->host, in_end_, hipMemcpyHostToDevice, ctx_->stream),
                  "H2D");
}

void Stager::finish() {
    hip_check(hipGetLastError(), "kernel launch");
    size_t lo = total_;
    for (auto &r : rects_)
        if ((r.dir & 2) && r.off < lo) lo = r.off;
    if (lo < total_)
        hip_check(hipMemcpyAsync(ctx_->host + lo, ctx_->dev + lo, total_ - lo, hipMemcpyDeviceToHost,
                                 ctx_->stream), "D2H");
    hip_check(hipStreamSynchronize(ctx_->stream), "hipStreamSynchronize");
    for (auto &r : rects_) {
        if (!(r.dir & 2)) continue;
        const long rb = r.bx1 - r.bx0;
        uint8_t *b = const_cast<uint8_t *>(r.base);
        for (long y = r.y0; y < r.y1; y++)
            memcpy(b + y * r.stride + r.bx0, ctx_->host + r.off + (y - r.y0) * r.pitch, rb);
    }
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

extern "C" const char *dav1d_gpu_version(void) { return "dav1d-gpu gfx950 r1"; }
