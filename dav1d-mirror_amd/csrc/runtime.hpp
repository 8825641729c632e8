// runtime.hpp -- host-side plumbing for the per-call (drop-in) tier.
//
// Each table entry of the reference (src/mc.h, src/ipred.h, src/itx.h) takes
// borrowed host pointers and must return with its outputs written
// (synchronous semantics, reentrant from n_tc worker threads).
// A Stager gathers exactly the byte extents the reference reads (inputs),
// writes (outputs) or updates in place (in/out), packs them into one pinned
// buffer, does one H2D copy, runs the kernel on the calling thread's own
// stream, one D2H copy, and scatters the results back.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <mutex>
#include <vector>

namespace dgpu {

// Error contract: a per-call entry never aborts and never
// writes part of its outputs.  A HIP failure latches a process-wide sticky
// error (dav1d_gpu_get_error) and the entry then runs the C default the
// caller's table held before the _gpu_ hook overwrote it (the fallback
// tables below), or, when the library replaced the whole table, leaves its
// outputs untouched.  Once latched, later entries skip the GPU until the
// caller clears the error (the reference's own error latch,
// src/thread_task.c:453 / src/lib.c:715, is checked the same way).
bool hip_ok(hipError_t e, const char *what);   // false: error latched
void latch_error(int code, const char *what);
bool gpu_usable();                             // no error latched

// The caller's table entries before a _gpu_ hook overwrote them: every slot
// of `caller` that is not the GPU entry itself (a second hook call must not
// make the GPU its own fallback).  Contexts are arrays of function pointers.
// Decoders of one process may run their init hooks on several threads at
// once: the saves are serialised.  The itx and loop-restoration hooks take
// the bit depth (the reference's arch code installs different 10- and 12-bit
// entries, src/x86/itx.h, src/x86/looprestoration.h:62-88), so their 16bpc
// fallbacks are one table per bit depth, chosen by bitdepth_max at the call;
// the other hooks have none (the reference installs the same entries for 10
// and 12 bit).
std::mutex &fallback_mutex();
inline int fb16_slot(int bpc) { return bpc == 12; }
inline int fb16_slot_bdmax(int bitdepth_max) { return bitdepth_max > 1023; }
template <typename Ctx>
inline void save_fallback(Ctx *fb, const Ctx *caller, const Ctx *gpu) {
    std::lock_guard<std::mutex> lock(fallback_mutex());
    constexpr int n = sizeof(Ctx) / sizeof(void *);
    static_assert(sizeof(Ctx) % sizeof(void *) == 0, "function-pointer tables only");
    void *const *c = reinterpret_cast<void *const *>(caller);
    void *const *g = reinterpret_cast<void *const *>(gpu);
    void **f = reinterpret_cast<void **>(fb);
    for (int i = 0; i < n; i++)
        if (c[i] != g[i]) f[i] = c[i];
}
// run the fallback entry when the GPU path did not complete
#define DGPU_OR_FALLBACK(ok, fn, ...)          \
    do {                                       \
        if (!(ok)) {                           \
            auto f_ = (fn);                    \
            if (f_) f_(__VA_ARGS__);           \
        }                                      \
    } while (0)

struct ThreadCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    uint8_t *host = nullptr;  // pinned
    uint8_t *dev = nullptr;
    size_t cap = 0;
    bool reserve(size_t bytes);
    // A worker thread's stream and staging buffers die with the thread
    // (dav1d starts and joins its n_tc workers per decoder instance, so a
    // long-running process would otherwise leak them on every instance).
    ~ThreadCtx();
};
ThreadCtx *thread_ctx();   // nullptr (error latched) when no usable device

// A rectangle of bytes relative to a caller base pointer:
// rows [y0, y1), byte columns [bx0, bx1), caller row stride `stride` (may be
// negative).  The device copy uses a positive, 16-byte aligned pitch.
struct Rect {
    const uint8_t *base;
    ptrdiff_t stride;
    long bx0, bx1, y0, y1;
    int dir;        // 1 in, 2 out, 3 in/out
    size_t off;     // assigned device offset
    size_t pitch;
};

class Stager {
public:
    // Returns an index; the device pointer for the caller's `base` (byte
    // (0,0) of the rect's coordinate system) is origin(idx), pitch pitch(idx).
    int add(const void *base, ptrdiff_t stride, long bx0, long bx1, long y0, long y1, int dir);
    int in(const void *b, ptrdiff_t s, long bx0, long bx1, long y0, long y1) { return add(b, s, bx0, bx1, y0, y1, 1); }
    int out(void *b, ptrdiff_t s, long bx0, long bx1, long y0, long y1) { return add(b, s, bx0, bx1, y0, y1, 2); }
    int inout(void *b, ptrdiff_t s, long bx0, long bx1, long y0, long y1) { return add(b, s, bx0, bx1, y0, y1, 3); }
    // 1-D helpers (single row)
    int in1(const void *b, long bytes) { return add(b, 0, 0, bytes, 0, 1, 1); }
    int out1(void *b, long bytes) { return add(b, 0, 0, bytes, 0, 1, 2); }
    int inout1(void *b, long bytes) { return add(b, 0, 0, bytes, 0, 1, 3); }

    // Lays out the buffer and uploads the inputs; after this origin()/pitch()
    // are valid and the caller launches its kernel on stream().  false: the
    // GPU is unusable (error latched); launch nothing, write nothing.
    [[nodiscard]] bool upload();
    template <typename T> T *origin(int i) const {
        const Rect &r = rects_[i];
        return reinterpret_cast<T *>(ctx_->dev + r.off - r.y0 * (long)r.pitch - r.bx0);
    }
    ptrdiff_t pitch(int i) const { return (ptrdiff_t)rects_[i].pitch; }
    hipStream_t stream() const { return ctx_->stream; }
    // Downloads outputs, waits, scatters them back into the caller's memory
    // -- all of them, or (on any HIP error, then latched) none: false.
    [[nodiscard]] bool finish();

private:
    ThreadCtx *ctx_ = nullptr;
    std::vector<Rect> rects_;
    size_t in_end_ = 0, total_ = 0;
};

}  // namespace dgpu
