// Probe: vector-load throughput on gfx950 by access shape.  Every wave
// issues ITER loads; lane addresses follow the pattern under test inside a
// 2 MiB L2-resident buffer.  Reports wave-load instructions per CU-us.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x3a1 __attribute__((ext_vector_type(3), aligned(1)));
typedef uint32_t u32x4a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int ITER = 64;

// MODE: 0 dword aligned, 1 dwordx3 unaligned (+1 byte), 2 dwordx4 aligned,
// 3 dwordx4 unaligned (+1), 4 dwordx3 aligned
template <int MODE>
__global__ __launch_bounds__(256) void k(const uint8_t *buf, uint32_t *out, int lanes_per_line, int stride) {
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t acc = 0;
    // lanes_per_line lanes share one 128-B line; lines of one instruction are
    // `stride` bytes apart (a picture row pitch)
    const int li = lane / lanes_per_line, sub = lane % lanes_per_line;
    for (int i = 0; i < ITER; i++) {
        const uint32_t base = ((uint32_t)(w * 97 + i * 61) * 4096u) & ((1u << 21) - 1);
        const uint32_t off = (base + (uint32_t)li * stride + (uint32_t)sub * (128 / lanes_per_line)) & ((1u << 21) - 64);
        const uint8_t *p = buf + off;
        if (MODE == 0) acc += *(const uint32_t *)p;
        if (MODE == 1) { u32x3a1 v = *(const u32x3a1 *)(p + 1); acc += v.x ^ v.y ^ v.z; }
        if (MODE == 2) { u32x4 v = *(const u32x4 *)p; acc += v.x ^ v.y ^ v.z ^ v.w; }
        if (MODE == 3) { u32x4a1 v = *(const u32x4a1 *)(p + 1); acc += v.x ^ v.y ^ v.z ^ v.w; }
        if (MODE == 4) { u32x3a1 v = *(const u32x3a1 *)(p + 4); acc += v.x ^ v.y ^ v.z; }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE>
static void run(const char *name, const uint8_t *buf, uint32_t *out, int lpl, int stride) {
    const int blocks = 256 * 8;   // 8 blocks (32 waves) per CU
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k<MODE><<<blocks, 256>>>(buf, out, lpl, stride);
    hipEventRecord(e0);
    k<MODE><<<blocks, 256>>>(buf, out, lpl, stride);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double instr = (double)blocks * 4 * ITER;
    printf("%-20s lanes/line=%2d stride=%5d: %7.1f us  %6.2f wave-loads per CU-us  (%.1f CU-cycles@2.4GHz each)\n",
           name, lpl, stride, ms * 1e3, instr / 256 / (ms * 1e3), 256 * ms * 1e-3 * 2.4e9 / instr);
}

int main() {
    uint8_t *buf;
    uint32_t *out;
    hipMalloc(&buf, 4 << 20);
    hipMemset(buf, 1, 4 << 20);
    hipMalloc(&out, 64 << 20);
    for (int lpl : {1, 4, 16, 64}) {
        run<0>("dword aligned", buf, out, lpl, 4096);
        run<4>("dwordx3 dw-aligned", buf, out, lpl, 4096);
        run<1>("dwordx3 unaligned", buf, out, lpl, 4096);
        run<2>("dwordx4 aligned", buf, out, lpl, 4096);
        run<3>("dwordx4 unaligned", buf, out, lpl, 4096);
    }
    return 0;
}
