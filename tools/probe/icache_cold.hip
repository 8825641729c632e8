// Probe: cost of executing cold straight-line code on gfx950.
// k_straight runs N_INSTR v_add_u32 as one straight-line block (4 B each);
// k_loop runs the same count as a small loop.  The difference per 64-B line
// is the instruction-fetch cost a wave pays on code the SQC has not cached.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ADD8(a, b)                                                   \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[0]) : "v"(b[0])); \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[1]) : "v"(b[1])); \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[2]) : "v"(b[2])); \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[3]) : "v"(b[3])); \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(b[0]) : "v"(a[0])); \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(b[1]) : "v"(a[1])); \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(b[2]) : "v"(a[2])); \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(b[3]) : "v"(a[3]));

template <int STRAIGHT, int NBLK>
__global__ __launch_bounds__(256) void k(int *out, unsigned long long *cyc) {
    int a[4], b[4];
    for (int i = 0; i < 4; i++) { a[i] = threadIdx.x * (i + 1); b[i] = a[i] + 7; }
    unsigned long long t0 = clock64();
    if (STRAIGHT) {
#pragma unroll
        for (int j = 0; j < NBLK; j++) { ADD8(a, b) }
    } else {
#pragma nounroll
        for (int j = 0; j < NBLK / 16; j++) {
#pragma unroll
            for (int u = 0; u < 16; u++) { ADD8(a, b) }
        }
    }
    unsigned long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a[0] + a[1] + a[2] + a[3] + b[0] + b[1] + b[2] + b[3];
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int S, int NB>
static void run(const char *name, int ncu, int wps, int *out, unsigned long long *cyc, unsigned long long *h) {
    const int blocks = ncu * wps;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k<S, NB><<<blocks, 256>>>(out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
    double s = 0, mx = 0;
    for (int i = 0; i < blocks * 4; i++) { s += h[i]; mx = h[i] > mx ? h[i] : mx; }
    s /= blocks * 4;
    const double n = NB * 8.0;
    printf("%-9s instrs=%6.0f (%5.1f KB) waves/SIMD=%d: mean %.0f cyc/wave (%.2f per instr, %.1f per 64B line) max %.0f; %.1f us\n",
           name, n, n * 4 / 1024, wps, s, s / n, s / (n * 4 / 64), mx, ms * 1e3);
}

int main() {
    int ncu = 256;
    int *out;
    unsigned long long *cyc, *h;
    hipMalloc(&out, 64 << 20);
    hipMalloc(&cyc, 8 << 20);
    h = (unsigned long long *)malloc(8 << 20);
    for (int rep = 0; rep < 2; rep++) {
        printf("rep %d\n", rep);
        for (int w = 1; w <= 8; w *= 2) {
            run<1, 1024>("straight", ncu, w, out, cyc, h);
            run<0, 1024>("loop", ncu, w, out, cyc, h);
            run<1, 256>("straight", ncu, w, out, cyc, h);
            run<0, 256>("loop", ncu, w, out, cyc, h);
        }
    }
    return 0;
}
