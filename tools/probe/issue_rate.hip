// Probe: VALU issue rate per SIMD vs waves per SIMD on gfx950.
// Each wave runs 4 independent v_dot4 chains (and, in a second kernel,
// plain v_add_u32 chains); s_memtime brackets the loop.  Reports cycles per
// wave-instruction per SIMD = (cycles per wave) / (instrs per wave * waves/SIMD).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int KIND>
__global__ __launch_bounds__(256) void k(int *out, unsigned long long *cyc, int iters, int seed) {
    int a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;
    int b0 = a0 + 11, b1 = a0 + 13, b2 = a0 + 17, b3 = a0 + 19;
    const int x = seed * 0x01010101;
    unsigned long long t0 = clock64();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            if (KIND == 0) {
                a0 = __builtin_amdgcn_sdot4(a0, x, a0, false);
                a1 = __builtin_amdgcn_sdot4(a1, x, a1, false);
                a2 = __builtin_amdgcn_sdot4(a2, x, a2, false);
                a3 = __builtin_amdgcn_sdot4(a3, x, a3, false);
                b0 = __builtin_amdgcn_sdot4(b0, x, b0, false);
                b1 = __builtin_amdgcn_sdot4(b1, x, b1, false);
                b2 = __builtin_amdgcn_sdot4(b2, x, b2, false);
                b3 = __builtin_amdgcn_sdot4(b3, x, b3, false);
            } else {
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b0));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a1) : "v"(b1));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(b2));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a3) : "v"(b3));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(b0) : "v"(a0));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(b1) : "v"(a1));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(b2) : "v"(a2));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(b3) : "v"(a3));
            }
        }
    }
    unsigned long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + b0 + b1 + b2 + b3;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
    int ncu = 256;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) == hipSuccess) ncu = p.multiProcessorCount;
    const int iters = 256;
    int *out;
    unsigned long long *cyc;
    hipMalloc(&out, 64 * 1024 * 1024);
    hipMalloc(&cyc, 8 * 1024 * 1024);
    unsigned long long *h = (unsigned long long *)malloc(8 * 1024 * 1024);
    for (int kind = 0; kind < 2; kind++) {
        for (int wps = 1; wps <= 8; wps *= 2) {
            const int blocks = ncu * wps;   // 4 waves per block -> wps waves per SIMD
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                if (kind == 0) k<0><<<blocks, 256>>>(out, cyc, iters, 3);
                else k<1><<<blocks, 256>>>(out, cyc, iters, 3);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h, cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < blocks * 4; i++) s += h[i];
            s /= blocks * 4;
            const double instr = iters * 16.0 * 8;
            const double total = instr * blocks * 4;   // wave-instructions
            printf("%s waves/SIMD=%d: %.1f cyc/wave-instr per wave; %.2f cyc per instr per SIMD; "
                   "%.3f ms -> %.2f T wave-instr/s (%.2f per CU-ns)\n",
                   kind ? "v_add_u32" : "v_dot4   ", wps, s / instr, s / instr / wps, ms,
                   total / ms * 1e-9, total / ms * 1e-6 / ncu);
        }
    }
    printf("CUs=%d clock=%d kHz\n", ncu, p.clockRate);
    return 0;
}
