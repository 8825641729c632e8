// Probe: latency of a chain of dependent scalar loads from the kernel
// argument segment vs from a device buffer (gfx950), per wave, s_memtime.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

struct Big {
    int idx[64];
    int pad[128];
};

__global__ void k_arg(Big a, unsigned long long *out, int *sink) {
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(t0) :: "memory");
    int i = a.idx[0];
    i = a.idx[i & 63];
    i = a.idx[i & 63];
    i = a.idx[i & 63];
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(i) :: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = t1 - t0;
        sink[blockIdx.x] = i;
    }
}

__global__ void k_ptr(const Big *__restrict__ a, unsigned long long *out, int *sink) {
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(t0) :: "memory");
    int i = a->idx[0];
    i = a->idx[i & 63];
    i = a->idx[i & 63];
    i = a->idx[i & 63];
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(i) :: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = t1 - t0;
        sink[blockIdx.x] = i;
    }
}

static void report(const char *name, unsigned long long *d, int n) {
    std::vector<unsigned long long> h(n);
    hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("%-8s blocks=%6d  4 dependent loads: p10 %llu  p50 %llu  p90 %llu cycles\n", name, n, h[n / 10], h[n / 2],
           h[n * 9 / 10]);
}

int main() {
    Big a;
    for (int i = 0; i < 64; i++) a.idx[i] = (i * 7 + 3) & 63;
    Big *d;
    hipMalloc(&d, sizeof(Big));
    hipMemcpy(d, &a, sizeof(Big), hipMemcpyHostToDevice);
    unsigned long long *out;
    int *sink;
    hipMalloc(&out, 8 << 20);
    hipMalloc(&sink, 4 << 20);
    for (int n : {1, 256, 2048, 20000}) {
        for (int rep = 0; rep < 2; rep++) {
            k_arg<<<n, 64>>>(a, out, sink);
            hipDeviceSynchronize();
            if (rep) report("kernarg", out, n);
            k_ptr<<<n, 64>>>(d, out, sink);
            hipDeviceSynchronize();
            if (rep) report("devptr", out, n);
        }
    }
    return 0;
}
