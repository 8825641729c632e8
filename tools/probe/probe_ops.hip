// Probe: VOP3P dot asm vs builtins, unaligned multi-dword global loads.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
typedef short v2i16 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3a1 __attribute__((ext_vector_type(3), aligned(1)));
__global__ void k(const uint32_t *a, const uint32_t *b, int *o, const uint8_t *bytes, uint32_t *uo, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int d1, d2, d3, d4;
    asm("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(d1) : "v"(a[i]), "v"(b[i]), "s"(0x2002));
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d2) : "v"(a[i]), "v"(b[i]), "s"(32));
    asm("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(d3) : "v"(a[i]), "v"(b[i]), "v"(d1));
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d4) : "v"(a[i]), "v"(b[i]), "v"(d2));
    // mixed chain as in the kernel: asm VOP3P start, builtin accumulate
    int m1;
    asm("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(m1) : "v"(a[i] ^ 0x80808080u), "v"(b[i]), "s"(0x2002));
    const uint32_t al = __builtin_amdgcn_alignbyte(a[i], b[i], 1);
    m1 = __builtin_amdgcn_sdot4((int)al, (int)b[i], m1, false);
    const int m2 = __builtin_amdgcn_sdot4((int)al, (int)b[i],
                   __builtin_amdgcn_sdot4((int)(a[i] ^ 0x80808080u), (int)b[i], 0x2002, false), false);
    o[8 * n + 2 * i] = m1; o[8 * n + 2 * i + 1] = m2;
    o[8 * i + 0] = d1;
    o[8 * i + 1] = __builtin_amdgcn_sdot4((int)a[i], (int)b[i], 0x2002, false);
    o[8 * i + 2] = d2;
    o[8 * i + 3] = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, a[i]), __builtin_bit_cast(v2i16, b[i]), 32, false);
    o[8 * i + 4] = d3;
    o[8 * i + 5] = __builtin_amdgcn_sdot4((int)a[i], (int)b[i], o[8 * i + 1], false);
    o[8 * i + 6] = d4;
    o[8 * i + 7] = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, a[i]), __builtin_bit_cast(v2i16, b[i]), o[8 * i + 3], false);
    __shared__ const uint8_t *sp[1];
    if (threadIdx.x == 0) sp[0] = bytes;
    __syncthreads();
    const uint8_t *fb = sp[0];   // generic pointer through LDS -> flat loads
    u32x3a1 v = *reinterpret_cast<const u32x3a1 *>(fb + 3 * i + (i % 7));
    uo[3 * i] = v.x; uo[3 * i + 1] = v.y; uo[3 * i + 2] = v.z;
}
int main() {
    const int n = 4096;
    uint32_t *ha = (uint32_t *)malloc(n * 4), *hb = (uint32_t *)malloc(n * 4);
    uint8_t *hbytes = (uint8_t *)malloc(4 * n + 64);
    srand(1);
    for (int i = 0; i < n; i++) { ha[i] = rand() * 2654435761u; hb[i] = rand() * 2246822519u; }
    for (int i = 0; i < 4 * n + 64; i++) hbytes[i] = rand();
    uint32_t *da, *db, *duo; int *dout; uint8_t *dbytes;
    hipMalloc(&da, n * 4); hipMalloc(&db, n * 4); hipMalloc(&dout, n * 40); hipMalloc(&dbytes, 4 * n + 64);
    hipMalloc(&duo, n * 12);
    hipMemcpy(da, ha, n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dbytes, hbytes, 4 * n + 64, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(da, db, dout, dbytes, duo, n);
    int *ho = (int *)malloc(n * 40); uint32_t *huo = (uint32_t *)malloc(n * 12);
    hipMemcpy(ho, dout, n * 40, hipMemcpyDeviceToHost);
    hipMemcpy(huo, duo, n * 12, hipMemcpyDeviceToHost);
    int bad[4] = {0, 0, 0, 0}, badu = 0;
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < 4; j++) if (ho[8 * i + 2 * j] != ho[8 * i + 2 * j + 1]) {
            if (bad[j] < 3) printf("op %d i %d asm %d builtin %d a %08x b %08x\n", j, i, ho[8*i+2*j], ho[8*i+2*j+1], ha[i], hb[i]);
            bad[j]++;
        }
        for (int j = 0; j < 3; j++) {
            uint32_t ref; memcpy(&ref, hbytes + 3 * i + (i % 7) + 4 * j, 4);
            if (huo[3 * i + j] != ref) { if (badu < 3) printf("unaligned i %d j %d got %08x want %08x\n", i, j, huo[3*i+j], ref); badu++; }
        }
    }
    int badm = 0;
    for (int i = 0; i < n; i++) if (ho[8 * n + 2 * i] != ho[8 * n + 2 * i + 1]) badm++;
    printf("mixed chain bad %d\n", badm);
    printf("dot4k bad %d dot2k bad %d dot4 bad %d dot2 bad %d unaligned bad %d\n", bad[0], bad[1], bad[2], bad[3], badu);
    return 0;
}
