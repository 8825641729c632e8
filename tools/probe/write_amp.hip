// Probe: WRITE_SIZE (rocprofv3) of one 3840x2160 u8 plane written in
// different store patterns, to separate the cost of partial-line stores from
// the order in which units write (k_recon's 3.4x write amplification).
//   hipcc -O3 --offload-arch=gfx950 tools/probe/write_amp.hip -o /tmp/write_amp
//   rocprofv3 --pmc WRITE_SIZE -- /tmp/write_amp
// Kernels (one dispatch each, in this order):
//   k<0> 16 B per lane, whole rows (the coalesced baseline)
//   k<1> 4 B per lane, whole rows
//   k<2> 4x4 blocks, 2 lanes per block (2 rows of 4 B each), blocks in raster
//        order, 32 per wave (k_recon's 4x4 class, spatially sorted)
//   k<3> the same blocks in a random order over the whole plane
//   k<4> random order inside 8 horizontal bands, band = the workgroup's XCD
//        (blockIdx % 8), as k_recon's XCD-contiguous schedule
//   k<5> 4x4 blocks in raster order, but every block row stored twice by
//        different waves far apart in time (the same line written partially
//        at two times)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

constexpr int W = 3840, H = 2160, BW = W / 4, BH = H / 4, NB = BW * BH;

template <int MODE>
__global__ __launch_bounds__(256) void k(uint8_t *dst, const int32_t *perm, int nwaves) {
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gw >= nwaves) return;
    if (MODE == 0) {   // 16 B per lane: a wave writes 1 KB of one row
        const size_t o = (size_t)gw * 1024 + lane * 16;
        if (o < (size_t)W * H) *(uint4 *)(dst + o) = make_uint4(o, o + 1, o + 2, o + 3);
        return;
    }
    if (MODE == 1) {   // 4 B per lane: 256 B per wave
        const size_t o = (size_t)gw * 256 + lane * 4;
        if (o < (size_t)W * H) *(uint32_t *)(dst + o) = (uint32_t)o;
        return;
    }
    // block modes: a wave = 32 blocks, 2 lanes per block
    const int slot = gw * 32 + (lane >> 1);
    const int half = lane & 1;
    int b = slot;
    if (MODE == 3 || MODE == 4) b = perm[slot];
    if (MODE == 5) b = (slot < NB) ? slot : slot - NB;   // two passes
    if (b >= NB) return;
    const int bx = b % BW, by = b / BW;
    uint8_t *p = dst + (size_t)(by * 4 + 2 * half) * W + bx * 4;
    *(uint32_t *)p = 0x01010101u * (uint32_t)b;
    *(uint32_t *)(p + W) = 0x02020202u * (uint32_t)b;
}

int main() {
    uint8_t *dst;
    int32_t *perm3, *perm4;
    hipMalloc(&dst, (size_t)W * H + 4096);
    hipMalloc(&perm3, sizeof(int32_t) * NB);
    hipMalloc(&perm4, sizeof(int32_t) * NB);
    std::vector<int32_t> p(NB);
    for (int i = 0; i < NB; i++) p[i] = i;
    std::mt19937 rng(1);
    std::shuffle(p.begin(), p.end(), rng);
    hipMemcpy(perm3, p.data(), sizeof(int32_t) * NB, hipMemcpyHostToDevice);
    // mode 4: slot s of workgroup g (4 waves x 32 blocks = 128 slots) takes
    // the next random block of band g % 8
    {
        std::vector<std::vector<int32_t>> band(8);
        for (int b = 0; b < NB; b++) band[(b / BW) * 8 / BH].push_back(b);
        for (auto &v : band) std::shuffle(v.begin(), v.end(), rng);
        std::vector<size_t> at(8, 0);
        // every slot the launch below can address: (nw_blk + 32) waves x 32
        const size_t nslots = ((size_t)(NB + 31) / 32 + 32) * 32;
        std::vector<int32_t> q(nslots + 128, NB);
        // workgroups are dealt round-robin over XCDs: give workgroup g band g % 8
        for (int g = 0;; g++) {
            bool any = false;
            const int bb = g % 8;
            for (int s = 0; s < 128; s++) {
                if (at[bb] < band[bb].size()) {
                    q[(size_t)g * 128 + s] = band[bb][at[bb]++];
                    any = true;
                }
            }
            bool left = false;
            for (int k = 0; k < 8; k++) left |= at[k] < band[k].size();
            if (!left || (size_t)(g + 1) * 128 + 128 > nslots) break;
            (void)any;
        }
        p.assign(q.begin(), q.begin() + NB);
        std::vector<int32_t> all(q.begin(), q.end());
        int32_t *tmp;
        hipMalloc(&tmp, sizeof(int32_t) * all.size());
        hipMemcpy(tmp, all.data(), sizeof(int32_t) * all.size(), hipMemcpyHostToDevice);
        hipFree(perm4);
        perm4 = tmp;
    }
    hipMemset(dst, 0, (size_t)W * H);
    hipDeviceSynchronize();
    const int nw_rows16 = (W * H + 1023) / 1024, nw_rows4 = (W * H + 255) / 256, nw_blk = (NB + 31) / 32;
    for (int rep = 0; rep < 3; rep++) {
        k<0><<<(nw_rows16 + 3) / 4, 256>>>(dst, nullptr, nw_rows16);
        k<1><<<(nw_rows4 + 3) / 4, 256>>>(dst, nullptr, nw_rows4);
        k<2><<<(nw_blk + 3) / 4, 256>>>(dst, nullptr, nw_blk);
        k<3><<<(nw_blk + 3) / 4, 256>>>(dst, perm3, nw_blk);
        k<4><<<(nw_blk + 3) / 4 + 8, 256>>>(dst, perm4, nw_blk + 32);
        k<5><<<(2 * nw_blk + 3) / 4, 256>>>(dst, nullptr, 2 * nw_blk);
    }
    hipDeviceSynchronize();
    printf("plane bytes %d\n", W * H);
    return 0;
}
