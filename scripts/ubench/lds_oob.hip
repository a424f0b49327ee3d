// Probe: LDS atomics whose address lies past the workgroup's LDS allocation.  Lane 0 adds to
// a real slot, lanes 1-63 to an address far beyond the allocation.  Each workgroup then dumps
// its whole allocation; the host checks that only the real slots changed, in every workgroup
// (1024 of them, several resident per CU, so a stray add would land in a neighbour's words).
// Build: hipcc --offload-arch=gfx950 -O2 -o lds_oob lds_oob.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

constexpr int kWords = 1024;                 // 4 KiB of LDS per workgroup

__global__ void probe(uint32_t* out, uint32_t far) {
    extern __shared__ uint32_t lds[];
    const int lane = threadIdx.x;
    for (int i = lane; i < kWords; i += 64) lds[i] = 0x7f800001u + (uint32_t)i;   // NaN patterns
    if (lane == 0) lds[13] = 0u;                                                 // the f32 slot: +0.0
    __syncthreads();
    const uint32_t base = lane == 0 ? (uint32_t)(uintptr_t)&lds[5] : far;
    for (int r = 0; r < 100; ++r) {
        __asm__ volatile("ds_add_u32 %0, %1 offset:16" :: "v"(base), "v"(1u) : "memory");
        __asm__ volatile("ds_add_f32 %0, %1 offset:32" :: "v"(base), "v"(1.0f) : "memory");
    }
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = lane; i < kWords; i += 64) out[(size_t)blockIdx.x * kWords + i] = lds[i];
}

int main() {
    const int G = 1024;
    uint32_t* d;
    if (hipMalloc(&d, (size_t)G * kWords * 4) != hipSuccess) { printf("alloc failed\n"); return 2; }
    const uint32_t fars[] = {0x10000u, 0x40000u, 0x00ff0000u, 0xffff0000u};
    uint32_t* h = (uint32_t*)malloc((size_t)G * kWords * 4);
    int bad_total = 0;
    for (uint32_t far : fars) {
        hipLaunchKernelGGL(probe, dim3(G), dim3(64), kWords * 4, 0, d, far);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
        hipMemcpy(h, d, (size_t)G * kWords * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int g = 0; g < G; ++g)
            for (int i = 0; i < kWords; ++i) {
                uint32_t want = 0x7f800001u + (uint32_t)i;
                if (i == 9) want += 100u;                                // u32 slot: 100 adds of 1
                if (i == 13) want = 0x42c80000u;                         // f32 slot: 100.0f
                const uint32_t got = h[(size_t)g * kWords + i];
                if (got != want) {
                    if (bad < 5) printf("far=%#x wg=%d word %d: %#x want %#x\n", far, g, i, got, want);
                    bad++;
                }
            }
        printf("far=%#x: %d words differ\n", far, bad);
        bad_total += bad;
    }
    free(h);
    printf(bad_total ? "LDS_OOB_NOT_DISCARDED\n" : "LDS_OOB_DISCARDED\n");
    return bad_total ? 1 : 0;
}
