// Latency micro-benchmarks for the engine's design choices (one wave, s_memtime):
// dependent chains of s_load (constant space), ds_read_b32 + readfirstlane,
// v_readlane -> SALU, global_load (L2-resident), and a global store -> load
// round trip.  Build: hipcc --offload-arch=gfx950 -O3 -o latency latency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CAS __attribute__((address_space(4)))
#define N 1024

__global__ void k_sload(const uint32_t* chain, uint64_t* out) {
    const CAS uint32_t* c = (const CAS uint32_t*)chain;
    uint32_t i = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) i = c[i];
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}

__global__ void k_lds(const uint32_t* chain, uint64_t* out) {
    __shared__ uint32_t s[1024];
    for (int j = threadIdx.x; j < 1024; j += 64) s[j] = chain[j];
    __syncthreads();
    uint32_t i = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) i = __builtin_amdgcn_readfirstlane(s[i]);
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}

__global__ void k_readlane(const uint32_t* chain, uint64_t* out) {
    uint32_t v = chain[threadIdx.x] & 63u;
    uint32_t i = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) i = __builtin_amdgcn_readlane(v, i) ;
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}

__global__ void k_gload(const uint32_t* chain, uint64_t* out) {
    uint32_t i = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) i = __builtin_amdgcn_readfirstlane(__builtin_nontemporal_load(chain + i) & 1023u);
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}

// store a value, read it back (different address each time), dependent chain
__global__ void k_storeload(uint32_t* buf, uint64_t* out) {
    uint32_t i = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) {
        if (threadIdx.x == 0) buf[(k * 16 + 1) & 0xffff] = i + 7;
        __builtin_amdgcn_s_waitcnt(0);
        i = __builtin_amdgcn_readfirstlane(((volatile uint32_t*)buf)[(k * 16 + 1) & 0xffff]) - 6;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}

// store-only stream: one 48-B record per iteration (12 lanes x 4 B), no waits
__global__ void k_store(uint32_t* buf, uint64_t* out) {
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) if (threadIdx.x < 12) buf[k * 12 + threadIdx.x] = k;
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; }
}

__global__ void k_store4(uint32_t* buf, uint64_t* out) {      // 3 lanes x 16 B
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) if (threadIdx.x < 3) ((uint4*)buf)[k * 3 + threadIdx.x] = make_uint4(k, k, k, k);
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; }
}
__global__ void k_store1(uint32_t* buf, uint64_t* out) {      // 1 lane x 4 B
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) if (threadIdx.x == 0) buf[k * 12] = k;
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; }
}
__global__ void k_store64(uint32_t* buf, uint64_t* out) {     // 64 lanes x 4 B
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) buf[k * 64 + threadIdx.x] = k;
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; }
}
__global__ void k_valu(const uint32_t* chain, uint64_t* out) { // dependent v_add chain
    uint32_t v = chain[threadIdx.x];
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) { asm volatile("v_add_u32 %0, %0, 1" : "+v"(v)); }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = v; }
}
__global__ void k_salu(const uint32_t* chain, uint64_t* out) { // dependent s_add chain
    uint32_t v = __builtin_amdgcn_readfirstlane(chain[0]);
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) { asm volatile("s_add_u32 %0, %0, 1" : "+s"(v)); }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = v; }
}
__global__ void k_vs(const uint32_t* chain, uint64_t* out) {   // VALU->SALU->VALU ping-pong (readfirstlane)
    uint32_t v = chain[threadIdx.x];
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; ++k) { uint32_t s = __builtin_amdgcn_readfirstlane(v); asm volatile("s_add_u32 %0, %0, 1" : "+s"(s)); v = v + s; }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = v; }
}

int main() {
    uint32_t h[65536];
    for (int j = 0; j < 65536; ++j) h[j] = (uint32_t)((j * 37 + 11) % 1024);
    uint32_t* d; uint64_t* o; uint64_t r[2];
    hipMalloc(&d, sizeof(h)); hipMalloc(&o, 16);
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    const char* names[] = {"s_load chain (constant AS)", "ds_read+readfirstlane chain", "v_readlane chain",
                           "global_load (nt) + readfirstlane chain", "store->waitcnt->load chain", "48-B record store stream (12 lanes x 4 B)",
                           "48-B record store stream (3 lanes x 16 B)", "4-B store stream (1 lane)", "256-B store stream (64 lanes)",
                           "dependent v_add chain", "dependent s_add chain", "readfirstlane->s_add->v_add chain"};
    for (int t = 0; t < 12; ++t) {
        for (int rep = 0; rep < 2; ++rep) {
            switch (t) {
            case 0: k_sload<<<1, 64>>>(d, o); break;
            case 1: k_lds<<<1, 64>>>(d, o); break;
            case 2: k_readlane<<<1, 64>>>(d, o); break;
            case 3: k_gload<<<1, 64>>>(d, o); break;
            case 4: k_storeload<<<1, 64>>>(d, o); break;
            case 5: k_store<<<1, 64>>>(d, o); break;
            case 6: k_store4<<<1, 64>>>(d, o); break;
            case 7: k_store1<<<1, 64>>>(d, o); break;
            case 8: k_store64<<<1, 64>>>(d, o); break;
            case 9: k_valu<<<1, 64>>>(d, o); break;
            case 10: k_salu<<<1, 64>>>(d, o); break;
            case 11: k_vs<<<1, 64>>>(d, o); break;
            }
            hipDeviceSynchronize();
        }
        hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
        printf("%-42s %8.1f cycles/iter\n", names[t], (double)r[0] / N);
    }
    return 0;
}
