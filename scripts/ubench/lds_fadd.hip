// Are LDS float atomics (ds_add_f32 / ds_add_f64, no return) bit-identical to
// sequential IEEE adds from one lane?  Prints mismatch counts over random
// sequences (incl. tiny and mixed-sign values).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#define N 4096
__global__ void k(const float* fin, const double* din, float* fout, double* dout) {
    __shared__ float f; __shared__ double d;
    if (threadIdx.x == 0) { f = 0; d = 0; }
    __syncthreads();
    for (int i = 0; i < N; ++i) {
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(&f, fin[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(&d, din[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        if (threadIdx.x == 0) { fout[i] = f; dout[i] = d; }
    }
}
int main() {
    static float fin[N], fo[N]; static double din[N], dout[N];
    int bad_f = 0, bad_d = 0;
    for (int trial = 0; trial < 8; ++trial) {
        srand(trial + 1);
        for (int i = 0; i < N; ++i) {
            double u = (rand() + 0.5) / (RAND_MAX + 1.0);
            double sc = (trial % 4 == 0) ? 1e-40 : (trial % 4 == 1) ? 1e-3 : (trial % 4 == 2) ? 1.0 : 1e-310;
            fin[i] = (float)((u - (trial & 4 ? 0.5 : 0.0)) * (trial % 4 == 3 ? 1e-3 : sc));
            din[i] = (u - (trial & 4 ? 0.5 : 0.0)) * sc;
        }
        float *a, *c; double *b, *e;
        hipMalloc(&a, sizeof(fin)); hipMalloc(&b, sizeof(din)); hipMalloc(&c, sizeof(fo)); hipMalloc(&e, sizeof(dout));
        hipMemcpy(a, fin, sizeof(fin), hipMemcpyHostToDevice); hipMemcpy(b, din, sizeof(din), hipMemcpyHostToDevice);
        k<<<1, 64>>>(a, b, c, e);
        hipMemcpy(fo, c, sizeof(fo), hipMemcpyDeviceToHost); hipMemcpy(dout, e, sizeof(dout), hipMemcpyDeviceToHost);
        float sf = 0; double sd = 0;
        int bf = 0, bd = 0;
        for (int i = 0; i < N; ++i) {
            sf = sf + fin[i]; sd = sd + din[i];
            if (memcmp(&sf, &fo[i], 4)) bf++;
            if (memcmp(&sd, &dout[i], 8)) bd++;
        }
        printf("trial %d: f32 mismatches %d, f64 mismatches %d (final %g / %g)\n", trial, bf, bd, (double)sf, sd);
        bad_f += bf; bad_d += bd;
        hipFree(a); hipFree(b); hipFree(c); hipFree(e);
    }
    printf("TOTAL f32 %d f64 %d\n", bad_f, bad_d);
    return 0;
}
