// mrg32k3a.h -- the MRG32k3a generator of ns-3's RngStream (L'Ecuyer, Simard, Chen, Kelton,
// "An object-oriented random-number package with many long streams and substreams",
// Operations Research 50(6), 2002), for the engine's ns-3 random-stream mode
// (prisma_params_t.rng_mode = PRISMA_RNG_NS3).
//
// ns-3 gives every RandomVariableStream object a stream of its own: the k-th object created
// in a run draws from stream k, whose initial state is the package seed (simSeed in all six
// components) advanced by k * 2^127 + run * 2^76 steps (RngStream(seed, stream, substream)).
// A jump of 2^127 steps is the matrix pair J = (A1^(2^127) mod m1, A2^(2^127) mod m2); the
// engine keeps, per replica, the initial state of the next stream to be created and applies J
// once per creation.  The host derives every power it needs by squaring A1 / A2
// (mrg_pow2); tests/test_mrg32k3a.py checks those powers against the constants the paper
// publishes (A1p127, A2p127, A1p76, A2p76).
#pragma once
#include <stdint.h>

namespace prisma {

constexpr uint64_t kMrgM1 = 4294967087ull, kMrgM2 = 4294944443ull;

// one 3x3 matrix per component, row-major: [0..8] mod m1, [9..17] mod m2
struct MrgMat { uint32_t a[18]; };

// s <- M s (both components)
__host__ __device__ inline void mrg_apply(const uint32_t* M, uint32_t* s) {
    uint32_t r[6];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const uint64_t m = c ? kMrgM2 : kMrgM1;
        const uint32_t* A = M + 9 * c;
        const uint32_t* v = s + 3 * c;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            uint64_t acc = 0;
#pragma unroll
            for (int j = 0; j < 3; ++j) acc = (acc + (uint64_t)A[3 * i + j] * v[j] % m) % m;
            r[3 * c + i] = (uint32_t)acc;
        }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) s[i] = r[i];
}

// RngStream::RandU01 from state s (advancing s by one step): the double arithmetic of the
// package, exact since every product is below 2^53
__host__ __device__ inline double mrg_u01(uint32_t* s) {
    double p1 = 1403580.0 * (double)s[1] - 810728.0 * (double)s[0];
    int64_t k = (int64_t)(p1 / 4294967087.0);
    p1 -= (double)k * 4294967087.0;
    if (p1 < 0.0) p1 += 4294967087.0;
    s[0] = s[1]; s[1] = s[2]; s[2] = (uint32_t)p1;
    double p2 = 527612.0 * (double)s[5] - 1370589.0 * (double)s[3];
    k = (int64_t)(p2 / 4294944443.0);
    p2 -= (double)k * 4294944443.0;
    if (p2 < 0.0) p2 += 4294944443.0;
    s[3] = s[4]; s[4] = s[5]; s[5] = (uint32_t)p2;
    return (p1 > p2) ? (p1 - p2) * 2.328306549295727688e-10 : (p1 - p2 + 4294967087.0) * 2.328306549295727688e-10;
}

// host helpers: matrix product, A^(2^e) by squaring, A^n for any n
inline MrgMat mrg_mul(const MrgMat& X, const MrgMat& Y) {
    MrgMat Z;
    for (int c = 0; c < 2; ++c) {
        const uint64_t m = c ? kMrgM2 : kMrgM1;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                uint64_t acc = 0;
                for (int k = 0; k < 3; ++k) acc = (acc + (uint64_t)X.a[9 * c + 3 * i + k] * Y.a[9 * c + 3 * k + j] % m) % m;
                Z.a[9 * c + 3 * i + j] = (uint32_t)acc;
            }
    }
    return Z;
}
inline MrgMat mrg_identity() {
    MrgMat I = {};
    for (int c = 0; c < 2; ++c)
        for (int i = 0; i < 3; ++i) I.a[9 * c + 4 * i] = 1u;
    return I;
}
inline MrgMat mrg_base() {                       // one step of the recurrence
    MrgMat A = {};
    A.a[1] = 1u; A.a[5] = 1u;
    A.a[6] = (uint32_t)(kMrgM1 - 810728u); A.a[7] = 1403580u; A.a[8] = 0u;
    A.a[9 + 1] = 1u; A.a[9 + 5] = 1u;
    A.a[9 + 6] = (uint32_t)(kMrgM2 - 1370589u); A.a[9 + 7] = 0u; A.a[9 + 8] = 527612u;
    return A;
}
inline MrgMat mrg_pow2(int e) {                  // A^(2^e)
    MrgMat A = mrg_base();
    for (int i = 0; i < e; ++i) A = mrg_mul(A, A);
    return A;
}
inline MrgMat mrg_pow(MrgMat M, uint64_t n) {    // M^n
    MrgMat R = mrg_identity();
    while (n) {
        if (n & 1u) R = mrg_mul(R, M);
        M = mrg_mul(M, M);
        n >>= 1;
    }
    return R;
}

}  // namespace prisma
