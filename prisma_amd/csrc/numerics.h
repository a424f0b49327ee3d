// numerics.h — scalar building blocks shared by host sizing code and the
// gfx950 kernels.  Every expression here is evaluated with the same IEEE-754
// operation sequence on host and device (compile with -ffp-contract=off), so
// results are bit-identical to the CPU oracle's independent restatement.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// ---------------------------------------------------------------------------
// numeric building blocks (device + host, identical IEEE sequences)
// ---------------------------------------------------------------------------
__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    uint32_t c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    c[0] = c0; c[1] = c1; c[2] = c2; c[3] = c3;
}

// ln(x) for x > 0 normal: range reduction to [sqrt(1/2), sqrt(2)] and the
// atanh series; + - * / only.
__host__ __device__ inline double det_log(double x) {
    uint64_t bits = __builtin_bit_cast(uint64_t, x);
    int e = (int)((bits >> 52) & 0x7ff) - 1023;
    double m = __builtin_bit_cast(double, (bits & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL);
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double z = s * s;
    double p = 2.0 / 19.0;
    p = p * z + 2.0 / 17.0;
    p = p * z + 2.0 / 15.0;
    p = p * z + 2.0 / 13.0;
    p = p * z + 2.0 / 11.0;
    p = p * z + 2.0 / 9.0;
    p = p * z + 2.0 / 7.0;
    p = p * z + 2.0 / 5.0;
    p = p * z + 2.0 / 3.0;
    double logm = 2.0 * s + s * (z * p);
    double de = (double)e;
    return de * 6.93147180369123816490e-01 + (de * 1.90821492927058770002e-10 + logm);
}

// expm1(x) for x <= 0 in double with + - * / only: x = k ln2 + r, |r| <= ln2/2,
// expm1(r) by its Taylor series, then 2^k (1 + expm1(r)) - 1.  Used by the
// in-kernel DQN MLP's ELU; identical bits on host and device.
__host__ __device__ inline double det_expm1(double x) {
    if (x < -60.0) return -1.0;
    double t = x * 1.4426950408889634 + 0.5;
    int64_t ki = (int64_t)t;                       // truncation toward zero ...
    if ((double)ki > t) ki -= 1;                   // ... to floor
    double k = (double)ki;
    double r = (x - k * 6.93147180369123816490e-01) - k * 1.90821492927058770002e-10;
    double p = r * (1.0 / 87178291200.0);          // 1/14!
    p = (p + 1.0 / 6227020800.0) * r;
    p = (p + 1.0 / 479001600.0) * r;
    p = (p + 1.0 / 39916800.0) * r;
    p = (p + 1.0 / 3628800.0) * r;
    p = (p + 1.0 / 362880.0) * r;
    p = (p + 1.0 / 40320.0) * r;
    p = (p + 1.0 / 5040.0) * r;
    p = (p + 1.0 / 720.0) * r;
    p = (p + 1.0 / 120.0) * r;
    p = (p + 1.0 / 24.0) * r;
    p = (p + 1.0 / 6.0) * r;
    p = (p + 0.5) * r;
    p = (p + 1.0) * r;                             // expm1(r)
    if (ki == 0) return p;
    double scale = __builtin_bit_cast(double, (uint64_t)(1023 + ki) << 52);
    return scale * (p + 1.0) - 1.0;
}

// expm1 for x <= 0 in fp32 with + - * and an int conversion only (the oracle's
// or_det_expm1f restates it: identical bits on host and device): Cody-Waite reduction
// x = k ln2 + r, |r| <= ln2/2, degree-7 Taylor polynomial, 2^k (1 + expm1(r)) - 1.
// Within 2 ulp of expm1 (tests/test_oracle.py); 7 % faster decisions than the f64 form.
__host__ __device__ inline float det_expm1f(float x) {
    if (!(x == x)) return x;                        // NaN
    if (x < -17.0f) return -1.0f;                   // expm1(-17) rounds to -1 + 1 ulp at most
    if (x > -5.9604645e-08f) return x;              // |x| < 2^-24: expm1(x) rounds to x
    const float t = x * 1.44269504f + 0.5f;
    int ki = (int)t;                                // truncation toward zero ...
    if ((float)ki > t) ki -= 1;                     // ... to floor
    const float k = (float)ki;
    const float r = (x - k * 0.693145751953125f) - k * 1.42860677e-06f;
    float p = r * 1.98412698e-04f;                  // 1/7!
    p = (p + 1.38888889e-03f) * r;
    p = (p + 8.33333333e-03f) * r;
    p = (p + 4.16666667e-02f) * r;
    p = (p + 1.66666667e-01f) * r;
    p = (p + 0.5f) * r;
    p = (p + 1.0f) * r;                             // expm1(r)
    if (ki == 0) return p;
    const float scale = __builtin_bit_cast(float, (uint32_t)(127 + ki) << 23);
    return scale * (p + 1.0f) - 1.0f;
}

// Keras ELU (alpha 1): x > 0 ? x : expm1(x)
__host__ __device__ inline float det_elu(float x) { return x > 0.0f ? x : det_expm1f(x); }

// det_elu without branches (the memory-resident engine's MLP, one wave per SIMD): det_expm1f's
// operations on every lane and its cases as selects -- the selected value is the same operation
// sequence's, so the bits equal det_elu's.  The branches had been exec-mask regions around ~25
// instructions (round 5: config 5 +1.7 %); the register-resident instances keep det_elu (at 2-4
// waves per SIMD the extra lanes' work and registers cost them 35-60 %).
__host__ __device__ inline float det_elu_sel(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    const float t = x * 1.44269504f + 0.5f;
    int ki = (int)t;
    ki = ((float)ki > t) ? ki - 1 : ki;
    const float k = (float)ki;
    const float r = (x - k * 0.693145751953125f) - k * 1.42860677e-06f;
    float p = r * 1.98412698e-04f;
    p = (p + 1.38888889e-03f) * r;
    p = (p + 8.33333333e-03f) * r;
    p = (p + 4.16666667e-02f) * r;
    p = (p + 1.66666667e-01f) * r;
    p = (p + 0.5f) * r;
    p = (p + 1.0f) * r;
    const float scale = __builtin_bit_cast(float, (uint32_t)(127 + ki) << 23);
    const float e = (ki == 0) ? p : scale * (p + 1.0f) - 1.0f;
    const float m = (x < -17.0f) ? -1.0f : ((x > -5.9604645e-08f) ? x : e);
    return (x > 0.0f || !(x == x)) ? x : m;
#else
    return det_elu(x);
#endif
}

// ns-3 Seconds(double) -> int64 ns (round to nearest)
__host__ __device__ inline int64_t sec_to_ns(double s) { return (int64_t)(s * 1e9 + 0.5); }
// a / d for a constant d with rd = RN(1 / d), on the device as q = a * rd and one FMA correction
// (Markstein): for 0 <= a < 2^53 and d = 1e9 or 1e6 this is the correctly rounded quotient, bit for
// bit the IEEE division the host and the oracle perform (tests/test_numerics_division.py checks
// 4e7 values; the C harness of this change checked 6.4e8), in 3 dependent f64 instructions
// instead of the ~10 of the hardware's division sequence (rcp, two Newton steps, div_fmas,
// div_fixup) -- three of which sat on every data arrival's dependent chain.
__host__ __device__ inline double div_const(double a, double d, double rd) {
#ifdef __HIP_DEVICE_COMPILE__
    const double q = a * rd;
    const double e = __builtin_fma(-q, d, a);
    return __builtin_fma(e, rd, q);
#else
    (void)rd;
    return a / d;
#endif
}
// ns-3 Time::GetSeconds()
__host__ __device__ inline double ns_to_sec(int64_t t) { return div_const((double)t, 1e9, 1e-9); }
// microseconds as Python's float of the "%f" string (forwarder.py:360)
__host__ __device__ inline double us_to_sec(uint64_t us) { return div_const((double)us, 1e6, 1e-6); }

// t / 1000 and t / 10^9 for 0 <= t < 2^42 ns (sim_time_s <= 4095, checked on the host) on the
// vector unit: floor(t * c) with c the double nearest 10^-3 (10^-9) is exact there -- both
// doubles lie above the true reciprocals, so a multiple of the divisor never lands below its
// quotient, and any other t sits at least 1/divisor above an integer, far beyond the product's
// rounding error (< 2^-20 here).  The scalar unit's 64-bit division by a constant is ~18
// instructions, and the scalar unit is the headline kernel's busiest resource.
__host__ __device__ inline uint64_t div_1e3(uint64_t t) {
#ifdef __HIP_DEVICE_COMPILE__
    return (uint64_t)(uint32_t)__builtin_floor((double)t * 0.001);
#else
    return t / 1000u;
#endif
}
__host__ __device__ inline uint64_t div_1e9(uint64_t t) {
#ifdef __HIP_DEVICE_COMPILE__
    return (uint64_t)(uint32_t)__builtin_floor((double)t * 1e-9);
#else
    return t / 1000000000u;
#endif
}

// microseconds of std::to_string(GetSeconds()) (%f, ties-to-even on the
// exact binary value) as Python reads them back (packet-manager.cc:127-128).
__host__ __device__ inline uint64_t py_micros(int64_t t) {
    uint64_t u = div_1e3((uint64_t)t);                  // t >= 0
    int64_t r = t - (int64_t)u * 1000;
    if (r != 500) return r < 500 ? u : u + 1;
    double x = ns_to_sec(t);
    uint64_t b = __builtin_bit_cast(uint64_t, x);
    int ex = (int)((b >> 52) & 0x7ff);
    uint64_t mant = (b & 0x000fffffffffffffULL) | (ex ? 0x0010000000000000ULL : 0);
    if (!ex) ex = 1;
    int sh = 1075 - ex;                      // x = mant * 2^-sh, sh > 0 here
    // lhs = mant * 2e6 (< 2^75), rhs = (2u+1) << sh, compared as 128-bit
    const uint64_t k = 2000000ull;
    uint64_t lo = mant * k;
#ifdef __HIP_DEVICE_COMPILE__
    uint64_t hi = __umul64hi(mant, k);
#else
    uint64_t hi = (uint64_t)(((unsigned __int128)mant * k) >> 64);
#endif
    uint64_t v = 2 * u + 1, rhi, rlo;
    if (sh >= 64) { rhi = v << (sh - 64); rlo = 0; }
    else if (sh == 0) { rhi = 0; rlo = v; }
    else { rhi = v >> (64 - sh); rlo = v << sh; }
    if (hi != rhi) return hi > rhi ? u + 1 : u;
    if (lo != rlo) return lo > rlo ? u + 1 : u;
    return (u & 1) ? u + 1 : u;
}

__host__ __device__ inline double py_reward(int64_t t_now, uint32_t us_prev) {
    return us_to_sec(py_micros(t_now)) - us_to_sec(us_prev);
}

