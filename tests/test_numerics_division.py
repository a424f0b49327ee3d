"""The device's constant divisions (prisma_amd/csrc/numerics.h div_const: q = a * RN(1/d), then one
FMA correction) equal IEEE division bit for bit for the kernels' operands: a = t ns < 2^42 over
d = 1e9 (ns_to_sec, ns-3's GetSeconds) and a = microseconds < 2^32 over d = 1e6 (the reward's
"%f" times, forwarder.py:360). The oracle divides; the kernels may not diverge from it by an ulp."""
import os
import subprocess
import tempfile

C_SRC = r'''
#include <stdio.h>
#include <stdint.h>
#include <math.h>
/* numerics.h div_const, device branch */
static double div_const(double a, double d, double rd) { double q = a * rd; double e = fma(-q, d, a); return fma(e, rd, q); }
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
int main(void) {
    const double D[2] = {1e9, 1e6}, RD[2] = {1e-9, 1e-6};
    const int BITS[2] = {42, 32};
    long bad = 0, n = 0;
    for (int k = 0; k < 2; ++k) {
        for (int64_t t = 0; t < 4000000; ++t, ++n)                     /* every small operand */
            if (div_const((double)t, D[k], RD[k]) != (double)t / D[k]) bad++;
        for (long i = 0; i < 8000000; ++i) {
            const int sh = (int)(xr() % (uint64_t)BITS[k]) + 1;        /* every magnitude */
            const int64_t t = (int64_t)(xr() & ((1ull << sh) - 1));
            n++; if (div_const((double)t, D[k], RD[k]) != (double)t / D[k]) bad++;
            const int64_t m = (int64_t)(xr() % ((1ull << BITS[k]) / (uint64_t)D[k] + 1)) * (int64_t)D[k]
                              + (int64_t)(xr() % 2001) - 1000;          /* around multiples of d */
            if (m >= 0) { n++; if (div_const((double)m, D[k], RD[k]) != (double)m / D[k]) bad++; }
        }
    }
    printf("%ld %ld\n", n, bad);
    return 0;
}
'''


def test_device_constant_division_equals_ieee_division():
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "div.c"), os.path.join(d, "div")
        open(src, "w").write(C_SRC)
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", exe, src, "-lm"])
        n, bad = map(int, subprocess.check_output([exe], text=True).split())
    assert n > 3e7 and bad == 0


C_DEG = r'''
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
/* engine_core.h div_deg: a / d for the node degree d with rd = RN(1/d) */
static float div_deg(float a, float d, float rd) { float q = a * rd; float e = fmaf(-q, d, a); return fmaf(e, rd, q); }
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
int main(void) {
    long bad = 0, n = 0;
    for (int d = 1; d <= 64; ++d) {
        const float fd = (float)d, rd = 1.0f / fd;
        for (uint32_t u = 0x3f800000u; u < 0x40000000u; u += 7u) {      /* the binade [1, 2) */
            float a; memcpy(&a, &u, 4); n++; if (div_deg(a, fd, rd) != a / fd) bad++;
        }
        for (int i = 0; i < 300000; ++i) {                              /* every exponent from 2^-120 */
            uint32_t u = 0x03800000u + (uint32_t)(xr() % (0x7f800000u - 0x03800000u));
            float a; memcpy(&a, &u, 4); n++; if (div_deg(a, fd, rd) != a / fd) bad++;
        }
        for (uint32_t k = 0; k < 400000; ++k) {                         /* integer sums (queued bytes) */
            const float a = (float)k; n++; if (div_deg(a, fd, rd) != a / fd) bad++;
        }
    }
    printf("%ld %ld\n", n, bad);
    return 0;
}
'''


def test_degree_division_equals_ieee_division():
    """engine_core.h div_deg (the memory-resident LayerNorm's mean and variance over the node degree):
    the Markstein correction with RN(1/d) equals IEEE float division for d = 1..64 on a sample here;
    scripts/checks/div_deg_exhaustive.c checks every float >= 2^-120 (0 mismatches)."""
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "deg.c"), os.path.join(d, "deg")
        open(src, "w").write(C_DEG)
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", exe, src, "-lm"])
        n, bad = map(int, subprocess.check_output([exe], text=True).split())
    assert n > 1e8 and bad == 0
