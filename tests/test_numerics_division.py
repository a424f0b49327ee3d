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
