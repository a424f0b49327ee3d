// Exhaustive check behind engine_core.h div_deg (round 5): for every float a >= 2^-120 and every
// integer d in [1, 64], q = RN(a * RN(1/d)), e = fma(-q, d, a), fma(e, RN(1/d), q) == RN(a / d).
// Build: gcc -O2 -ffp-contract=off -o div_deg div_deg_exhaustive.c -lpthread -lm; run ./div_deg 1 8 ... 57 64
// Result (this container, 8 runs of 8 divisors): 0 mismatches for d = 1..64 (a below 2^-120 gives
// subnormal quotients, where the correction is not exact: d = 6 mismatches there; the kernels
// divide sums of non-negative integers or of squared deviations, never that small).
// exhaustive: for every positive finite float a and integer d in [1, 64]:
// y = RN(1/d); q = RN(a*y); r = fma(-q, d, a); q' = fma(r, y, q)  ==  RN(a/d) ?
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <stdlib.h>
#include <pthread.h>
static int D0, D1;
static long bad[65];
static void* run(void* arg) {
    int d = (int)(long)arg;
    float fd = (float)d, y = 1.0f / fd;
    long nb = 0;
    for (uint32_t u = 0x03800000u; u < 0x7f800000u; ++u) {   // positive normal floats
        float a; memcpy(&a, &u, 4);
        float q = a * y;
        float r = fmaf(-q, fd, a);
        float q2 = fmaf(r, y, q);
        float t = a / fd;
        if (memcmp(&q2, &t, 4) != 0) { if (nb < 3) printf("d=%d a=%a got %a want %a\n", d, a, q2, t); nb++; }
    }
    bad[d] = nb;
    return 0;
}
int main(int argc, char** argv) {
    D0 = atoi(argv[1]); D1 = atoi(argv[2]);
    pthread_t th[65];
    for (int d = D0; d <= D1; ++d) pthread_create(&th[d], 0, run, (void*)(long)d);
    for (int d = D0; d <= D1; ++d) pthread_join(th[d], 0);
    long tot = 0;
    for (int d = D0; d <= D1; ++d) { if (bad[d]) printf("d=%d bad=%ld\n", d, bad[d]); tot += bad[d]; }
    printf("d %d..%d total mismatches %ld\n", D0, D1, tot);
}
