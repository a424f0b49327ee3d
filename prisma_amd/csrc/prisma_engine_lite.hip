// prisma_engine_lite.hip -- the register-resident engine's step kernels without the --train
// echo and notify_dest code paths (step_kernel.h), picked by prisma_create when neither is set
// (every table-policy benchmark configuration).  A separate translation unit so the two
// instance sets compile in parallel.
#include "step_kernel.h"

const void* prisma_pick_step_lite(int fs, int ls, bool mlp, bool tun) { return pick_step<false>(fs, ls, mlp, tun); }

#if PRISMA_TIMING
// diagnostic build only: this translation unit's per-phase cycle totals (scripts/timing.py)
extern "C" int prisma_debug_timing_lite(unsigned long long* out32) {
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_prisma_timing), 32 * sizeof(unsigned long long)) != hipSuccess) return -1;
    unsigned long long z[32] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_prisma_timing), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
