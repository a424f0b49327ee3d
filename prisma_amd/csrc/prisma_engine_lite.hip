// prisma_engine_lite.hip -- the register-resident engine's table-policy step kernels without
// the --train echo and notify_dest code paths (step_kernel.h), picked by prisma_create when
// neither is set (every table-policy benchmark configuration, the headline among them).
#include "step_kernel.h"

const void* prisma_pick_step_lite(int fs, int ls, bool tun) { return pick_step<false, false>(fs, ls, tun); }

PRISMA_TU_TIMING(prisma_debug_timing_lite)
PRISMA_TU_WAVE_TIMES(prisma_debug_wave_times_lite)
