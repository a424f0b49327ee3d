// prisma_engine_lite_mlp.hip -- the register-resident engine's step kernels with the in-kernel
// DQN-buffer policy and without the --train echo / notify_dest code paths (step_kernel.h):
// configs 3 and 4.
#include "step_kernel.h"

const void* prisma_pick_step_lite_mlp(int fs, int ls, bool tun) { return pick_step<false, true>(fs, ls, tun); }

PRISMA_TU_TIMING(prisma_debug_timing_lite_mlp)
