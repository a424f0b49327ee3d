// prisma_engine_mlp.hip -- the register-resident engine's step kernels with the in-kernel
// DQN-buffer policy and the --train echo / notify_dest code paths (step_kernel.h).
#include "step_kernel.h"

const void* prisma_pick_step_ctrl_mlp(int fs, int ls, bool tun) { return pick_step<true, true>(fs, ls, tun); }

PRISMA_TU_TIMING(prisma_debug_timing_mlp)
