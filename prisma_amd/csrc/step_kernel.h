// step_kernel.h -- the register-resident engine's step kernel template and its instance table,
// included by prisma_engine.hip (instances with the --train echo / notify_dest code, CTRL) and
// prisma_engine_lite.hip (instances without it: the compiler allocates registers for every
// path a kernel contains, and these rarely-taken ones cost the common case ~2 %).
#pragma once
#include "engine_core.h"

// waves per SIMD the register allocator must leave room for: 4 (<= 128
// VGPRs) for small replicas so 4096 of them are resident on 256 CUs at
// once, 2 (<= 256) up to 512 flows x 128 links
template <int FS, int LS> struct StepOcc {
#ifdef PRISMA_DEV_WAVES
    static constexpr int waves = PRISMA_DEV_WAVES;     // register-allocation experiments only
#else
    static constexpr int waves = (FS <= 2 && LS == 1) ? 4 : (LS <= 2 ? 2 : 1);
#endif
#ifndef PRISMA_MLP_B_WIDE
#define PRISMA_MLP_B_WIDE 8
#endif
#ifndef PRISMA_MLP_B_NARROW
#define PRISMA_MLP_B_NARROW 4
#endif
    static constexpr int mlp_batch = waves >= 4 ? PRISMA_MLP_B_NARROW : PRISMA_MLP_B_WIDE;   // DQN-buffer loads in flight
};

// MLP: the in-kernel DQN-buffer policy is compiled in (mode 4 only); the table /
// external instances carry none of its code or registers.  CTRL: the --train echo and
// notify_dest paths are compiled in (used when either is set).
#if PRISMA_WAVE_TIMES
// diagnostic build only (scripts/wave_times.py): each replica's wave start / end (s_memrealtime,
// 100 MHz) and hardware ids of its last launch
__device__ unsigned long long g_wave_times[4 * 65536];
#define WT_START() const uint64_t wt0_ = __builtin_amdgcn_s_memrealtime()
#define WT_END()                                                                                       \
    do {                                                                                               \
        const uint64_t wt1_ = __builtin_amdgcn_s_memrealtime();                                        \
        if (lane == 0 && r < 65536) {                                                                  \
            g_wave_times[4 * r] = wt0_; g_wave_times[4 * r + 1] = wt1_;                                \
            g_wave_times[4 * r + 2] = (unsigned)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)); \
            g_wave_times[4 * r + 3] = (unsigned)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)); \
        }                                                                                              \
    } while (0)
#else
#define WT_START() do { } while (0)
#define WT_END() do { } while (0)
#endif

template <int FS, int LS, bool MLP, bool TUN, bool CTRL>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(StepOcc<FS, LS>::waves)))
prisma_step_kernel_t(KParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int r = blockIdx.x, lane = threadIdx.x;
    WT_START();
    CLayout& LC = *(CLayout*)P.lay;
    LV lv;
    lv.load(P.lay, lane);
    Regs<FS, LS> R;
    stage_in(lds, P, r, lane, R);
    __syncthreads();
    Sim S;
    sim_bind(S, lv, lds, P.topo, P.log + (size_t)r * LC.log_cap * LC.rec_bytes, LC.replica_base + (uint32_t)r, lane);
    S.tun = TUN;
    S.ctrl = CTRL;
    if (TUN) S.ring = (uint32_t*)(P.state + (size_t)r * LC.state_bytes + LC.s_ring);   // HBM FIFOs
    uint32_t budget = (uint32_t)P.max_hops;
    // (4-wave instances only: at 2 waves per SIMD, config 4's, the same thresholds lost 2 %)
    S.prio_total = StepOcc<FS, LS>::waves >= 4 ? budget : 0u;
    const uint32_t done = event_loop<MLP, StepOcc<FS, LS>::mlp_batch>(P, S, R, r, budget);
    // an episode ended with hop budget left (fused run with auto_reset): the next episode from
    // its prebuilt image, in a second inlined copy of the event loop.  A restart inside the first
    // loop would give its clock and sequence numbers a second incoming value each iteration and
    // cost the hot loop ~20 VGPRs (scripts/asm_headline.sh); this copy runs at most once per
    // launch, after which a second episode end stops the replica as before.
    if (P.spare && done < budget) {
        // the kernel arguments are read again here rather than kept in SGPRs across the first loop
        const KParams* kp = (const KParams*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        const KParams P2 = *kp;
        if (spare_restart(P2, S, R, r, done, budget)) {
            S.prio_base = done;
            event_loop<MLP, StepOcc<FS, LS>::mlp_batch>(P2, S, R, r, budget);
            // stage out from the reloaded arguments too: with P's pointers kept live across this
            // loop the headline instance spilled 7 VGPRs and reloaded them inside it (round 6:
            // 128 VGPRs + 32 B scratch -> 123 VGPRs, no scratch)
            stage_out(lds, P2, r, lane, R);
            WT_END();
            return;
        }
    }
    stage_out(lds, P, r, lane, R);
    WT_END();
}

// instantiations: flow slots FS in {1,2,4,8} (F <= 512), link slots LS in {1,2,4} (L <= 256)
template <int FS, int LS, bool CTRL, bool MLP> const void* step_kernel(bool tun) {
    return tun ? (const void*)prisma_step_kernel_t<FS, LS, MLP, true, CTRL>
               : (const void*)prisma_step_kernel_t<FS, LS, MLP, false, CTRL>;
}

// tun: tunnelled-overlay instance (identity overlays run code without the tunnel paths).
// One translation unit per (CTRL, MLP) instance set, so the four sets compile in parallel:
// prisma_engine.hip (CTRL, tables), prisma_engine_mlp.hip (CTRL, MLP), prisma_engine_lite.hip
// and prisma_engine_lite_mlp.hip (without the ctrl paths)
template <bool CTRL, bool MLP>
static const void* pick_step(int fs, int ls, bool tun) {
#ifdef PRISMA_DEV_HEADLINE
    // register-allocation experiments only: compile the headline instance alone
    return (!CTRL && !MLP && fs == 2 && ls == 1 && !tun) ? (const void*)prisma_step_kernel_t<2, 1, false, false, false>
                                                         : nullptr;
#else
#define PK(F_, L_) if (fs == F_ && ls == L_) return step_kernel<F_, L_, CTRL, MLP>(tun);
    PK(1, 1) PK(1, 2) PK(1, 4) PK(2, 1) PK(2, 2) PK(2, 4) PK(4, 1) PK(4, 2) PK(4, 4) PK(8, 1) PK(8, 2) PK(8, 4)
#undef PK
    return nullptr;
#endif
}

#if PRISMA_WAVE_TIMES
#define PRISMA_TU_WAVE_TIMES(NAME)                                                                      \
    extern "C" int NAME(unsigned long long* out, int n) {                                               \
        return (hipDeviceSynchronize() == hipSuccess &&                                                 \
                hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_times), 4 * sizeof(unsigned long long) * n) == hipSuccess) ? 0 : -1; \
    }
#else
#define PRISMA_TU_WAVE_TIMES(NAME)
#endif

#if PRISMA_TIMING
// diagnostic build only: read and clear this translation unit's per-phase cycle totals
// (g_prisma_timing is one copy per translation unit; scripts/timing.py)
#define PRISMA_TU_TIMING(NAME)                                                                          \
    extern "C" int NAME(unsigned long long* out32) {                                                    \
        if (hipDeviceSynchronize() != hipSuccess ||                                                     \
            hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_prisma_timing), kTimingWords * sizeof(unsigned long long)) != \
                hipSuccess) return -1;                                                                  \
        unsigned long long z[kTimingWords] = {0};                                                                 \
        return hipMemcpyToSymbol(HIP_SYMBOL(g_prisma_timing), z, sizeof(z)) == hipSuccess ? 0 : -1;     \
    }
#else
#define PRISMA_TU_TIMING(NAME)
#endif
