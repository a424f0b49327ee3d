// engine_core.h — device code shared by the two gfx950 engines:
//   * the register-resident engine (prisma_engine.hip): link / flow / ping state
//     lane-distributed in VGPRs (Regs<FS, LS>), FIFOs and wires in LDS -- topologies
//     up to 255 nodes, 256 links and 512 flows;
//   * the memory-resident engine (prisma_engine_mem.hip): the same state as
//     128-byte link records and a 64-ary tournament tree of event keys in HBM
//     (MemSt), for large irregular topologies (ER-256: 2 304 links, 65 280 flows).
// The event handlers below are written once, templated on the store (RS), and
// compiled into both; only the store primitives (link_get / link_put, flow keys,
// ping state, the observation, event selection, init and staging) differ.
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/prisma.h"
#include "engine_layout.h"
#include "numerics.h"
#include "mrg32k3a.h"

using namespace prisma;

#define HIP_OK(x) ((x) == hipSuccess)

// Diagnostic timing builds only (scripts/ablate.sh; results are NOT the
// reference's): bit 0 skips the previous-record read (relay entries carry
// dst/start), bit 1 skips the decision-record stores, bit 2 skips observe(), bit 3 draws from a
// cheap hash instead of Philox, bit 4 takes a float log, bit 5 drops the reward's microsecond
// formatting, bit 6 replaces the ping statistic by queued bytes (profiles/r06_ab/).
#ifndef PRISMA_ABLATE
#define PRISMA_ABLATE 0
#endif
#ifndef PRISMA_REWARD_LANES
#define PRISMA_REWARD_LANES 1
#endif


// instruction-count experiments (A/B builds)

// Diagnostic timing build (-DPRISMA_TIMING=1, scripts/timing.py): s_memtime
// cycle totals per loop phase, summed over waves into g_prisma_timing.
#ifndef PRISMA_TIMING
#define PRISMA_TIMING 0
#endif
// Diagnostic event-trace build (-DPRISMA_TRACE=1, scripts/diag_trace.py): lane 0 of
// replicas 0-7 appends (time, kind, id) of every executed event to a device buffer.
#ifndef PRISMA_TRACE
#define PRISMA_TRACE 0
#endif
#if PRISMA_TRACE
static __device__ long long* g_prisma_trace;      // [8][cap][3]
static __device__ unsigned int g_prisma_trace_cap;
static __device__ unsigned int g_prisma_trace_n[8];
#endif
#if PRISMA_TIMING
// one copy per engine (translation unit): 0-7 loop phases, 8-15 their counts, 16-19 mlp_action
// phases, 20-23 memory-resident on_flow phases, 24-39 fine probes TP(i), 40-55 their counts
constexpr int kTimingWords = 64;
static __device__ unsigned long long g_prisma_timing[kTimingWords];
#define TM_NOW() ((uint64_t)__builtin_amdgcn_s_memtime())
#define TM_FLOW(i) do { const uint64_t t_ = TM_NOW(); S.tflow[i] += t_ - S.tfl; S.tfl = t_; } while (0)
// fine probes: cycles since the previous probe (or TP_START) into slot i, scheduling fenced
#define TP_START() do { __builtin_amdgcn_sched_barrier(0); S.tpl = TM_NOW(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define TP(i) do { __builtin_amdgcn_sched_barrier(0); const uint64_t t_ = TM_NOW(); S.tp[i] += t_ - S.tpl; S.tpn[i]++; \
                   S.tpl = t_; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define TM_FLOW(i) do { } while (0)
#define TP_START() do { } while (0)
#define TP(i) do { } while (0)
#endif
// probe sets (timing build, -DPRISMA_TP_SET): 0 the decision (mlp_action, apply_decision), 1 the
// memory-resident arrival / completion / flow handlers, 2 the register-resident ones
#ifndef PRISMA_TP_SET
#define PRISMA_TP_SET 0
#endif
#if PRISMA_TP_SET == 0
#define TP0(i) TP(i)
#else
#define TP0(i) do { } while (0)
#endif
#if PRISMA_TP_SET == 1
#define TP1(i) TP(i)
#define TP1_START() TP_START()
#else
#define TP1(i) do { } while (0)
#define TP1_START() do { } while (0)
#endif
#if PRISMA_TP_SET == 2
#define TP2(i) do { if (!S.mem) TP(i); } while (0)
#define TP2_START() do { if (!S.mem) TP_START(); } while (0)
#else
#define TP2(i) do { } while (0)
#define TP2_START() do { } while (0)
#endif

// ---------------------------------------------------------------------------
// kernel parameters
// ---------------------------------------------------------------------------
struct KParams {
    const Layout* __restrict__ lay;  // device copy (read through the scalar cache)
    unsigned char* state;        // [R][state_bytes]
    const unsigned char* topo;   // [topo_bytes]
    unsigned char* log;          // [R][log_cap][rec_bytes]
    prisma_counters_t* cnt_out;  // [R]
    const int32_t* actions;      // [R] or null
    int32_t* obs_out;            // [R][W] or null
    uint8_t* mask_out;           // [R] or null
    int32_t* node_out;           // [R] or null
    const uint8_t* table;        // [N][N] or null
    const float* mlp;            // packed DQN-buffer weights or null (mode 4)
    const float* mlp_rp;         // layers 2-4 of `mlp` interleaved by 4 inputs (mlp_repack), mode 4
    int32_t R;
    int32_t max_hops;
    uint32_t episode;            // reset kernel only
    int32_t mode;                // 0 reset, 1 external step, 2 table run, 3 auto-reset, 4 MLP run
    unsigned char* spare;        // [R][state_bytes] next-episode images (register engine with
                                 // auto_reset), or null
    const uint32_t* rng;         // ns-3 stream mode: the rng table (engine_layout.h kMrgPowers), or null
};

// ---------------------------------------------------------------------------
// cross-lane helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}
// write one lane of a VGPR (v_cmp + v_cndmask; there is no writelane builtin)
__device__ __forceinline__ uint32_t wrl(uint32_t old, uint32_t v, uint32_t lane) {
    return threadIdx.x == lane ? v : old;
}
// lane `src` of v (a wave-wide ds_bpermute; src < 64, no lane-id arithmetic as in __shfl)
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
__device__ __forceinline__ int64_t mk64(uint32_t lo, uint32_t hi) { return (int64_t)(((uint64_t)hi << 32) | lo); }
__device__ __forceinline__ uint32_t lo32(int64_t v) { return (uint32_t)(uint64_t)v; }
__device__ __forceinline__ uint32_t hi32(int64_t v) { return (uint32_t)((uint64_t)v >> 32); }

// A lane-distributed u32 array of 64*S elements: element i lives in lane
// i % 64, register slot i / 64.  get/set take a wave-uniform index.
template <int S>
struct LA {
    uint32_t v[S];
    // Every slot is read / compared unconditionally so the slot index never
    // becomes a dynamic array index (which would demote v[] to scratch).
    __device__ __forceinline__ uint32_t get(uint32_t i) const {
        const uint32_t slot = i >> 6, owner = i & 63u;
        uint32_t r = rdl(v[0], owner);
#pragma unroll
        for (int j = 1; j < S; ++j) {
            const uint32_t t = rdl(v[j], owner);
            r = (slot == (uint32_t)j) ? t : r;
        }
        return r;
    }
    __device__ __forceinline__ void set(uint32_t i, uint32_t x) {
#pragma unroll
        for (int j = 0; j < S; ++j)
            v[j] = (threadIdx.x + 64u * (uint32_t)j == i) ? x : v[j];
    }
    __device__ __forceinline__ void load(const uint32_t* img, int lane) {
#pragma unroll
        for (int j = 0; j < S; ++j) v[j] = img[lane + 64 * j];
    }
    __device__ __forceinline__ void store(uint32_t* img, int lane) const {
#pragma unroll
        for (int j = 0; j < S; ++j) img[lane + 64 * j] = v[j];
    }
};

// Per-episode counters live in the LDS image and are bumped by lane 0 with
// no-return LDS atomics (ds_add_u32/u64/f32/f64): fire-and-forget, in order
// per wave, and bit-identical to sequential IEEE adds on gfx950 (checked by
// scripts/ubench/lds_fadd.hip) -- no read-modify-write to wait on, no VGPRs.
template <class T>
__device__ __forceinline__ void lds_add(T* p, T v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
#define CNT_ADD(S_, field_, v_) \
    do { if ((S_).lane == 0) lds_add(&(S_).c->field_, (decltype((S_).c->field_))(v_)); } while (0)

// register-resident replica state (image order: the fields below, each a
// [64*S] u32 array)
template <int FS, int LS>
struct Regs {
    LA<FS> fk_lo, fk_hi, fk_seq, f_draw;         // flow next event (time, seq) + draw index
    // link times are kept as their low 32 bits: every pending link event is
    // less than 2^31 ns ahead of the clock (checked on the host), so
    // t = now + (uint32)(t_lo - lo32(now)); select_event derives each link's candidate event
    LA<LS> cp_t, cp_seq;                         // tx completion event (valid while busy)
    LA<LS> wh_t, wh_seq;                         // arrival event of the wire head (valid while n_wire > 0)
    LA<LS> p0, p1, p2, qb;                       // head|txp<<16, tail|n_wire<<16, n_queue|busy<<16, queued bytes
    // per TUNNEL t (lane t % 64, slot t / 64; tunnel == link on identity overlays):
    LA<LS> pm_lo, pm_mlo, pm_mhi;                // ping: oldest unacked round, acked bits of rounds lo+1..lo+64
    LA<LS> pm_win;                               // win_n | win_head << 16 | saturated << 31
    LA<LS> pav_lo, pav_hi;                       // ping window mean (double), refreshed per ping-back
    LA<LS> od_lo, od_hi;                         // send time (s) of round lo
    static constexpr int NF = 4, NL = 16;
    static constexpr bool kLazy = true;          // empty-queue transmit completions elided (lazy_resolve)
    static constexpr bool kMem = false;
    // the draw cache's code (flow_next) in the instances of up to 128 flows: larger scenarios
    // have no LDS room for it (GEANT's 506 flows: 4 KB at 8 replicas per CU), and its code cost
    // their register allocation 1.3 % (config 4)
    static constexpr bool kDcache = FS <= 2;
    // not staged: each lane's earliest flow (time, seq, code), refreshed when one of its flows
    // changes (flow_set, ~0.3 per hop) instead of on every event selection (~2.6 per hop)
    int64_t fm_t;
    uint32_t fm_s, fm_c;
};

template <int FS, int LS>
__device__ __forceinline__ void regs_io(Regs<FS, LS>& R, uint32_t* img, int lane, bool store) {
    uint32_t* fb = img;
    uint32_t* lb = img + 4 * 64 * FS;
#define RIO_F(fld, a) if (store) R.fld.store(fb + (a) * 64 * FS, lane); else R.fld.load(fb + (a) * 64 * FS, lane);
#define RIO_L(fld, a) if (store) R.fld.store(lb + (a) * 64 * LS, lane); else R.fld.load(lb + (a) * 64 * LS, lane);
    RIO_F(fk_lo, 0) RIO_F(fk_hi, 1) RIO_F(fk_seq, 2) RIO_F(f_draw, 3)
    RIO_L(wh_t, 0) RIO_L(cp_t, 1) RIO_L(wh_seq, 2)
    RIO_L(cp_seq, 3) RIO_L(p0, 4) RIO_L(p1, 5) RIO_L(p2, 6) RIO_L(qb, 7) RIO_L(pm_lo, 8)
    RIO_L(pm_mlo, 9) RIO_L(pm_mhi, 10) RIO_L(pm_win, 11) RIO_L(pav_lo, 12) RIO_L(pav_hi, 13)
    RIO_L(od_lo, 14) RIO_L(od_hi, 15)
#undef RIO_F
#undef RIO_L
}

// wave-uniform scalar state ("SGPR state"): clock, counters, event sources
struct Hot {
    int64_t  now, ping_t;
    uint32_t ping_seq, seq, uid, dec, ping_rounds, episode;
    uint32_t pend, over, error, stop, hops_launch;
    uint32_t ev_launch;          // events executed in this launch (the running
                                 // totals stay in the LDS header until exit)
    uint32_t cur_seq;            // seq of the event being executed (0 at launch start)
};


// Read-only topology in HBM through the constant address space: every index
// is wave-uniform, so these become s_load through the scalar cache.
#define CAS __attribute__((address_space(4)))
typedef const CAS int32_t c_i32;
typedef const CAS uint32_t c_u32;
typedef const CAS int64_t c_i64;
typedef const CAS double c_f64;
typedef const CAS Layout CLayout;        // scenario constants: s_load, never clobbered

// Scenario constants in one VGPR: lane i holds dword i of the Layout, read
// with v_readlane (25-cycle dependent latency on gfx950, measured by
// scripts/ubench/latency.hip) instead of s_load through the scalar cache
// (60 cycles) -- the compiler re-issued those loads inside the event loop
// because the constants do not fit in SGPRs next to the replica state.
static_assert(offsetof(Layout, mem) == 4 * kLVWords && kLVWords == kWave, "LV covers the first 64 dwords");
struct LV {
    uint32_t w;
    __device__ __forceinline__ void load(const Layout* lay, int lane) {
        w = ((const uint32_t*)lay)[lane];
    }
    __device__ __forceinline__ uint32_t u(int i) const { return (uint32_t)__builtin_amdgcn_readlane((int)w, i); }
    __device__ __forceinline__ int32_t N() const { return (int32_t)u(offsetof(Layout, N) / 4); }
    __device__ __forceinline__ int32_t E() const { return (int32_t)u(offsetof(Layout, E) / 4); }
    __device__ __forceinline__ int32_t L() const { return (int32_t)u(offsetof(Layout, L) / 4); }
    __device__ __forceinline__ int32_t F() const { return (int32_t)u(offsetof(Layout, F) / 4); }
    __device__ __forceinline__ int32_t W() const { return (int32_t)u(offsetof(Layout, W) / 4); }
    __device__ __forceinline__ int32_t max_deg() const { return (int32_t)u(offsetof(Layout, max_deg) / 4); }
    __device__ __forceinline__ int32_t WCAP() const { return (int32_t)u(offsetof(Layout, WCAP) / 4); }
    __device__ __forceinline__ int32_t MA() const { return (int32_t)u(offsetof(Layout, MA) / 4); }
    __device__ __forceinline__ uint32_t topo_bytes() const { return (uint32_t)u(offsetof(Layout, topo_bytes) / 4); }
    __device__ __forceinline__ uint32_t state_bytes() const { return (uint32_t)u(offsetof(Layout, state_bytes) / 4); }
    __device__ __forceinline__ uint32_t lds_bytes() const { return (uint32_t)u(offsetof(Layout, lds_bytes) / 4); }
    __device__ __forceinline__ uint32_t s_dcache() const { return (uint32_t)u(offsetof(Layout, s_dcache) / 4); }
    __device__ __forceinline__ uint32_t s_hdr() const { return (uint32_t)u(offsetof(Layout, s_hdr) / 4); }
    __device__ __forceinline__ uint32_t s_cnt() const { return (uint32_t)u(offsetof(Layout, s_cnt) / 4); }
    __device__ __forceinline__ uint32_t s_obs() const { return (uint32_t)u(offsetof(Layout, s_obs) / 4); }
    __device__ __forceinline__ uint32_t s_wt() const { return (uint32_t)u(offsetof(Layout, s_wt) / 4); }
    __device__ __forceinline__ uint32_t s_wseq() const { return (uint32_t)u(offsetof(Layout, s_wseq) / 4); }
    __device__ __forceinline__ uint32_t s_ring() const { return (uint32_t)u(offsetof(Layout, s_ring) / 4); }
    __device__ __forceinline__ uint32_t s_win() const { return (uint32_t)u(offsetof(Layout, s_win) / 4); }
    __device__ __forceinline__ uint32_t s_pbd() const { return (uint32_t)u(offsetof(Layout, s_pbd) / 4); }
    __device__ __forceinline__ uint32_t s_mlp() const { return (uint32_t)u(offsetof(Layout, s_mlp) / 4); }
    __device__ __forceinline__ int32_t T() const { return (int32_t)u(offsetof(Layout, T) / 4); }
    __device__ __forceinline__ int32_t NO() const { return (int32_t)u(offsetof(Layout, NO) / 4); }
    __device__ __forceinline__ uint32_t tunnels() const { return (uint32_t)u(offsetof(Layout, tunnels) / 4); }
    __device__ __forceinline__ uint32_t PLEN() const { return (uint32_t)u(offsetof(Layout, PLEN) / 4); }
    __device__ __forceinline__ uint32_t ring_total() const { return (uint32_t)u(offsetof(Layout, ring_total) / 4); }
    __device__ __forceinline__ uint32_t lds_state_bytes() const { return (uint32_t)u(offsetof(Layout, lds_state_bytes) / 4); }
    __device__ __forceinline__ uint32_t s_regs() const { return (uint32_t)u(offsetof(Layout, s_regs) / 4); }
    __device__ __forceinline__ uint32_t PBK() const { return (uint32_t)u(offsetof(Layout, PBK) / 4); }
    __device__ __forceinline__ int32_t FS() const { return (int32_t)u(offsetof(Layout, FS) / 4); }
    __device__ __forceinline__ int32_t LS() const { return (int32_t)u(offsetof(Layout, LS) / 4); }
    __device__ __forceinline__ int64_t sw_txd() const { return mk64(u(offsetof(Layout, sw_txd) / 4), u(offsetof(Layout, sw_txd) / 4 + 1)); }
    __device__ __forceinline__ int64_t sw_txp() const { return mk64(u(offsetof(Layout, sw_txp) / 4), u(offsetof(Layout, sw_txp) / 4 + 1)); }
    __device__ __forceinline__ int64_t sw_txe() const { return mk64(u(offsetof(Layout, sw_txe) / 4), u(offsetof(Layout, sw_txe) / 4 + 1)); }
    __device__ __forceinline__ int64_t sw_prop() const { return mk64(u(offsetof(Layout, sw_prop) / 4), u(offsetof(Layout, sw_prop) / 4 + 1)); }
    __device__ __forceinline__ uint32_t qcap_s() const { return (uint32_t)u(offsetof(Layout, qcap_s) / 4); }
    __device__ __forceinline__ uint32_t qcap_a() const { return (uint32_t)u(offsetof(Layout, qcap_a) / 4); }
    __device__ __forceinline__ uint32_t qmax_bytes() const { return (uint32_t)u(offsetof(Layout, qmax_bytes) / 4); }
    __device__ __forceinline__ uint32_t acc_qmax_pkts() const { return (uint32_t)u(offsetof(Layout, acc_qmax_pkts) / 4); }
    __device__ __forceinline__ int64_t t_end() const { return mk64(u(offsetof(Layout, t_end) / 4), u(offsetof(Layout, t_end) / 4 + 1)); }
    __device__ __forceinline__ int64_t ping_period() const { return mk64(u(offsetof(Layout, ping_period) / 4), u(offsetof(Layout, ping_period) / 4 + 1)); }
    __device__ __forceinline__ uint32_t data_size() const { return (uint32_t)u(offsetof(Layout, data_size) / 4); }
    __device__ __forceinline__ uint32_t ping_size() const { return (uint32_t)u(offsetof(Layout, ping_size) / 4); }
    __device__ __forceinline__ uint32_t echo_size() const { return (uint32_t)u(offsetof(Layout, echo_size) / 4); }
    __device__ __forceinline__ uint32_t ma() const { return (uint32_t)u(offsetof(Layout, ma) / 4); }
    __device__ __forceinline__ uint32_t ping_as_obs() const { return (uint32_t)u(offsetof(Layout, ping_as_obs) / 4); }
    __device__ __forceinline__ uint32_t auto_reset() const { return (uint32_t)u(offsetof(Layout, auto_reset) / 4); }
    __device__ __forceinline__ uint32_t notify_dest() const { return (uint32_t)u(offsetof(Layout, notify_dest) / 4); }
    __device__ __forceinline__ uint32_t train() const { return (uint32_t)u(offsetof(Layout, train) / 4); }
    __device__ __forceinline__ uint32_t seed_lo() const { return (uint32_t)u(offsetof(Layout, seed_lo) / 4); }
    __device__ __forceinline__ uint32_t replica_base() const { return (uint32_t)u(offsetof(Layout, replica_base) / 4); }
    __device__ __forceinline__ uint32_t log_cap() const { return (uint32_t)u(offsetof(Layout, log_cap) / 4); }
    __device__ __forceinline__ uint32_t rec_bytes() const { return (uint32_t)u(offsetof(Layout, rec_bytes) / 4); }
    __device__ __forceinline__ double loss_penalty() const { return __longlong_as_double(mk64(u(offsetof(Layout, loss_penalty) / 4), u(offsetof(Layout, loss_penalty) / 4 + 1))); }
    __device__ __forceinline__ float loss_penalty_f() const { return __uint_as_float(u(offsetof(Layout, loss_penalty_f) / 4)); }
    __device__ __forceinline__ uint32_t rng_mode() const { return (uint32_t)u(offsetof(Layout, rng_mode) / 4); }
};


// LDS views of one replica + its topology
struct Sim {
    LV lv;                                  // scenario constants (one VGPR)
    unsigned char* base;
    Hdr* h;
    prisma_counters_t* c;
    uint32_t* obs;
    uint32_t* wt; uint32_t* wseq;           // wire: arrival time (low 32 bits) and seq
    uint32_t* went;                         // tunnelled overlays: wire packet entries (LDS)
    uint32_t* qwin;                         // ... and the FIFO windows of relay_ip kernels (LDS, q_put)
    uint32_t* ring;                         // link FIFOs: LDS, or HBM (tunnelled / memory-resident)
    float* win;
    float* pbd;                             // ping-back delays [responder slot][PBK]
    const CAS TopoImage* T;                 // topology (scalar loads at fixed offsets)
    const uint8_t* table;                   // action table in LDS (register engine, table_in_lds)
    const uint8_t* table_g;                 // ... or in HBM (memory-resident engine, or not in LDS)
    bool tab_lds;
    const float* mlp;                       // DQN-buffer weights (HBM) or null
    const float* mlp_rp;                    // layers 2-4 interleaved by 4 inputs (mlp_repack)
    float* hbuf;                            // 64 floats of LDS: a layer's activations
    unsigned char* logrep;
    uint32_t gid;
    int lane;
    uint32_t m1, m2, m4, m8;                // per-lane word masks -(lane & 1), -(lane>>1 & 1), -(lane>>2 & 1), -(lane < 8)
    bool tun;                               // tunnelled overlay: a compile-time constant in the
                                            // step kernels (template TUN), folded after inlining
    bool mem;                               // memory-resident engine (compile-time constant, folded)
    bool ctrl;                              // --train echo / notify_dest paths compiled in (constant)
    bool mlp_inst;                          // an in-kernel MLP instance (event_loop's MLP, constant)
    // memory-resident engine: variable-size topology arrays (scalar loads)
    const CAS int32_t* m_rowptr;
    const CAS int32_t* m_ldst;
    const CAS int32_t* m_lrev;
    const CAS int64_t* m_acctx;
    const CAS int32_t* m_fsrc;
    const CAS int32_t* m_fdst;
    const CAS double* m_fmean;
    const CAS uint32_t* m_esz;              // ... and the signalling arrays of the --train instances
    const CAS uint32_t* m_etx;
    const CAS uint32_t* m_abtx;
    const CAS uint32_t* m_bpair;
    const CAS uint32_t* m_fseq;
    const CAS BigSig* m_bs;
    uint32_t* lrec;                         // link records [L][kLRec] (HBM)
    // issue priority by launch progress (prio_update): hops of the whole launch (0: off), hops done
    // before this event loop, and the loop's hop count at which the priority next drops
    uint32_t prio_total, prio_base, prio_next;
#if PRISMA_TIMING
    mutable uint64_t tsub[2], tlast;             // sub-phase cycles inside apply_decision
    mutable uint64_t tmlp[4];                    // mlp_action phases (timing build)
    mutable uint64_t tflow[4], tfl;              // memory-resident on_flow phases (timing build)
    mutable uint64_t tp[16], tpl;                // fine probes TP(i) (timing build)
    mutable uint32_t tpn[16];
#endif
};

__device__ inline void sim_bind(Sim& S, const LV& L, unsigned char* lds, const unsigned char* topo,
                                unsigned char* logrep, uint32_t gid, int lane) {
    S.lv = L;
    S.base = lds;
    S.h = (Hdr*)(lds + kOffHdr);                // fixed offsets (asserted in build_layout)
    S.c = (prisma_counters_t*)(lds + kOffCnt);
    S.obs = (uint32_t*)(lds + kOffObs);
    S.wt = (uint32_t*)(lds + L.s_wt());
    S.wseq = (uint32_t*)(lds + L.s_wseq());
    S.went = S.wseq + (uint32_t)L.L() * (uint32_t)L.WCAP();
    S.qwin = S.went + (uint32_t)L.L() * (uint32_t)L.WCAP();
    S.ring = (uint32_t*)(lds + L.s_ring());
    S.win = (float*)(lds + L.s_win());
    S.pbd = (float*)(lds + L.s_pbd());
    S.T = (const CAS TopoImage*)topo;
    S.table = (const uint8_t*)(lds + L.lds_state_bytes());
    S.table_g = nullptr;
    S.tab_lds = true;
    S.hbuf = (float*)(lds + L.s_mlp());
    S.mlp = nullptr;
    S.mlp_rp = nullptr;
    S.logrep = logrep;
    S.gid = gid;
    S.lane = lane;
    // opaque to the optimiser, so write_record's selects stay bitfield inserts on VGPR masks
    // instead of loop-invariant lane-compare SGPR pairs (which the headline kernel spilled)
    S.m1 = 0u - ((uint32_t)lane & 1u);
    S.m2 = 0u - (((uint32_t)lane >> 1) & 1u);
    S.m4 = 0u - (((uint32_t)lane >> 2) & 1u);
    S.m8 = lane < 8 ? ~0u : 0u;
    asm volatile("" : "+v"(S.m1), "+v"(S.m2), "+v"(S.m4), "+v"(S.m8));
    S.tun = L.tunnels() != 0u;
    S.mem = false;
    S.ctrl = true;
    S.mlp_inst = false;
    S.lrec = nullptr;
    S.prio_total = 0; S.prio_base = 0; S.prio_next = 0xffffffffu;
}

// Issue priority by launch progress.  A SIMD arbitrates its waves' issue by priority, then age
// (MI355X_MICROARCH.md, two waves per SIMD), so at equal priority the oldest of a SIMD's 4
// replicas runs ahead and the youngest finishes alone: measured on the headline
// (scripts/wave_times.py), the 4 waves of a SIMD ended at about 89, 113, 124 and 146 ms of a
// 146-ms launch, the last ~22 ms with one wave left to hide its own latency.  Here a wave's priority
// drops as its share of the launch's hops is done (3 below 5/8, 2 below 13/16, 1 below 15/16, then 0),
// so a wave that is ahead yields issue to the ones behind it and the SIMD keeps all four to the end.
#ifndef PRISMA_PRIO
#define PRISMA_PRIO 1
#endif
// (round-6 A/B on one box, profiles/r06_ab/ab_prio.txt: thresholds 5/8, 13/16, 15/16 +13.4 % at
// the headline and +8.9 % at config 3; 1/2, 3/4, 7/8 (PRISMA_PRIO=2) +13.2 %; 1/4, 1/2, 3/4 +10 %;
// 7/8, 15/16, 31/32 +4.5 %; a least-progress-first rank over the SIMD's four waves, exchanged
// through global memory every 64 or 256 hops, -2 %)
__device__ __forceinline__ void prio_update(Sim& S, uint32_t hops_loop) {
    const uint32_t T = S.prio_total, p = S.prio_base + hops_loop;
    uint32_t t1, t2, t3;
    if (PRISMA_PRIO == 2) { t1 = T / 2; t2 = T - T / 4; t3 = T - T / 8; }
    else { t1 = T / 2 + T / 8; t2 = T - T / 8 - T / 16; t3 = T - T / 16; }
    uint32_t next;
    if (p < t1) { __builtin_amdgcn_s_setprio(3); next = t1; }
    else if (p < t2) { __builtin_amdgcn_s_setprio(2); next = t2; }
    else if (p < t3) { __builtin_amdgcn_s_setprio(1); next = t3; }
    else { __builtin_amdgcn_s_setprio(0); next = 0xffffffffu; }
    S.prio_next = next == 0xffffffffu ? next : next - S.prio_base;
}

// Topology reads.  The register-resident engine reads the fixed-offset TopoImage,
// the memory-resident one its variable-size arrays; S.mem is a compile-time
// constant in every kernel, so each accessor folds to one scalar load.
__device__ __forceinline__ int32_t t_ovrow(const Sim& S, uint32_t u) { return S.mem ? S.m_rowptr[u] : S.T->ovrow[u]; }
__device__ __forceinline__ int32_t t_ldst(const Sim& S, uint32_t l) { return S.mem ? S.m_ldst[l] : S.T->ldst[l]; }
__device__ __forceinline__ int32_t t_lrev(const Sim& S, uint32_t l) { return S.mem ? S.m_lrev[l] : S.T->lrev[l]; }
__device__ __forceinline__ int64_t t_acctx(const Sim& S, uint32_t u) { return S.mem ? S.m_acctx[u] : S.T->acctx[u]; }
__device__ __forceinline__ int32_t t_fsrc(const Sim& S, uint32_t f) { return S.mem ? S.m_fsrc[f] : S.T->fsrc[f]; }
__device__ __forceinline__ int32_t t_fdst(const Sim& S, uint32_t f) { return S.mem ? S.m_fdst[f] : S.T->fdst[f]; }
__device__ __forceinline__ double t_fmean(const Sim& S, uint32_t f) { return S.mem ? S.m_fmean[f] : S.T->fmean[f]; }
__device__ __forceinline__ uint32_t t_esz(const Sim& S, uint32_t l) { return S.mem ? S.m_esz[l] : S.T->esz[l]; }
__device__ __forceinline__ uint32_t t_etx(const Sim& S, uint32_t l) { return S.mem ? S.m_etx[l] : S.T->etx[l]; }
__device__ __forceinline__ uint32_t t_abtx(const Sim& S, uint32_t u) { return S.mem ? S.m_abtx[u] : S.T->abtx[u]; }
__device__ __forceinline__ uint32_t t_bpair(const Sim& S, uint32_t g) { return S.mem ? S.m_bpair[g] : S.T->bpair[g]; }
__device__ __forceinline__ uint32_t t_fseq(const Sim& S, uint32_t f) { return S.mem ? S.m_fseq[f] : S.T->fseq[f]; }
__device__ __forceinline__ uint32_t t_ngen(const Sim& S) { return S.mem ? S.m_bs->n_gen : S.T->n_bsig; }
__device__ __forceinline__ uint32_t t_bs_nseg(const Sim& S) { return S.mem ? S.m_bs->nseg : S.T->bs_nseg; }
__device__ __forceinline__ uint32_t t_bs_size(const Sim& S) { return S.mem ? S.m_bs->size : S.T->bs_size; }
__device__ __forceinline__ int64_t t_bs_period(const Sim& S) { return S.mem ? S.m_bs->period : S.T->bs_period; }

// A store to replica state that every lane may read back, by every lane (same address, same
// value): no exec-mask juggling in LDS, and in HBM each lane's later read of the address is
// ordered after its own store.
template <class T>
__device__ __forceinline__ void st_rep(const Sim& S, T* p, T v) {
    *p = v;
}

// A FIFO entry, written by every lane (same address, same value).  Identity overlays of the
// register-resident engine keep the rings in LDS, where an all-lane store needs no exec-mask
// juggling (A/B +1 % against lane 0 only); tunnelled overlays and the memory-resident engine
// keep them in the HBM state image (their arrivals read the packet from the wire slot, so only
// a dequeue behind a busy transmitter reads the ring back).
__device__ __forceinline__ void ring_put(const Sim& S, uint32_t i, uint32_t e) {
    S.ring[i] = e;
}

// Relay entries carry (decision, live TTL, tunnel target) -- rip_make, engine_layout.h -- in the
// register-resident engine's tunnelled-overlay kernels without the --train / notify_dest paths
// (a compile-time constant): a switch inside a tunnel forwards a data packet on its entry alone,
// as IpForward does on the IP header (ipv4-l3-protocol.cc IpForward), instead of reading the
// deciding node, action and TTL back from the decision record in HBM.
__device__ __forceinline__ bool relay_ip(const Sim& S) { return S.tun && !S.mem && !S.ctrl; }

// The same kernels keep the first kQWin packets queued behind each link's busy transmitter -- the
// ones its next completions dequeue -- in an LDS window, slot = ring index mod kQWin, stored
// complemented (0 = empty; none of these kernels' entries is all ones); a packet with kQWin or
// more queued ahead of it goes to the HBM ring.  A dequeue finds the queue head in its window slot
// iff it was stored there: any later packet for that slot would have had kQWin packets ahead of it
// (ring capacities are multiples of kQWin, so indices stay consecutive across the wrap).  Their
// FIFOs had read every dequeued packet back from HBM, most of the time after the line had left L2.
__device__ __forceinline__ void q_put(const Sim& S, uint32_t l, uint32_t off, uint32_t idx, uint32_t ahead,
                                      uint32_t e) {
    if (relay_ip(S) && ahead < kQWin) S.qwin[l * kQWin + (idx & (kQWin - 1u))] = ~e;
    else ring_put(S, off + idx, e);
}
__device__ __forceinline__ uint32_t q_take(const Sim& S, uint32_t l, uint32_t off, uint32_t idx) {
    if (relay_ip(S)) {
        uint32_t* w = &S.qwin[l * kQWin + (idx & (kQWin - 1u))];
        const uint32_t v = rfl(*w);
        if (v != 0u) { *w = 0u; return ~v; }
    }
    return rfl(S.ring[off + idx]);
}

// uniform LDS reads (every lane reads the same address: broadcast, no conflict)
__device__ __forceinline__ uint32_t u_ld32(const uint32_t* p) { return rfl(*p); }
__device__ __forceinline__ int32_t u_ldi(const int32_t* p) { return (int32_t)rfl((uint32_t)*p); }
__device__ __forceinline__ int64_t u_ld64(const int64_t* p) {
    int64_t v = *p;
    return mk64(rfl(lo32(v)), rfl(hi32(v)));
}
__device__ __forceinline__ double u_ldd(const double* p) {
    double v = *p;
    uint64_t b = __double_as_longlong(v);
    return __longlong_as_double((long long)(((uint64_t)rfl((uint32_t)(b >> 32)) << 32) | rfl((uint32_t)b)));
}

__device__ inline void hot_load(const Sim& S, Hot& H) {
    const Hdr& h = *S.h;
    H.now = u_ld64(&h.now); H.ping_t = u_ld64(&h.ping_t);
    H.ping_seq = u_ld32(&h.ping_seq); H.seq = u_ld32(&h.seq); H.uid = u_ld32(&h.uid);
    H.dec = u_ld32(&h.dec_count); H.ping_rounds = u_ld32(&h.ping_rounds); H.episode = u_ld32(&h.episode);
    H.pend = u_ld32(&h.pend); H.over = u_ld32(&h.over); H.error = u_ld32(&h.error);
    H.stop = u_ld32(&h.stop); H.hops_launch = u_ld32(&h.hops_launch);
    H.ev_launch = 0;
    H.cur_seq = 0;
}

template <class RS>
__device__ inline void hot_store(Sim& S, const RS& R, const Hot& H) {
    if (S.lane == 0) {
        Hdr& h = *S.h;
        h.now = H.now; h.ping_t = H.ping_t; h.ping_seq = H.ping_seq; h.seq = H.seq; h.uid = H.uid;
        h.dec_count = H.dec; h.ping_rounds = H.ping_rounds; h.episode = H.episode; h.pend = H.pend;
        h.over = H.over; h.error = H.error; h.stop = H.stop; h.hops_launch = H.hops_launch;
        h.hops_total += H.hops_launch; h.events_total += H.ev_launch;
        prisma_counters_t& c = *S.c;
        c.now_ns = H.now; c.episode = H.episode; c.ping_rounds = H.ping_rounds; c.seq = H.seq; c.uid = H.uid;
        c.dec_count = H.dec; c.error = H.error; c.episode_over = H.over;
        c.hops_total = h.hops_total; c.events_total = h.events_total;
        c.events += H.ev_launch;
    }
}

__device__ __forceinline__ void fail(Hot& H, uint32_t bit) {
    H.error |= bit;
    H.over = 1;
    H.stop = 1;
}

__device__ __forceinline__ bool key_less(int64_t t, uint32_t s, int64_t bt, uint32_t bs) {
    return t < bt || (t == bt && s < bs);
}

// size on the wire of entry x on link l.  The --train instances read an echo's size per
// link (its sender's payload with signalling type "NN" or "target", sim.cc:373-392) and
// know the big-signalling segment; the other instances never see either.
__device__ __forceinline__ uint32_t ent_size(const Sim& S, uint32_t x, uint32_t l) {
    const LV& L = S.lv;
    if (S.ctrl) {
        if (ent_is_echo(x)) return t_esz(S, l);
        if (ent_is_big(x)) return t_bs_size(S);
    }
    return ent_is_data(x) ? L.data_size() : (ent_is_echo(x) ? L.echo_size() : L.ping_size());
}
// whole seconds of a (non-negative) time, on the vector unit (numerics.h div_1e9)
#define TSEC(t) div_1e9((uint64_t)(t))
// class of entry x (type | echo bit << 2): index of TopoImage::ctx
__device__ __forceinline__ uint32_t ent_cls(uint32_t x) { return (x & 3u) | ((x >> 29) & 4u); }
// FIFO ring of link l: uniform capacities on identity overlays, per-link (sized by the
// control traffic crossing each link) on tunnelled ones.  The register-resident engine
// reads (offset | capacity << 16) from the topology image: one scalar load instead of the
// scalar arithmetic on scenario constants (A/B: +3.7 % at the headline)
__device__ __forceinline__ uint32_t ring_off(const Sim& S, uint32_t l) {
    const LV& L = S.lv;
    if (!S.mem) return S.T->rinfo[l] & 0xffffu;
    return l < (uint32_t)L.E() ? l * L.qcap_s() : (uint32_t)L.E() * L.qcap_s() + (l - (uint32_t)L.E()) * L.qcap_a();
}
__device__ __forceinline__ uint32_t ring_cap(const Sim& S, uint32_t l) {
    const LV& L = S.lv;
    if (!S.mem) return S.T->rinfo[l] >> 16;
    return l < (uint32_t)L.E() ? L.qcap_s() : L.qcap_a();
}

// one link's fields as uniform scalars
struct LinkV {
    uint32_t head, txp, tail, n_wire, n_queue, busy, qb;
    uint32_t cp_t, cp_seq;       // completion time (low 32 bits), seq
    uint32_t wh_t, wh_seq;       // wire-head arrival time (low 32 bits), seq
    uint32_t rec;                // memory-resident engine: the link's record, lane j = word j
};

template <int FS, int LS>
__device__ __forceinline__ LinkV link_get(const Regs<FS, LS>& R, uint32_t l) {
    LinkV k;
    uint32_t a = R.p0.get(l), b = R.p1.get(l), c = R.p2.get(l);
    k.head = a & 0xffffu; k.txp = a >> 16;
    k.tail = b & 0xffffu; k.n_wire = b >> 16;
    k.n_queue = c & 0xffffu; k.busy = c >> 16;
    k.qb = R.qb.get(l);
    k.cp_t = R.cp_t.get(l);
    k.cp_seq = R.cp_seq.get(l);
    k.wh_t = R.wh_t.get(l);
    k.wh_seq = R.wh_seq.get(l);
    return k;
}

// write back a link's fields and recompute its candidate key (registers only:
// the wire head's key is cached in wh_t / wh_seq)
// fields a link write-back stores: all, or (wire_pop) only the head, wire count and head key --
// the readlanes of the fields it leaves alone are then dead code
constexpr unsigned LP_ALL = 0u, LP_WIRE = 1u;
template <unsigned MASK = LP_ALL, int FS, int LS>
__device__ __forceinline__ void link_put(const Sim& S, Regs<FS, LS>& R, const Hot& H, uint32_t l, const LinkV& k) {
    R.p0.set(l, k.head | (k.txp << 16));
    R.p1.set(l, k.tail | (k.n_wire << 16));
    if (MASK == LP_ALL) {
        R.p2.set(l, k.n_queue | (k.busy << 16));
        R.qb.set(l, k.qb);
        R.cp_t.set(l, k.cp_t);
        R.cp_seq.set(l, k.cp_seq);
    }
    R.wh_t.set(l, k.wh_t);
    R.wh_seq.set(l, k.wh_seq);
}

__device__ __forceinline__ int64_t wave_min_i64(int64_t v);
__device__ __forceinline__ uint32_t wave_umin_fast(uint32_t v);
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v);

// Elided completions.  A transmit completion that finds its queue empty only clears
// `busy` (point-to-point-net-device.cc:305-336: TransmitComplete with no packet left
// schedules nothing and consumes no event uid), so the register-resident engine keeps it
// out of the event set (link_put) and settles it lazily: in link_send when the link is used
// again, and for every link at once when a launch stops (lazy_resolve).  Settling counts the
// event the reference executed (events / events_total), so every counter equals the eager
// schedule's.  Whether an elided completion precedes the event being executed (now,
// cur_seq): if the wire is empty, the transmitted packet's arrival -- scheduled after its
// completion -- has run, so the completion has too; otherwise that arrival is still ahead,
// so the completion lies within one propagation delay before the clock or one transmission
// after it (< 2^31 ns, checked on the host) and its 32-bit time offset is exact.
__device__ __forceinline__ bool lazy_due(uint32_t n_wire, uint32_t cp_t, uint32_t cp_seq, const Hot& H) {
    // (dt, cp_seq) < (0, cur_seq) with dt = cp_t - lo32(now) as a signed 32-bit offset: the sign
    // of dt * 2^32 + cp_seq - cur_seq, one 64-bit subtraction (|dt| < 2^31 whenever the wire holds
    // a packet, so the difference does not wrap; with an empty wire it is not consulted)
    const uint64_t d = ((uint64_t)(cp_t - lo32(H.now)) << 32) + (uint64_t)cp_seq - (uint64_t)H.cur_seq;
    return n_wire == 0u || (int64_t)d < 0;
}

// Settle every elided completion that precedes the current event, or -- at the end of an
// episode -- every one before simTime, moving the clock to the latest of them
// (Simulator::Stop runs every event < simTime).
template <int FS, int LS>
__device__ __forceinline__ void lazy_resolve(const Sim& S, Regs<FS, LS>& R, Hot& H, bool episode_end) {
    const LV& L = S.lv;
    const uint32_t n0 = lo32(H.now);
    const int64_t t_end = L.t_end();
    uint32_t n = 0;
    int64_t tmax = H.now;
#pragma unroll
    for (int j = 0; j < LS; ++j) {
        const uint32_t p1 = R.p1.v[j], p2 = R.p2.v[j];
        const int32_t dt = (int32_t)(R.cp_t.v[j] - n0);
        const int64_t t = H.now + (int64_t)dt;
        const bool lazy = (p2 >> 16) != 0u && (p2 & 0xffffu) == 0u;
        const bool due = lazy && (episode_end ? ((p1 >> 16) == 0u || t < t_end)
                                              : lazy_due(p1 >> 16, R.cp_t.v[j], R.cp_seq.v[j], H));
        R.p2.v[j] = due ? (p2 & 0xffffu) : p2;
        if (due && (p1 >> 16) != 0u && t > tmax) tmax = t;
        n += (uint32_t)__builtin_popcountll(__ballot(due));
    }
    H.ev_launch += n;
    if (episode_end && n) {
        const int64_t m = -wave_min_i64(-tmax);          // times are >= 0
        if (m > H.now) H.now = m;
    }
}

// flow f's next send: time, seq, draw index of that send
template <int FS, int LS>
__device__ __forceinline__ uint32_t flow_draw(const Sim& S, const Regs<FS, LS>& R, uint32_t f) {
    return R.f_draw.get(f);
}
template <int FS, int LS>
__device__ __forceinline__ void flow_min_refresh(const Sim& S, Regs<FS, LS>& R, const Hot& H) {
    int64_t ft = INT64_MAX;
    uint32_t s = 0xffffffffu, c = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < FS; ++j) {
        const int64_t tj = mk64(R.fk_lo.v[j], R.fk_hi.v[j]);
        const uint32_t sj = R.fk_seq.v[j];
        if (key_less(tj, sj, ft, s)) { ft = tj; s = sj; c = (K_FLOW << 28) | (uint32_t)(S.lane + 64 * j); }
    }
    // the ping timer competes in lane 0 (refreshed when a round re-arms it)
    if (S.lane == 0 && key_less(H.ping_t, H.ping_seq, ft, s)) { ft = H.ping_t; s = H.ping_seq; c = K_PING << 28; }
    R.fm_t = ft; R.fm_s = s; R.fm_c = c;
}
template <int FS, int LS>
__device__ __forceinline__ void flow_set(const Sim& S, Regs<FS, LS>& R, const Hot& H, uint32_t f, int64_t t,
                                         uint32_t seq, uint32_t draw) {
    R.fk_lo.set(f, lo32(t));
    R.fk_hi.set(f, hi32(t));
    R.fk_seq.set(f, seq);
    R.f_draw.set(f, draw);
    flow_min_refresh(S, R, H);
}

// ping state of tunnel t (ping_ack): oldest unacked round, acked mask, window
// state; the window mean and round lo's send time are written back only
struct PingV { uint32_t lo, mlo, mhi, win; };
template <int FS, int LS>
__device__ __forceinline__ PingV ping_get(const Sim& S, const Regs<FS, LS>& R, uint32_t t) {
    PingV p;
    p.lo = R.pm_lo.get(t); p.mlo = R.pm_mlo.get(t); p.mhi = R.pm_mhi.get(t); p.win = R.pm_win.get(t);
    return p;
}
template <int FS, int LS>
__device__ __forceinline__ void ping_set_lo(const Sim& S, Regs<FS, LS>& R, uint32_t t, uint32_t lo, uint64_t od) {
    R.pm_lo.set(t, lo);
    R.od_lo.set(t, (uint32_t)od);
    R.od_hi.set(t, (uint32_t)(od >> 32));
}
template <int FS, int LS>
__device__ __forceinline__ void ping_set_mask(const Sim& S, Regs<FS, LS>& R, uint32_t t, uint64_t mask) {
    R.pm_mlo.set(t, (uint32_t)mask);
    R.pm_mhi.set(t, (uint32_t)(mask >> 32));
}
template <int FS, int LS>
__device__ __forceinline__ void ping_set_win(const Sim& S, Regs<FS, LS>& R, uint32_t t, uint32_t win, uint64_t avg) {
    R.pm_win.set(t, win);
    R.pav_lo.set(t, (uint32_t)avg);
    R.pav_hi.set(t, (uint32_t)(avg >> 32));
}

// Wire slot i of link l: arrival time (low 32 bits), seq and -- memory-resident
// engine -- the packet entry.  Register-resident: LDS arrays; memory-resident: words
// LR_WT + {i, WCAP + i, 2 WCAP + i} of the link record held in k.rec (written back by
// link_put), so an arrival reads its packet without a ring access.
__device__ __forceinline__ void wire_set(const Sim& S, LinkV& k, uint32_t l, uint32_t i, uint32_t t, uint32_t s,
                                         uint32_t x) {
    const uint32_t W = (uint32_t)S.lv.WCAP();
    if (S.mem) {
        const uint32_t j = (uint32_t)S.lane;
        k.rec = j == LR_WT + i ? t : (j == LR_WT + W + i ? s : (j == LR_WT + 2u * W + i ? x : k.rec));
    } else {                                  // every lane stores the same value to the same address:
        S.wt[l * W + i] = t;                  // no exec-mask juggling (A/B +1 % against lane 0 only)
        S.wseq[l * W + i] = s;
        if (S.tun) S.went[l * W + i] = x;
    }
}
__device__ __forceinline__ void wire_get(const Sim& S, const LinkV& k, uint32_t l, uint32_t i, uint32_t& t,
                                         uint32_t& s) {
    const uint32_t W = (uint32_t)S.lv.WCAP();
    if (S.mem) {
        t = rdl(k.rec, LR_WT + i);
        s = rdl(k.rec, LR_WT + W + i);
    } else {
        t = u_ld32(S.wt + l * W + i);
        s = u_ld32(S.wseq + l * W + i);
    }
}
__device__ __forceinline__ uint32_t wire_ent(const Sim& S, const LinkV& k, uint32_t i) {
    return rdl(k.rec, LR_WT + 2u * (uint32_t)S.lv.WCAP() + i);
}

// ---- link FIFO / transmitter (point-to-point-net-device.cc:273-336, 595-666)
__device__ __forceinline__ void transmit_start(const Sim& S, Hot& H, uint32_t l, LinkV& k, uint32_t ring_idx,
                                               uint32_t x) {
    const LV& L = S.lv;
    const bool sw = l < (uint32_t)L.E();
    x = rfl(x);                  // uniform entry: its class indexes the topology image with a scalar load
    // register-resident engine: a switch link's tx time by entry class from the topology image
    // (--train instances: an echo's by link, sized by its sender)
    // (memory-resident: by entry type from the scenario constants; --train instances: echoes by
    // link, big-signalling segments from the BigSig header)
    uint32_t at;
    k.busy = 1;
    if (S.mem) {
        int64_t tx = sw ? ((S.ctrl && ent_is_echo(x)) ? (int64_t)t_etx(S, l)
                           : ((S.ctrl && ent_is_big(x)) ? (int64_t)S.m_bs->tx_sw
                              : (ent_is_data(x) ? L.sw_txd() : (ent_is_echo(x) ? L.sw_txe() : L.sw_txp()))))
                        : ((S.ctrl && ent_is_big(x)) ? (int64_t)t_abtx(S, l - (uint32_t)L.E())
                                                     : t_acctx(S, l - (uint32_t)L.E()));
        int64_t prop = sw ? L.sw_prop() : 0;
        k.cp_t = lo32(H.now + tx);
        at = lo32(H.now + tx + prop);
    } else {
        // register-resident engine: (tx, tx + propagation) of link l for the entry's class, low 32
        // bits, one scalar load from the topology image (TopoImage::ltx) -- the switch/access
        // selects, the 64-bit adds and the second load are the host's
        const uint32_t i = 2u * (l * 8u + ent_cls(x));
        k.cp_t = lo32(H.now) + S.T->ltx[i];
        at = lo32(H.now) + S.T->ltx[i + 1u];
    }
    k.cp_seq = H.seq++;                                        // TransmitComplete
    const uint32_t w = ring_idx & (uint32_t)(L.WCAP() - 1);
    const uint32_t as = H.seq++;                               // channel Receive
    wire_set(S, k, l, w, at, as, x);
    if (k.n_wire == 1) { k.wh_t = at; k.wh_seq = as; }        // the wire was empty: new head
    if (k.n_wire > (uint32_t)L.WCAP()) fail(H, PRISMA_EBIT_WIRE);
}

// Whether a send must store its packet in the link's FIFO ring.  Tunnelled overlays and the
// memory-resident engine keep the packets on a wire in wire slots (LDS / the link record), so a
// packet that finds the transmitter idle and nothing queued goes straight onto the wire and its
// ring slot is never read (PRISMA_RING_DIRECT): the store -- an HBM write there -- is skipped.  The
// register-resident identity overlays read arrivals from the ring and always store.
#ifndef PRISMA_RING_DIRECT
#define PRISMA_RING_DIRECT 1
#endif
__device__ __forceinline__ bool ring_store_needed(const Sim& S, const LinkV& k) {
    if (PRISMA_RING_DIRECT && (S.tun || S.mem)) return k.busy || k.n_queue != 0u;
    return true;
}

// returns 1 if enqueued, 0 if dropped (a ring overflow fails the replica)
// link_send with the link's state already fetched (the memory-resident engine's flow event
// issues the record load early); the register-resident engine keeps the plain form below,
// whose register allocation the by-value LinkV disturbs
template <class RS>
__device__ __forceinline__ int link_send_k(const Sim& S, RS& R, Hot& H, uint32_t l, uint32_t e, LinkV k) {
    const LV& L = S.lv;
    TP1_START();
    uint32_t size = ent_size(S, e, l);
    bool ok = l < (uint32_t)L.E() ? (k.qb + size <= L.qmax_bytes()) : (k.n_queue + 1u <= L.acc_qmax_pkts());
    TP1(11);
    if (!ok) return 0;
    if (RS::kLazy) {
        // the transmitter's completion was elided (nothing queued behind it): if it precedes
        // the event being executed it has happened -- count it now (lazy_due)
        const bool due = k.busy && k.n_queue == 0u && lazy_due(k.n_wire, k.cp_t, k.cp_seq, H);
        k.busy = due ? 0u : k.busy;
        H.ev_launch += due ? 1u : 0u;
    }
    uint32_t cap = ring_cap(S, l), off = ring_off(S, l);
    if (k.n_wire + k.n_queue + 1u > cap) { fail(H, PRISMA_EBIT_RING); return 0; }
    if (ring_store_needed(S, k)) q_put(S, l, off, k.tail, k.n_queue, e);
    k.tail = (k.tail + 1 == cap) ? 0 : k.tail + 1;
    k.n_queue++;
    k.qb += size;
    TP1(12);
    if (!k.busy) {                                              // :643-650
        uint32_t xi = k.txp;
        uint32_t hx = (k.n_queue == 1) ? e : q_take(S, l, off, xi);
        k.txp = (xi + 1 == cap) ? 0 : xi + 1;
        k.n_queue--;
        k.n_wire++;
        k.qb -= ent_size(S, hx, l);
        transmit_start(S, H, l, k, xi, hx);
    }
    TP1(13);
    link_put(S, R, H, l, k);
    TP1(15);
    return 1;
}
template <class RS>
__device__ __forceinline__ int link_send(const Sim& S, RS& R, Hot& H, uint32_t l, uint32_t e) {
    const LV& L = S.lv;
    LinkV k = link_get(R, l);
    uint32_t size = ent_size(S, e, l);
    // admission (switch links by queued bytes, access links by queued packets) as one compare
    // of selected operands: the compiler had branched on the link kind
    const bool sw = l < (uint32_t)L.E();
    const uint32_t have = sw ? k.qb + size : k.n_queue + 1u;
    const uint32_t lim = sw ? L.qmax_bytes() : L.acc_qmax_pkts();
    if (have > lim) return 0;
    if (RS::kLazy) {
        // the transmitter's completion was elided (nothing queued behind it): if it precedes
        // the event being executed it has happened -- count it now (lazy_due).  A uniform branch
        // on the elided state: the combined condition had become ~15 scalar mask operations
        // (busy is 0 or 1: one compare of the packed transmitter word instead of two conditions
        // the compiler combined as 64-bit lane masks)
        if (((k.busy << 16) | k.n_queue) == 0x10000u) {
            if (lazy_due(k.n_wire, k.cp_t, k.cp_seq, H)) { k.busy = 0u; H.ev_launch++; }
        }
    }
    uint32_t cap = ring_cap(S, l), off = ring_off(S, l);
    if (k.n_wire + k.n_queue + 1u > cap) { fail(H, PRISMA_EBIT_RING); return 0; }
    if (ring_store_needed(S, k)) q_put(S, l, off, k.tail, k.n_queue, e);
    k.tail = (k.tail + 1 == cap) ? 0 : k.tail + 1;
    k.n_queue++;
    k.qb += size;
    if (!k.busy) {                                              // :643-650
        uint32_t xi = k.txp;
        uint32_t hx = (k.n_queue == 1) ? e : q_take(S, l, off, xi);
        k.txp = (xi + 1 == cap) ? 0 : xi + 1;
        k.n_queue--;
        k.n_wire++;
        k.qb -= ent_size(S, hx, l);
        transmit_start(S, H, l, k, xi, hx);
    }
    link_put(S, R, H, l, k);
    return 1;
}


template <class RS>
__device__ __forceinline__ void on_complete(const Sim& S, RS& R, Hot& H, uint32_t l) {   // :305-336
    const LV& L = S.lv;
    if (S.mem) TP1_START();
    TP2_START();
    LinkV k = link_get(R, l);
    k.busy = 0;
    if (S.mem) TP1(7);
    TP2(11);
    if (k.n_queue) {
        uint32_t cap = ring_cap(S, l);
        uint32_t xi = k.txp;
        uint32_t hx = q_take(S, l, ring_off(S, l), xi);
        if (S.mem) TP1(8);
        k.txp = (xi + 1 == cap) ? 0 : xi + 1;
        k.n_queue--;
        k.n_wire++;
        k.qb -= ent_size(S, hx, l);
        transmit_start(S, H, l, k, xi, hx);
    }
    if (S.mem) TP1(9);
    TP2(12);
    link_put(S, R, H, l, k);
    if (S.mem) TP1(10);
    TP2(13);
}

// ---- observation (data-packet-manager.cc:171-206)
// send time in seconds of ping round k as the ping-back manager stores it:
// (double)GetMilliSeconds() * 0.001 (ping-back-packet-manager.cc:98-116)
// floor((k + 1) period / 10^6) on the vector unit: the product is exact (< 2^42 ns), and the
// reciprocal of 10^6 rounded up keeps a multiple of 10^6 on its quotient (numerics.h div_1e3)
__device__ __forceinline__ double ping_send_s(const LV& L, int64_t k) {
    const double ms = __builtin_floor((double)(k + 1) * (double)L.ping_period() * 0x1.0c6f7a0b5ed8ep-20);
    return ms * 0.001;
}

__device__ __forceinline__ double ld_d(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// 1000 * max(mean(window), min(now - oldest unacknowledged send, 2.6)) of a
// tunnel (data-packet-manager.cc:171-206).  The unacknowledged list is kept
// as its oldest round lo (pending iff lo < rounds sent) plus the acked bits
// of the 64 rounds after it; the window mean and lo's send time are cached
// per tunnel and refreshed on every ping-back.  Evaluated per lane for the
// tunnels the lane owns.
__device__ __forceinline__ uint32_t ping_value_lane(double avg, uint32_t lo, double od, uint32_t rounds, double now_s) {
    const bool pend = lo < rounds;
    const double a = now_s - od;
    const double b = 2.60;
    const float mt = pend ? (float)((b < a) ? b : a) : 0.0f;
    const double mx = (avg < (double)mt) ? (double)mt : avg;
    return (uint32_t)(1000 * mx);
}

// Observation of node v as a per-lane register (lane i holds obs[i], lane 0
// left 0 for the destination): every lane evaluates the tunnels (ping
// statistic) or links (queued bytes) it owns in parallel, then lane i pulls
// the value of action i-1 with one permute per register slot.  Action a of v
// is tunnel ovrow[v] + a; its queue is that of the tunnel's first link
// (the device RouteOutput picks, data-packet-manager.cc:180-195), which is
// the tunnel itself on identity overlays.
// (r0, deg: node v's row pointer and degree, read by the caller, which hands them on to the
// decision's send)
template <int FS, int LS>
__device__ __forceinline__ uint32_t observe_links(const Sim& S, const Regs<FS, LS>& R, const Hot& H, uint32_t v,
                                                  double now_s, int r0 = -1, int deg = 0) {
    if (PRISMA_ABLATE & 4) return 0u;
    if (r0 < 0) { r0 = t_ovrow(S, v); deg = t_ovrow(S, v + 1) - r0; }
    const int lane = S.lane;
    uint32_t src = (uint32_t)(r0 + lane - 1);
    const bool pobs = S.lv.ping_as_obs() != 0u;
    if (!pobs && S.tun) {
        const bool act = lane >= 1 && lane <= deg;
        src = act ? ti_link(S.T->tinfo[act ? src : 0u]) : 0u;
    }
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < LS; ++j) {
        uint32_t val;
        if (pobs && !(PRISMA_ABLATE & 64))
            val = ping_value_lane(ld_d(R.pav_lo.v[j], R.pav_hi.v[j]), R.pm_lo.v[j], ld_d(R.od_lo.v[j], R.od_hi.v[j]),
                                  H.ping_rounds, now_s);
        else
            val = R.qb.v[j];
        const uint32_t g = bperm(val, src & 63u);
        if ((src >> 6) == (uint32_t)j) o = g;
    }
    return (lane >= 1 && lane <= deg) ? o : 0u;
}

// one coalesced wave store of a decision record (lane i writes word i)
__device__ __forceinline__ void write_record(const Sim& S, const Hot& H, uint32_t d, double reward, uint32_t uid,
                                             int32_t prev, uint32_t node, uint32_t dst, uint32_t start, int action,
                                             uint32_t status, uint32_t obs_reg, uint32_t ttl) {
    if (PRISMA_ABLATE & 2) return;
    const int lane = S.lane;
    uint64_t rb = __double_as_longlong(reward);
    uint32_t w7 = (uint32_t)(uint8_t)(int8_t)action | (status << 8) | (ttl << 16) | ((H.episode & 0xffu) << 24);
    // lane l < 8 picks header word l with three lane-bit selects, no per-lane compares
    // (A/B +3.5 % at the headline against a switch on the lane id)
    // (bitfield inserts on the per-lane masks, v_bfi_b32: A/B +1.4 % at the headline against
    // lane-bit selects, whose loop-invariant SGPR-pair conditions were spilled and reloaded)
    auto bfi = [](uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); };
    const uint32_t a01 = bfi(S.m1, hi32(H.now), lo32(H.now));
    const uint32_t a23 = bfi(S.m1, (uint32_t)prev, uid);
    const uint32_t a45 = bfi(S.m1, (uint32_t)(rb >> 32), (uint32_t)rb);
    const uint32_t a67 = bfi(S.m1, w7, node | (dst << 8) | (start << 16));
    const uint32_t a03 = bfi(S.m2, a23, a01);
    const uint32_t a47 = bfi(S.m2, a67, a45);
    const uint32_t hw = bfi(S.m4, a47, a03);
    uint32_t ob = bperm(obs_reg, (uint32_t)(lane - 8) & 63u);
    uint32_t word = bfi(S.m8, hw, ob);
    uint32_t* p = (uint32_t*)(S.logrep + (size_t)(d & (S.lv.log_cap() - 1)) * S.lv.rec_bytes());
    if (lane < 8 + S.lv.W()) p[lane] = word;
}

// action + status of a record written earlier (TTL and episode bytes kept)
__device__ __forceinline__ void patch_record(const Sim& S, const Hot& H, uint32_t d, int action, uint32_t status) {
    if (PRISMA_ABLATE & 2) return;
    if (S.lane == 0) {
        unsigned char* p = S.logrep + (size_t)(d & (S.lv.log_cap() - 1)) * S.lv.rec_bytes();
        *(uint16_t*)(p + 28) = (uint16_t)((uint32_t)(uint8_t)(int8_t)action | (status << 8));
    }
}
__device__ __forceinline__ void patch_status(const Sim& S, uint32_t d, uint32_t status) {
    if (PRISMA_ABLATE & 2) return;
    if (S.lane == 0) S.logrep[(size_t)(d & (S.lv.log_cap() - 1)) * S.lv.rec_bytes() + 29] = (unsigned char)status;
}

// Receive tail after the MacRx trace (point-to-point-net-device.cc:430-463).
// arrived: a data packet at its destination (start = its start second).
// l: the arrival link (the size of an echo)
template <class RS>
__device__ __forceinline__ void receive_counters(const Sim& S, RS& R, const Hot& H, uint32_t x, bool arrived,
                                                 uint32_t start, uint32_t l) {
    const LV& L = S.lv;
    if (arrived) {
        // valable, nextHop == finalDest on identity overlays
        CNT_ADD(S, ov_arrived, 1u);
        const float cost = (float)(ns_to_sec(H.now) - (double)start);
        CNT_ADD(S, cost_sum, cost);
        CNT_ADD(S, cost_n, 1u);
        CNT_ADD(S, e2e_sum, cost);
        CNT_ADD(S, e2e_n, 1u);
    }
    // pings are always addressed to the node that receives them
    if (!ent_is_data(x)) CNT_ADD(S, bytes_signaling, ent_size(S, x, l) - 2u);
    if (ent_type(x) == T_FRESH) {
        CNT_ADD(S, ov_injected, 1u);
        CNT_ADD(S, bytes_data, L.data_size() - 2u);
    }
}

constexpr uint32_t kNoLink = 0xffffffffu;

// source node of a data entry (MyTag source) that arrived at node v: a fresh
// packet arrives at its own source switch
__device__ __forceinline__ uint32_t ent_src(uint32_t x, uint32_t v) {
    return ent_type(x) == T_FRESH ? v : r_src(x);
}

// DataPacketManager::sendSmallSignalingPacket (data-packet-manager.cc:301-347): a 0-B
// payload (30 B on the wire, signalling type "ideal") back on the arrival device,
// addressed to the data packet's last hop `to`
template <class RS>
__device__ __forceinline__ void send_echo(const Sim& S, RS& R, Hot& H, uint32_t link, uint32_t uid,
                                          uint32_t to) {
    if (!link_send(S, R, H, link, e_make(uid, to))) CNT_ADD(S, ctrl_dropped, 1u);
}

// routing table of a tunnelled overlay: next link x -> y | hops(x, y) << 8
__device__ __forceinline__ uint32_t route(const Sim& S, uint32_t x, uint32_t y) {
    const c_u32* rt = (const c_u32*)((const CAS unsigned char*)S.T + sizeof(TopoImage));
    return rt[x * (uint32_t)S.lv.N() + y];
}
// first link of tunnel t
__device__ __forceinline__ uint32_t tunnel_link(const Sim& S, uint32_t t) {
    return S.tun ? ti_link(S.T->tinfo[t]) : t;
}

// (relay_ip: ring_put)
__device__ __forceinline__ uint32_t relay_dist(const Sim& S, uint32_t d, uint32_t x) {
    return relay_ip(S) ? (d - rip_dec(x)) & kRipMask : (d - r_dec(x)) & kRelayMask;
}
// byte offsets of record words 6 (node | dst << 8 | start << 16) and 7 (action | status << 8 |
// TTL << 16 | episode << 24): write_record
__device__ __forceinline__ uint32_t record_word(const Sim& S, uint32_t d, uint32_t off) {
    return rfl(*(const uint32_t*)(S.logrep + (size_t)(d & (S.lv.log_cap() - 1)) * S.lv.rec_bytes() + off));
}
// a relayed data packet dropped on an intermediate FIFO: point-to-point-net-device.cc:655-664 at
// switch v, MacTxDrop -> the sender's loss (data-packet-manager.cc:88-98, forwarder.py:214-244)
__device__ __forceinline__ void relay_dropped(const Sim& S, uint32_t dd, uint32_t dst, uint32_t v) {
    const LV& L = S.lv;
    if (dst != v) {
        CNT_ADD(S, ov_lost, 1u);
        CNT_ADD(S, cost_sum, L.loss_penalty_f());
        CNT_ADD(S, cost_n, 1u);
    } else {
        CNT_ADD(S, un_lost, 1u);
        CNT_ADD(S, un_cost_sum, L.loss_penalty_f());
        CNT_ADD(S, un_cost_n, 1u);
    }
    patch_status(S, dd, PRISMA_ST_DROPPED);
    CNT_ADD(S, reward_sum, L.loss_penalty());
}

// DataPacketManager::sendPacket (data-packet-manager.cc:251-299) for decision
// d at node v, then the Receive tail.  x is the arriving entry (for the
// counters); fused: the record is written here once, with the final status
// (table policy).
// ROW: r0_in / deg_in hold node v's row pointer and degree (read on the arrival)
template <bool ROW = false, class RS>
__device__ __forceinline__ void apply_decision(const Sim& S, RS& R, Hot& H, uint32_t x, uint32_t dst,
                                               uint32_t start, uint32_t uid, uint32_t v, uint32_t d, int action,
                                               bool fused, double reward, int32_t prev, uint32_t obs_reg,
                                               uint32_t echo_link, uint32_t last, uint32_t ttl,
                                               int r0_in = -1, int deg_in = 0) {
    const LV& L = S.lv;
#if PRISMA_TIMING
    S.tlast = TM_NOW();
#endif
    // ExecuteActions (packet-routing-gym.cc:203-208): the --train echo goes first
    if (echo_link != kNoLink) send_echo(S, R, H, echo_link, uid, last);
    TP2_START();
    v = rfl(v);                                     // (scalar loads of the row pointers)
    int r0 = r0_in, deg = deg_in;
    if (!ROW) { r0 = t_ovrow(S, v); deg = t_ovrow(S, v + 1) - r0; }
    uint32_t status;
    if ((uint32_t)action < (uint32_t)deg) {                      // 0 <= action < deg
        const uint32_t tiw = S.tun ? (uint32_t)S.T->tinfo[(uint32_t)(r0 + action)] : 0u;
        const uint32_t l = S.tun ? ti_link(tiw) : (uint32_t)(r0 + action);   // RouteOutput (:281-287)
        if (RS::kMem || S.mlp_inst) {
            CNT_ADD(S, hops, 1u);
            CNT_ADD(S, hop_deg_sum, (uint64_t)deg);
        }
        // (memory-resident engine without the ctrl paths: the destination instead of the
        // source, engine_layout.h)
        const uint32_t src = (RS::kMem && !S.ctrl) ? dst : ent_src(x, v);
        const uint32_t fwd = relay_ip(S) ? rip_make(d, ttl, ti_tgt(tiw))
                           : ((PRISMA_ABLATE & 1) ? (T_RELAY | (dst << 2) | (start << 10) | (src << 24)) : r_make(d, src));
        TP2(7);
        if (link_send(S, R, H, l, fwd)) {                         // lastHop = v, previous decision = d
            status = PRISMA_ST_ENQUEUED;
        } else {
            status = PRISMA_ST_DROPPED;              // :655-664 + forwarder.py:214-244
            CNT_ADD(S, ov_lost, 1u);
            CNT_ADD(S, cost_sum, L.loss_penalty_f());
            CNT_ADD(S, cost_n, 1u);
            CNT_ADD(S, reward_sum, L.loss_penalty());
        }
    } else {
        status = PRISMA_ST_DISCARDED;
    }
#if PRISMA_TIMING
    { const uint64_t t = TM_NOW(); S.tsub[0] += t - S.tlast; S.tlast = t; }
#endif
    TP0(12);
    TP2(8);
    if (fused) write_record(S, H, d, reward, uid, prev, v, dst, start, action, status, obs_reg, ttl);
    else patch_record(S, H, d, action, status);
    TP2(9);
    if (RS::kMem || S.mlp_inst) {
        receive_counters(S, R, H, x, false, 0u, 0u);
    } else if (S.lane == 0) {
        // table instances: the hop's integer counters and the Receive tail's (a data packet:
        // receive_counters) in one lane-0 region -- integer adds, so their order is free (A/B:
        // headline +0.7 %)
        if ((uint32_t)action < (uint32_t)deg) {
            lds_add(&S.c->hops, (decltype(S.c->hops))1u);
            lds_add(&S.c->hop_deg_sum, (decltype(S.c->hop_deg_sum))deg);
        }
        if (ent_type(x) == T_FRESH) {
            lds_add(&S.c->ov_injected, (decltype(S.c->ov_injected))1u);
            lds_add(&S.c->bytes_data, (decltype(S.c->bytes_data))(L.data_size() - 2u));
        }
    }
    TP2(10);
#if PRISMA_TIMING
    { const uint64_t t = TM_NOW(); S.tsub[1] += t - S.tlast; S.tlast = t; }
#endif
    TP0(13);
}

// Answer to the pending notification.  Returns 1 if a hop was executed (0 for a
// destination or control notification, whose action is ignored: sendPacket at
// the destination does nothing (:256-260), ExecuteActions sends nothing for a
// small-signalling packet).
template <class RS>
__device__ __forceinline__ int finish_pending(const Sim& S, RS& R, Hot& H, int action) {
    const Hdr& h = *S.h;
    H.pend = 0;
    const uint32_t x = u_ld32(&h.pend_ent[0]), flags = u_ld32(&h.pend_ent[3]);
    if (S.ctrl && (flags & PEND_CTRL)) {
        receive_counters(S, R, H, x, false, 0u, u_ld32(&h.pend_link));
        return 0;
    }
    const uint32_t echo_link = (S.ctrl && (flags & PEND_ECHO)) ? (uint32_t)t_lrev(S, u_ld32(&h.pend_link)) : kNoLink;
    const uint32_t last = u_ld32(&h.pend_last);
    if (S.ctrl && (flags & PEND_DEST)) {
        if (echo_link != kNoLink) send_echo(S, R, H, echo_link, u_ld32(&h.pend_uid), last);
        receive_counters(S, R, H, x, true, u_ld32(&h.pend_ent[2]), 0u);
        return 0;
    }
    // (relay entries with the TTL: the pending decision's, from its record)
    const uint32_t pdec = u_ld32(&h.pend_dec);
    const uint32_t ttl = relay_ip(S) ? (record_word(S, pdec, 28) >> 16) & 255u : 0u;
    apply_decision(S, R, H, x, 0u, 0u, u_ld32(&h.pend_uid), u_ld32(&h.pend_node), pdec, action,
                   false, 0.0, 0, 0u, echo_link, last, ttl);
    return 1;
}

// ---- handlers (uniform) ------------------------------------------------------
template <class RS>
__device__ __forceinline__ void on_ping_round(const Sim& S, RS& R, Hot& H) {   // data-packet-manager.cc:350-413
    const LV& L = S.lv;
    uint32_t k = H.ping_rounds;
    uint32_t first_rearm = 0;
    for (int i = 0; i < L.NO(); ++i) {                            // timers in overlay order (sim.cc:528-546)
        const int u = S.tun ? S.T->ovnode[i] : i;
        const int r0 = t_ovrow(S, u), r1 = t_ovrow(S, u + 1);
        for (int t = r0; t < r1; ++t) {
            if (!link_send(S, R, H, tunnel_link(S, (uint32_t)t), p_make(T_PFWD, (uint32_t)t, 0u, k)))
                CNT_ADD(S, ctrl_dropped, 1u);
        }
        uint32_t s = H.seq++;                                    // re-arm of node u
        if (i == 0) first_rearm = s;
    }
    H.ping_rounds = k + 1;
    // one ns-3 event per overlay node timer (the round is NO consecutive events)
    H.ev_launch += (uint32_t)(L.NO() - 1);
    H.ping_t = H.now + L.ping_period();
    H.ping_seq = first_rearm;
    flow_min_refresh(S, R, H);
}

// ns-3 stream mode (PRISMA_RNG_NS3): the uniform of the ExponentialRandomVariable that
// ScheduleNextTx creates for every packet (poisson-application.cc:281-284) -- the first value
// of a new stream.  A packet's SendPacket creates a UniformRandomVariable first (:311-314; its
// value only sets the tag's overlay flag, 1 for every flow here), so draws after the first skip
// one stream.  State: the next stream's initial state and the jump J, in LDS (kRngBytes).
__device__ __forceinline__ double ns3_exp_u01(const Sim& S, uint32_t draw) {
    uint32_t* g = (uint32_t*)(S.base + S.lv.lds_state_bytes() - kRngBytes);
    uint32_t st[6], J[18];
#pragma unroll
    for (int i = 0; i < 6; ++i) st[i] = u_ld32(g + i);
#pragma unroll
    for (int i = 0; i < 18; ++i) J[i] = u_ld32(g + 8 + i);
    if (draw != 0) mrg_apply(J, st);                              // SendPacket's uniform stream
    uint32_t e[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) e[i] = st[i];
    const double U = mrg_u01(e);
    mrg_apply(J, st);
#pragma unroll
    for (int i = 0; i < 6; ++i) st_rep(S, g + i, st[i]);
    return U;
}

// ns-3 stream mode at an episode start: flow f's start offset comes from the
// UniformRandomVariable the flow loop creates for it (sim.cc:610-620), the f-th stream from
// rng_stream_offset on -- state J^f T, from the table's powers of J -- and the LDS image gets
// the run's first stream (the one after the flows') and J.  rep: the replica's table entry.
__device__ __forceinline__ double ns3_start_u01(const uint32_t* rng, const uint32_t* rep, uint32_t f) {
    uint32_t st[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) st[i] = rep[i];
    for (uint32_t b = 0; b < kMrgPowers; ++b)
        if ((f >> b) & 1u) mrg_apply(rng + 18u * b, st);
    return mrg_u01(st);
}
__device__ __forceinline__ void ns3_init_lds(const Sim& S, const uint32_t* rng, const uint32_t* rep) {
    uint32_t* g = (uint32_t*)(S.base + S.lv.lds_state_bytes() - kRngBytes);
    if (S.lane < 6) g[S.lane] = rep[6 + S.lane];
    else if (S.lane >= 8 && S.lane < 26) g[S.lane] = rng[S.lane - 8];
}

template <class RS>
__device__ __forceinline__ void flow_next(const Sim& S, RS& R, Hot& H, uint32_t f, uint32_t draw) {
    // (only the CTRL instances carry the ns-3 streams: the host picks them for rng_mode, so the
    // Philox instances' event loop keeps its registers)
    if (S.ctrl && S.lv.rng_mode()) {
        const double delay = -t_fmean(S, f) * det_log(ns3_exp_u01(S, draw));
        flow_set(S, R, H, f, H.now + sec_to_ns(delay), H.seq++, draw + 1);
        return;
    }
    // The draw cache (register-resident engine, where LDS has room: Layout::s_dcache = LDS offset
    // | K): a flow's draws come in groups of K (2 or 3). The first draw of a group is computed in
    // lane 0 and the next K - 1 in lanes 1 .. K-1 by the same vector instructions -- Philox, the
    // logarithm and the conversion cost one draw -- and their send delays wait in the flow's LDS
    // slots for its next sends. Every draw keeps its own Philox counter (flow, draw, episode), so
    // the values are the uncached ones; an episode starts each flow at draw 0, which refills the
    // slots before the first read.
    constexpr bool kDc = !RS::kMem && RS::kDcache;
    const uint32_t dcw = kDc ? S.lv.s_dcache() : 0u;
    if (kDc && dcw != 0u) {
        const uint32_t K = dcw & 15u;
        int64_t* slot = (int64_t*)(S.base + (dcw & ~15u)) + f * (K - 1u);
        const uint32_t g = (K == 2u) ? (draw & 1u) : draw - 3u * (uint32_t)(((uint64_t)draw * 0xAAAAAAABull) >> 33);
        int64_t dns;
        if (g != 0u) {
            dns = u_ld64(slot + (g - 1u));
        } else {
            const uint32_t j = (uint32_t)S.lane < K ? (uint32_t)S.lane : 0u;
            uint32_t c[4] = { f, draw + j, H.episode, 1u };
            philox4x32_10(c, S.lv.seed_lo(), S.gid);
            const uint64_t u53 = ((uint64_t)(c[0] >> 5) << 26) | (uint64_t)(c[1] >> 6);
            const double U = ((double)u53 + 1.0) * (1.0 / 9007199254740992.0);
            const int64_t dn = sec_to_ns(-t_fmean(S, f) * det_log(U));
            if (j != 0u) slot[j - 1u] = dn;
            dns = mk64(rfl(lo32(dn)), rfl(hi32(dn)));
        }
        flow_set(S, R, H, f, H.now + dns, H.seq++, draw + 1);
        return;
    }
    uint32_t c[4] = { f, draw, H.episode, 1u };                   // poisson-application.cc:265-295
    // The table-policy instances run the rounds on the vector unit (the values pass through
    // VGPRs, so the compiler cannot keep them scalar) and take back the two words they use:
    // ~80 scalar instructions per flow event moved off the headline's busiest unit.  The MLP
    // instances keep the scalar rounds with their keys hoisted out of the event loop.
    uint32_t k0 = S.lv.seed_lo(), k1 = S.gid;
    if (PRISMA_ABLATE & 8) {                                      // diagnostic: a cheap hash, not Philox
        c[0] = (f * 2654435761u) ^ (draw * 2246822519u) ^ (k1 * 3266489917u) ^ H.episode;
        c[1] = c[0] * 668265263u ^ (c[0] >> 15);
    } else {
    if (!S.mlp_inst) asm volatile("" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(k0), "+v"(k1));
    philox4x32_10(c, k0, k1);
    if (!S.mlp_inst) { c[0] = __builtin_amdgcn_readfirstlane(c[0]); c[1] = __builtin_amdgcn_readfirstlane(c[1]); }
    }
    uint64_t u53 = ((uint64_t)(c[0] >> 5) << 26) | (uint64_t)(c[1] >> 6);
    double U = ((double)u53 + 1.0) * (1.0 / 9007199254740992.0);
    double delay = (PRISMA_ABLATE & 16) ? -t_fmean(S, f) * (double)__logf((float)U) : -t_fmean(S, f) * det_log(U);
    int64_t t = H.now + sec_to_ns(delay);
    if constexpr (RS::kMem) TM_FLOW(2);
    flow_set(S, R, H, f, t, H.seq++, draw + 1);
    if constexpr (RS::kMem) TM_FLOW(3);
}

// The BigSignalingGeneratorApplications (big-signaling-application.cc:224-309), all in flow
// slot F.  Every generator starts at AppStartTime and sends one 512-B segment per period, so
// all of them fire at the same instants, in install order (their seqs were taken in that order
// one period earlier, and every seq taken in between belongs to an access-link event of the
// group, at most one transmission later): like a ping round, one slot executes the G
// consecutive ns-3 events -- the first of them starts the sends (StartSending), the others
// hand segment k to the traffic node's access link (SendPacket :261-309) -- and re-arms with
// the seq of the first reschedule (ScheduleNextTx :235-259).
template <class RS>
__device__ __forceinline__ void on_bsig(const Sim& S, RS& R, Hot& H, uint32_t f) {
    const uint32_t k = flow_draw(S, R, f);
    const uint32_t G = t_ngen(S), E = (uint32_t)S.lv.E();
    if (k > kGenSendMask) fail(H, PRISMA_EBIT_TIME);                // 17-bit send index (host-checked)
    uint32_t first = 0;
    for (uint32_t g = 0; g < G; ++g) {
        if (k != 0 && !link_send(S, R, H, E + bp_src(t_bpair(S, g)), g_make(g, k))) CNT_ADD(S, ctrl_dropped, 1u);
        const uint32_t sq = H.seq++;
        if (g == 0) first = sq;
    }
    H.ev_launch += G - 1u;
    flow_set(S, R, H, f, H.now + t_bs_period(S), first, k + 1u);
}

template <class RS>
__device__ __forceinline__ void on_flow(const Sim& S, RS& R, Hot& H, uint32_t f) {
    // memory-resident engine: the access link's record is fetched first, so its load and the
    // flow block's are in flight together (one HBM round trip)
    uint32_t draw;
#if PRISMA_TIMING
    S.tfl = TM_NOW();
#endif
    if constexpr (RS::kMem) {
        if (S.ctrl && f >= (uint32_t)S.lv.F()) { on_bsig(S, R, H, f); return; }
        const uint32_t acc = (uint32_t)S.lv.E() + (uint32_t)t_fsrc(S, f);
        const LinkV k = link_get(R, acc);
        draw = flow_draw(S, R, f);
        TM_FLOW(0);
        if (draw != 0) {                                            // SendPacket :297-358
            const uint32_t par = (uint32_t)(TSEC(H.now)) & 1u;          // start second (its parity)
            link_send_k(S, R, H, acc, f_make((uint32_t)t_fdst(S, f), par, H.uid & kUidMask), k);
            H.uid++;
        }
        TM_FLOW(1);
    } else {
        if (S.ctrl && f >= (uint32_t)S.lv.F()) { on_bsig(S, R, H, f); return; }
        TP2_START();
        draw = flow_draw(S, R, f);
        if (draw != 0) {
            const uint32_t src = (uint32_t)t_fsrc(S, f);
            const uint32_t par = (uint32_t)(TSEC(H.now)) & 1u;
            TP2(14);
            link_send(S, R, H, (uint32_t)S.lv.E() + src, f_make((uint32_t)t_fdst(S, f), par, H.uid & kUidMask));
            H.uid++;
        }
        TP2(15);
    }
    flow_next(S, R, H, f, draw);                                    // StartSending / ScheduleNextTx
}

// ---- in-kernel DQN_buffer_model (models.py:258-306; fixed fp32 operation order,
// DESIGN.md §2, restated by the oracle's mlp_action): lane j computes unit j of
// each layer, activations are broadcast through 64 floats of LDS, weights are
// read per lane from HBM (L2-resident, shared by every replica).
// The layers read their weights from an interleaved per-node copy (prisma_mlp_repack_kernel,
// filled by prisma_run from the caller's row-major weights). Node block = [L1][L2][L3][L4]:
// * L1: the buffers branch, chunk c holding Wb[4c..4c+3][j] as one float4 per unit j < 32
//   (rows k >= D zero), then bb[32] and b1[32] (the one-hot rows of W1 stay in the caller's
//   buffer: one row per decision);
// * L2, L3, L4: chunk c holding W[4c..4c+3][j] as one float4 per output unit j, then the
//   bias row.
// Lane j loads one coalesced 16-B value per 4 inputs instead of 4 dependent 4-B ones, and
// the accumulation order (input 0, 1, 2, ..., one fmaf each) is unchanged.
__host__ __device__ constexpr int mlp_rp_l1_floats(int D) { return 128 * ((D + 3) / 4) + 64; }
__host__ __device__ constexpr int mlp_rp_layer_floats(int units) { return 64 * units + units; }
__host__ __device__ constexpr int mlp_rp_node_floats(int D) {   // rounded to whole float4s
    return (mlp_rp_l1_floats(D) + 2 * mlp_rp_layer_floats(64) + mlp_rp_layer_floats(D) + 3) & ~3;
}

// B: float4 weight loads in flight per lane (one L2 round trip per B chunks); 4 where the
// kernel must fit 128 VGPRs (4 waves per SIMD), more where it has 256
template <int B>
__device__ __forceinline__ float mlp_dense64(const Sim& S, const float* __restrict__ Wl, int lane, int units) {
    const float4* __restrict__ W4 = (const float4*)Wl;
    const float4* __restrict__ hb = (const float4*)S.hbuf;
    const float b = Wl[64 * units + lane];
    float acc = 0.0f;
#pragma unroll
    for (int c0 = 0; c0 < 16; c0 += B) {
        float4 w[B];
#pragma unroll
        for (int c = 0; c < B; ++c) w[c] = W4[(c0 + c) * units + lane];
#pragma unroll
        for (int c = 0; c < B; ++c) {
            const float4 h = hb[c0 + c];
            acc = __builtin_fmaf(h.x, w[c].x, acc);
            acc = __builtin_fmaf(h.y, w[c].y, acc);
            acc = __builtin_fmaf(h.z, w[c].z, acc);
            acc = __builtin_fmaf(h.w, w[c].w, acc);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    return __fadd_rn(acc, b);
}

// B == kMlpAll (memory-resident engine, one wave per SIMD and VGPRs to spare): every
// weight of layers 2-4 is loaded when the decision starts, one round trip in all
constexpr int kMlpAll = 64;
struct MlpPre {
    float4 w2[16], w3[16], w4[16];
    float b2, b3, b4;
};
// what the memory-resident engine's arrival handler fetches for the decision that follows
// (layer 1's buffer-branch chunks and bias, layer 2): it rides along the arrival's second
// round trip, and layers 3-4 load while layers 1-2 compute
struct MlpPre1 {
    float4 w2[16];
    float b2;
    float4 wb[4];
    float b1v;
    float w1v;                   // the one-hot row element, when the destination was known (has_w1)
    bool has_w1;
};

__device__ __forceinline__ void mlp_preload(MlpPre& M, const float* __restrict__ RP, int lane, int D, int deg,
                                            bool l2 = true) {
    const float4* __restrict__ W2 = l2 ? (const float4*)RP : nullptr;
    const float4* __restrict__ W3 = (const float4*)(RP + mlp_rp_layer_floats(64));
    const float4* __restrict__ W4 = (const float4*)(RP + 2 * mlp_rp_layer_floats(64));
    if (W2) {
#pragma unroll
        for (int c = 0; c < 16; ++c) M.w2[c] = W2[c * 64 + lane];
        M.b2 = RP[64 * 64 + lane];
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) M.w3[c] = W3[c * 64 + lane];
    // layer 4: lanes past deg read lane 0's weights (their outputs are discarded), so every
    // load of the stream is unconditional and the in-order load counter can be waited on
    // exactly (exec-masked loads made the compiler wait for layer 3's weights in layer 1)
    const int l4 = lane < deg ? lane : 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) M.w4[c] = W4[c * D + l4];
    M.b3 = RP[mlp_rp_layer_floats(64) + 64 * 64 + lane];
    M.b4 = RP[2 * mlp_rp_layer_floats(64) + 64 * D + l4];
}

// mlp_preload's layer-3 and layer-4 halves (the memory-resident engine issues them apart)
__device__ __forceinline__ void mlp_preload_w3(MlpPre& M, const float* __restrict__ RP, int lane) {
    const float4* __restrict__ W3 = (const float4*)(RP + mlp_rp_layer_floats(64));
#pragma unroll
    for (int c = 0; c < 16; ++c) M.w3[c] = W3[c * 64 + lane];
    M.b3 = RP[mlp_rp_layer_floats(64) + 64 * 64 + lane];
}
__device__ __forceinline__ void mlp_preload_w4(MlpPre& M, const float* __restrict__ RP, int lane, int D, int deg) {
    const float4* __restrict__ W4 = (const float4*)(RP + 2 * mlp_rp_layer_floats(64));
    const int l4 = lane < deg ? lane : 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) M.w4[c] = W4[c * D + l4];
    M.b4 = RP[2 * mlp_rp_layer_floats(64) + 64 * D + l4];
}

// layers 1-2 of a decision at node v (the one-hot row too when the destination dst is
// known, has_w1): issued by the memory-resident engine's arrival handler together with
// its second round trip (previous decision record, observation), so the decision finds
// them in registers
// PRISMA_PRE_W2: layer 2's weights ride along the arrival's second round trip (1) or are issued when
// the decision starts (0, round 5: +4.8 % at config 5 -- the arrival's gather no longer waits behind
// 17 weight loads, and their 64 VGPRs are not held across the arrival's tree repair)
#ifndef PRISMA_PRE_W2
#define PRISMA_PRE_W2 0
#endif
__device__ __forceinline__ void mlp_preload_node(MlpPre1& M, const Sim& S, uint32_t v, uint32_t dst, bool has_w1) {
    const int lane = S.lane;
    v = rfl(v);                  // uniform: the row pointers come from scalar loads
    const int D = S.lv.max_deg();
    const float* __restrict__ RP1 = S.mlp_rp + (size_t)v * mlp_rp_node_floats(D);
    const float* __restrict__ RP = RP1 + mlp_rp_l1_floats(D);
    const int deg = t_ovrow(S, v + 1) - t_ovrow(S, v);
    M.has_w1 = has_w1;
    M.w1v = 0.0f;
    if (has_w1 && lane < 32) M.w1v = S.mlp[((int)v * S.lv.N() + (int)dst) * 32 + (lane & 31)];
    if (PRISMA_PRE_W2) {
#pragma unroll
        for (int c = 0; c < 16; ++c) M.w2[c] = ((const float4*)RP)[c * 64 + lane];
        M.b2 = RP[64 * 64 + lane];
    }
    const int j32 = lane & 31, nck = (deg + 3) >> 2;
    const float4* __restrict__ Wb4 = (const float4*)RP1;
#pragma unroll
    for (int c = 0; c < 4; ++c) M.wb[c] = (c < nck) ? Wb4[c * 32 + j32] : make_float4(0.f, 0.f, 0.f, 0.f);
    M.b1v = (lane < 32) ? RP1[128 * ((D + 3) / 4) + 32 + j32] : RP1[128 * ((D + 3) / 4) + j32];
}

__device__ __forceinline__ float mlp_dense64_pre(const Sim& S, const float4 (&w)[16], float b) {
    const float4* __restrict__ hb = (const float4*)S.hbuf;
    float acc = 0.0f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const float4 h = hb[c];
        acc = __builtin_fmaf(h.x, w[c].x, acc);
        acc = __builtin_fmaf(h.y, w[c].y, acc);
        acc = __builtin_fmaf(h.z, w[c].z, acc);
        acc = __builtin_fmaf(h.w, w[c].w, acc);
    }
    return __fadd_rn(acc, b);
}

// Layers 2-4 of the register-resident instances with the weight loads one batch ahead: batch
// t+1's loads (across layer boundaries too) are issued before batch t's FMAs, so each L2 round
// trip overlaps a batch of FMAs instead of standing alone.  Per lane the same operations in
// the same order as mlp_dense64 for each layer (bit-identical); layer 4's lanes past deg read
// lane 0's weights and their outputs are discarded by the caller.
#ifndef PRISMA_MLP_PIPE
#define PRISMA_MLP_PIPE 1
#endif
template <int B>
__device__ __forceinline__ void mlp_l2_first(float4 (&w0)[B], const float* __restrict__ RP, int lane) {
    const float4* __restrict__ W4 = (const float4*)RP;
#pragma unroll
    for (int c = 0; c < B; ++c) w0[c] = W4[c * 64 + lane];
}
// w0: layer 2's first batch, issued by the caller before layer 1 (mlp_l2_first) when EARLY
// (the 256-VGPR instances: config 4 +1.2 % over issuing it here; the 128-VGPR ones lose 0.5 %)
template <int B, bool EARLY>
__device__ __forceinline__ float mlp_l234_pipe(const Sim& S, const float* __restrict__ RP, int lane, int D, int deg,
                                               const float4 (&w0)[B]) {
    constexpr int NB = 16 / B, T = 3 * NB;
    // B must divide the 16 chunks of a layer, and EARLY (issue(0) skipped: the caller issued
    // batch 0) needs a later batch of layer 2 to load its bias
    static_assert(16 % B == 0 && (!EARLY || NB >= 2), "mlp_l234_pipe: B must divide 16; EARLY needs 16 / B >= 2");
    const float4* __restrict__ hb = (const float4*)S.hbuf;
    const int l4 = lane < deg ? lane : 0;
    float4 w[2][B];
    float bias[3];
    if constexpr (EARLY) {
#pragma unroll
        for (int c = 0; c < B; ++c) w[0][c] = w0[c];
    }
    auto issue = [&](int t) {
        const int Lk = t / NB, c0 = (t % NB) * B;
        const int units = Lk < 2 ? 64 : D, ln = Lk < 2 ? lane : l4;
        const float* __restrict__ Wl = RP + Lk * mlp_rp_layer_floats(64);
        const float4* __restrict__ W4 = (const float4*)Wl;
#pragma unroll
        for (int c = 0; c < B; ++c) w[t & 1][c] = W4[(c0 + c) * units + ln];
        if (t % NB == NB - 1) bias[Lk] = Wl[64 * units + ln];
    };
    float acc = 0.0f, q = 0.0f;
    if constexpr (!EARLY) issue(0);
#pragma unroll
    for (int t = 0; t < T; ++t) {
        if (t + 1 < T) issue(t + 1);
        __builtin_amdgcn_sched_barrier(0);
        const int c0 = (t % NB) * B;
#pragma unroll
        for (int c = 0; c < B; ++c) {
            const float4 h = hb[c0 + c];
            acc = __builtin_fmaf(h.x, w[t & 1][c].x, acc);
            acc = __builtin_fmaf(h.y, w[t & 1][c].y, acc);
            acc = __builtin_fmaf(h.z, w[t & 1][c].z, acc);
            acc = __builtin_fmaf(h.w, w[t & 1][c].w, acc);
        }
        if (t % NB == NB - 1) {
            const int Lk = t / NB;
            const float o = det_elu(__fadd_rn(acc, bias[Lk]));
            acc = 0.0f;
            if (Lk < 2) {
                __builtin_amdgcn_wave_barrier();
                S.hbuf[lane] = o;
                __builtin_amdgcn_wave_barrier();
            } else {
                q = o;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    return q;
}

// one-hot input: obs[0] (the destination's overlay index, lane 0 of obs_reg)
__device__ __forceinline__ float rdlf(float x, uint32_t k) { return __uint_as_float(rdl(__float_as_uint(x), k)); }

// x of lanes 1..n summed in lane order (((0 + x1) + x2) + ...), four readlanes issued per
// step; a lane past n contributes -0.0f, the identity of round-to-nearest addition (the sum
// starts at +0 and so is never -0), so the result equals the one-add-per-lane loop's
__device__ __forceinline__ float lane_sum_ordered(float x, int n) {
    float sum = 0.0f;
    for (int k0 = 0; k0 < n; k0 += 4) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = (k0 + i < n) ? rdlf(x, (uint32_t)(k0 + i + 1) & 63u) : -0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) sum = __fadd_rn(sum, v[i]);
    }
    return sum;
}

// tf.argmin over q of lanes 0..n-1 as the reference's scan: the first minimum (learner.py:145)
// (the register-resident instances: their degrees are small)
__device__ __forceinline__ int lane_argmin_first_seq(float q, int n) {
    int best = 0;
    float bq = rdlf(q, 0);
    for (int a = 1; a < n; ++a) {
        const float qa = rdlf(q, (uint32_t)a);
        if (qa < bq) { bq = qa; best = a; }
    }
    return best;
}

// tf.argmin over q of lanes 0..n-1, the first minimum (learner.py:145): the result of
// `best = 0; for a in 1..n-1: if q[a] < q[best]: best = a`, as one DPP reduction of an
// order-preserving key (+0 and -0 equal; a NaN past lane 0 never wins; a NaN in lane 0 wins,
// since nothing compares below it) and a ballot for the lowest lane among equal keys
__device__ __forceinline__ int lane_argmin_first(float q, int n) {
    const int lane = (int)threadIdx.x;
    uint32_t u = __float_as_uint(q);
    u = (u << 1) == 0u ? 0u : u;                                    // -0 -> +0
    uint32_t key = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    key = (lane >= n || (q != q)) ? 0xffffffffu : key;
    const uint32_t kmin = wave_umin_fast(key);
    const float q0 = rdlf(q, 0);
    if (q0 != q0) return 0;
    return (int)__builtin_ctzll(__ballot(key == kmin));
}

// LayerNorm and layer 1 from LDS (the memory-resident engine, PRISMA_LN_LDS): the deg buffer
// values (and later their squared deviations and normalised values) sit at hbuf[0..deg-1], +0
// past the degree, and every lane reads them back as 16-B broadcasts -- the sums and the layer-1
// FMA chain run in the oracle's order on VGPR operands instead of a v_readlane per term.  A +0 term
// is an exact identity here: the sums start at +0 and add non-negative values (never -0), and
// fma(+0, w, acc) = acc for finite w and acc != -0 (acc starts at +0 and an exact cancellation
// rounds to +0).
#ifndef PRISMA_LN_LDS
#define PRISMA_LN_LDS 1
#endif
__device__ __forceinline__ float lds_sum_ordered(const float4* hb4, int nck) {
    float4 h[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) h[c] = hb4[c];                      // 32 slots, all written
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if (c >= nck) break;                                        // uniform
        s = __fadd_rn(s, h[c].x); s = __fadd_rn(s, h[c].y); s = __fadd_rn(s, h[c].z); s = __fadd_rn(s, h[c].w);
    }
    for (int c = 8; c < nck; ++c) {                                 // degrees beyond 32
        const float4 g = hb4[c];
        s = __fadd_rn(s, g.x); s = __fadd_rn(s, g.y); s = __fadd_rn(s, g.z); s = __fadd_rn(s, g.w);
    }
    return s;
}
// a / d for an integer d (the node's degree) with rd = RN(1/d): q = a rd and one FMA correction
// (Markstein), the correctly rounded quotient for 2^-120 <= a (and a = 0) and 1 <= d <= 64 --
// checked exhaustively over every float a in that range (scripts/checks/div_deg_exhaustive.c; a
// sample in tests/test_numerics_division.py)
__device__ __forceinline__ float div_deg(float a, float d, float rd) {
    const float q = __fmul_rn(a, rd);
    const float e = __builtin_fmaf(-q, d, a);
    return __builtin_fmaf(e, rd, q);
}

template <int B, bool PRE = false>
__device__ __forceinline__ int mlp_action(const Sim& S, uint32_t v, uint32_t obs_reg, const MlpPre1& P1) {
    const LV& L = S.lv;
    const int lane = S.lane;
    const int N = L.N(), D = L.max_deg();
    // v (and with it deg) uniform: the row pointers then come from scalar loads.  Passed through
    // the decision record the compiler had lost that, loaded deg with vector loads and waited
    // for them behind the layer 3-4 weight stream (s_waitcnt vmcnt), and ran the LayerNorm
    // sums as exec-mask loops
    v = rfl(v);
    const float* __restrict__ W1 = S.mlp;
    const float* __restrict__ RP1 = S.mlp_rp + (size_t)v * mlp_rp_node_floats(D);
    const float* __restrict__ RP = RP1 + mlp_rp_l1_floats(D);
#if PRISMA_TIMING
    uint64_t tq = TM_NOW(), tq1;
#define TM_MLP(i) do { tq1 = TM_NOW(); S.tmlp[i] += tq1 - tq; tq = tq1; } while (0)
#else
#define TM_MLP(i) do { } while (0)
#endif
    if (PRISMA_TP_SET == 0) TP_START();
#if PRISMA_TIMING
    if constexpr (PRE) __builtin_amdgcn_s_waitcnt(0);     // the arrival's loads (probe only)
#endif
    TP0(0);
    const int deg = t_ovrow(S, v + 1) - t_ovrow(S, v);
    const uint32_t dst = rdl(obs_reg, 0);
    // layer-1 weights first (independent of the normalisation): one W1 row element and
    // b1 for the one-hot branch (lanes 0-31), the Wb chunks and bb for the buffers branch
    // (lanes 32-63; deg <= D, so at most ceil(D/4) chunks).  The row element is issued
    // before the layer 3-4 loads: the in-order load counter makes layer 1 wait for
    // everything issued before it.
    const int j32 = lane & 31;
    const int nck = (deg + 3) >> 2;
    const float4* __restrict__ Wb4 = (const float4*)RP1;
    float w1v;
    if (PRE && P1.has_w1) w1v = P1.w1v;
    else w1v = (lane < 32) ? W1[((int)v * N + (int)dst) * 32 + j32] : 0.0f;
    // memory-resident engine: buffer-branch chunks 4-7 (degrees 17-32) are loaded here, BEFORE
    // the layer 3-4 stream: the load counter is in order, so a chunk loaded inside layer 1
    // made layer 1 wait for the whole stream (and the compiler, unable to count the loop's
    // loads, waited for everything before layer 2)
    float4 wx[4];
    if constexpr (B == kMlpAll) {
        // (always issued, chunk 0 again past the node's degree: no branch for the scheduler to
        // hoist the stream's loads above)
#pragma unroll
        for (int c = 0; c < 4; ++c) wx[c] = Wb4[((c + 4 < nck) ? c + 4 : 0) * 32 + j32];
        __builtin_amdgcn_sched_barrier(0);
    }
    MlpPre M;
    // PRE (memory-resident engine): layer 2 came with the arrival, and layers 3-4 are issued in
    // two halves inside the LayerNorm below, so their issue overlaps its dependent chain instead
    // of holding the wave in front of it
    if constexpr (B == kMlpAll && !PRE) mlp_preload(M, RP, lane, D, deg, true);
    if constexpr (B == kMlpAll && PRE && !PRISMA_PRE_W2) {
#pragma unroll
        for (int c = 0; c < 16; ++c) M.w2[c] = ((const float4*)RP)[c * 64 + lane];
        M.b2 = RP[64 * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
    }
    float b1v;
    float4 wb[4];
    if constexpr (PRE) {
        b1v = P1.b1v;
#pragma unroll
        for (int c = 0; c < 4; ++c) wb[c] = P1.wb[c];
    } else {
        b1v = (lane < 32) ? RP1[128 * ((D + 3) / 4) + 32 + j32] : RP1[128 * ((D + 3) / 4) + j32];
#pragma unroll
        for (int c = 0; c < 4; ++c) wb[c] = (c < nck) ? Wb4[c * 32 + j32] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // register-resident instances (PRISMA_MLP_PIPE): layer 2's first weights go out now and
    // load during the LayerNorm and layer 1
    constexpr int kPipeB = (B != kMlpAll && B >= 2) ? B / 2 : 1;
    constexpr bool kPipeEarly = B != kMlpAll && B >= 8;
    float4 w20[kPipeB];
    if constexpr (kPipeEarly && PRISMA_MLP_PIPE) mlp_l2_first<kPipeB>(w20, RP, lane);
    // LayerNormalization of the deg buffer values (population variance, epsilon 1e-3):
    // lane k+1 holds buffer value k; sums run in k order through readlanes
    // (the memory-resident engine's single wave per SIMD gains from the 4-wide sums and the
    // DPP argmin below; the register-resident MLP instances lost 1 % with them, A/B on GEANT)
    const float xf = (float)obs_reg;
    // (the register-resident instances lost 0.5-1.2 % with it at 4 waves per SIMD, round-5 A/B)
    constexpr bool kLnLds = (B == kMlpAll) && PRISMA_LN_LDS;
    const float4* hb4 = (const float4*)S.hbuf;
    const bool inb = lane >= 1 && lane <= deg;
    const float fdeg = (float)deg;
    float rdeg = 0.0f;
    float sum = 0.0f;
    if constexpr (kLnLds) {
        rdeg = __fdiv_rn(1.0f, fdeg);                               // off the sums' chain
        S.hbuf[(lane - 1) & 63] = inb ? xf : 0.0f;                  // value k at hbuf[k]
        __builtin_amdgcn_wave_barrier();
        sum = lds_sum_ordered(hb4, nck);
    } else if constexpr (B == kMlpAll) sum = lane_sum_ordered(xf, deg);
    else for (int k = 0; k < deg; ++k) sum = __fadd_rn(sum, rdlf(xf, (uint32_t)(k + 1)));
    TP0(1);
    if constexpr (B == kMlpAll && PRE) {
        __builtin_amdgcn_sched_barrier(0);
        mlp_preload_w3(M, RP, lane);
        __builtin_amdgcn_sched_barrier(0);
    }
    TP0(2);
    const float mean = kLnLds ? div_deg(sum, fdeg, rdeg) : __fdiv_rn(sum, (float)deg);
    const float dv = __fsub_rn(xf, mean);
    const float sq = __fmul_rn(dv, dv);
    float var = 0.0f;
    if constexpr (kLnLds) {
        __builtin_amdgcn_wave_barrier();
        S.hbuf[(lane - 1) & 63] = inb ? sq : 0.0f;
        __builtin_amdgcn_wave_barrier();
        var = lds_sum_ordered(hb4, nck);
    } else if constexpr (B == kMlpAll) var = lane_sum_ordered(sq, deg);
    else for (int k = 0; k < deg; ++k) var = __fadd_rn(var, rdlf(sq, (uint32_t)(k + 1)));
    TP0(3);
    if constexpr (B == kMlpAll && PRE) {
        __builtin_amdgcn_sched_barrier(0);
        mlp_preload_w4(M, RP, lane, D, deg);
        __builtin_amdgcn_sched_barrier(0);
    }
    TP0(4);
    var = kLnLds ? div_deg(var, fdeg, rdeg) : __fdiv_rn(var, (float)deg);
    const float den = __fsqrt_rn(__fadd_rn(var, 1e-3f));
    const float xn = __fdiv_rn(dv, den);                          // lane k+1: normalised value k
    if constexpr (kLnLds) {
        __builtin_amdgcn_wave_barrier();
        S.hbuf[(lane - 1) & 63] = inb ? xn : 0.0f;
        __builtin_amdgcn_wave_barrier();
    }
    TP0(5);
    // layer 1: one-hot(dst) branch in lanes 0-31, buffers branch in lanes 32-63. The
    // buffers dot product runs with every lane active (lanes 0-31 discard it): its
    // readlanes read xn from lanes 1..deg, which must not sit in an inactive branch.
    float acc = 0.0f;
    auto chunk = [&](int c, const float4& w) {
        const int k = 4 * c;
        acc = __builtin_fmaf(rdlf(xn, (uint32_t)(k + 1)), w.x, acc);
        if (k + 1 < deg) acc = __builtin_fmaf(rdlf(xn, (uint32_t)(k + 2)), w.y, acc);
        if (k + 2 < deg) acc = __builtin_fmaf(rdlf(xn, (uint32_t)(k + 3)), w.z, acc);
        if (k + 3 < deg) acc = __builtin_fmaf(rdlf(xn, (uint32_t)(k + 4)), w.w, acc);
    };
    if constexpr (kLnLds) {
        // every term of a chunk (+0 past the degree), the inputs as LDS broadcasts
        auto chunk4 = [&](const float4& x, const float4& w) {
            acc = __builtin_fmaf(x.x, w.x, acc);
            acc = __builtin_fmaf(x.y, w.y, acc);
            acc = __builtin_fmaf(x.z, w.z, acc);
            acc = __builtin_fmaf(x.w, w.w, acc);
        };
        float4 h[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) h[c] = hb4[c];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if (c >= nck) break;
            if constexpr (B == kMlpAll) chunk4(h[c], c < 4 ? wb[c & 3] : wx[c & 3]);
            else chunk4(h[c], c < 4 ? wb[c & 3] : Wb4[c * 32 + j32]);
        }
        for (int c = 8; c < nck; ++c) chunk4(hb4[c], Wb4[c * 32 + j32]);
    } else if constexpr (B == kMlpAll) {
        // chunks named at compile time (a runtime-indexed select over wb/wx put them on the stack)
#pragma unroll
        for (int c = 0; c < 8; ++c)
            if (c < nck) chunk(c, c < 4 ? wb[c & 3] : wx[c & 3]);
        for (int c = 8; c < nck; ++c) chunk(c, Wb4[c * 32 + j32]);
    } else {
        for (int c = 0; c < nck; ++c) {
            float4 w;
            if (c < 4) {
                w = (c == 0) ? wb[0] : (c == 1) ? wb[1] : (c == 2) ? wb[2] : wb[3];
            } else {
                w = Wb4[c * 32 + j32];
            }
            chunk(c, w);
        }
    }
    TP0(6);
    float h = (B == kMlpAll) ? det_elu_sel(__fadd_rn(lane < 32 ? w1v : acc, b1v))
                             : det_elu(__fadd_rn(lane < 32 ? w1v : acc, b1v));
    if constexpr (kLnLds) __builtin_amdgcn_wave_barrier();
    S.hbuf[lane] = h;
    __builtin_amdgcn_wave_barrier();
    TP0(7);
    TM_MLP(0);
    if constexpr (B != kMlpAll && PRISMA_MLP_PIPE) {
        // (half batches double-buffered: the same weight registers as B loads in flight)
        const float q4 = mlp_l234_pipe<kPipeB, kPipeEarly>(S, RP, lane, D, deg, w20);
        __builtin_amdgcn_wave_barrier();
        return lane_argmin_first_seq(q4, deg);
    }
    if constexpr (PRE && PRISMA_PRE_W2) h = det_elu_sel(mlp_dense64_pre(S, P1.w2, P1.b2));
    else if constexpr (PRE) h = det_elu_sel(mlp_dense64_pre(S, M.w2, M.b2));
    else if constexpr (B == kMlpAll) h = det_elu_sel(mlp_dense64_pre(S, M.w2, M.b2));
    else h = det_elu(mlp_dense64<B>(S, RP, lane, 64));
    __builtin_amdgcn_wave_barrier();
    S.hbuf[lane] = h;
    __builtin_amdgcn_wave_barrier();
    TP0(8);
    TM_MLP(1);
    if constexpr (B == kMlpAll) h = det_elu_sel(mlp_dense64_pre(S, M.w3, M.b3));
    else h = det_elu(mlp_dense64<B>(S, RP + mlp_rp_layer_floats(64), lane, 64));
    __builtin_amdgcn_wave_barrier();
    S.hbuf[lane] = h;
    __builtin_amdgcn_wave_barrier();
    TP0(9);
    TM_MLP(2);
    float q = 0.0f;
    if constexpr (B == kMlpAll) {
        const float q4 = det_elu_sel(mlp_dense64_pre(S, M.w4, M.b4));
        if (lane < deg) q = q4;
    } else {
        if (lane < deg) q = det_elu(mlp_dense64<B>(S, RP + 2 * mlp_rp_layer_floats(64), lane, D));
    }
    __builtin_amdgcn_wave_barrier();
    TP0(10);
    // tf.argmin: first minimum (learner.py:145)
    int best;
    if constexpr (B == kMlpAll) best = lane_argmin_first(q, deg);
    else best = lane_argmin_first_seq(q, deg);
    TP0(11);
    TM_MLP(3);
    return best;
}

// the head packet leaves the wire of link l (arrival at the far end)
template <class RS>
__device__ __forceinline__ void wire_pop(const Sim& S, RS& R, const Hot& H, uint32_t l, LinkV& k) {
    const LV& L = S.lv;
    const uint32_t cap = ring_cap(S, l);
    k.head = (k.head + 1 == cap) ? 0 : k.head + 1;
    k.n_wire--;
    if (k.n_wire) {                                                 // next packet on the wire
        const uint32_t w = k.head & (uint32_t)(L.WCAP() - 1);
        wire_get(S, k, l, w, k.wh_t, k.wh_seq);
    }
    link_put<LP_WIRE>(S, R, H, l, k);
}

struct Decision {
    uint32_t x, dst, start, uid, v, d; double reward; int32_t prev; uint32_t obs, flags, last, ttl;
    int32_t r0, deg;             // register-resident engine: node v's row pointer and degree (r0 < 0: not read)
};

// a control packet (or a data packet inside a tunnel) continues along the
// underlay route to `to` (Ipv4L3Protocol::IpForward through the patched
// Ipv4Interface::Send, ipv4-interface.cc:213-229)
template <class RS>
__device__ __forceinline__ void ctrl_forward(const Sim& S, RS& R, Hot& H, uint32_t v, uint32_t to,
                                             uint32_t x) {
    if (!link_send(S, R, H, ti_link(route(S, v, to)), x)) CNT_ADD(S, ctrl_dropped, 1u);
}

// PingBackPacketManager::receivePacket (ping-back-packet-manager.cc:120-144) on
// tunnel lt with the one-hop delay the ping-back carries
template <class RS>
__device__ __forceinline__ void ping_ack(const Sim& S, RS& R, Hot& H, uint32_t lt, uint32_t rnd,
                                         float delay) {
    const LV& L = S.lv;
    // the round itself (rounds in flight are less than 2^18 behind the last one sent)
    const uint32_t last = H.ping_rounds - 1u;
    const uint32_t k = last - ((last - rnd) & kRoundMask);
    // erase round k from the unacknowledged list (first match; none if already acked)
    const PingV pv = ping_get(S, R, lt);
    uint32_t lo = pv.lo;
    uint64_t mask = ((uint64_t)pv.mhi << 32) | pv.mlo;
    uint32_t pw = pv.win;
    if (k == lo) {
        if (pw >> 31) fail(H, PRISMA_EBIT_ACKORDER);               // acked bits were lost (see below)
        const uint32_t n = (uint32_t)__builtin_ctzll(~mask);       // rounds lo+1.. already acked
        lo += 1u + n;
        mask = (n >= 63u) ? 0ull : (mask >> (n + 1u));
        ping_set_lo(S, R, lt, lo, (uint64_t)__double_as_longlong(ping_send_s(L, lo)));
        ping_set_mask(S, R, lt, mask);
    } else if (k > lo) {
        const uint32_t b = k - lo - 1u;
        if (b < 64u) {
            mask |= 1ull << b;
            ping_set_mask(S, R, lt, mask);
        } else {
            pw |= 1u << 31;      // round lo is lost for good unless acked > 64 rounds late
        }
    }
    // tunnelsDelay window (MA newest delays, oldest first)
    const uint32_t MA = L.ma();
    uint32_t wn = pw & 0xffffu, wh = (pw >> 16) & 0x7fffu, slot;
    if (wn >= MA) {
        slot = wh;
        wh = (wh + 1 == MA) ? 0 : wh + 1;
    } else {
        slot = wh + wn;
        if (slot >= MA) slot -= MA;
        wn++;
    }
    const uint32_t pw_new = wn | (wh << 16) | (pw & (1u << 31));
    st_rep(S, &S.win[lt * MA + slot], delay);
    // refresh the cached window mean (data-packet-manager.cc:55-65), summed oldest first
    double sum = 0.0;
    uint32_t i = wh;
    if constexpr (RS::kMem) {
        // the memory-resident engine's windows are in HBM: one load of the whole window (lane m:
        // slot m), then the slots in order through readlanes -- one round trip instead of one per
        // slot (the loop had waited for each load in turn; round 5, config 5 +0.2 %)
        const uint32_t wl = ((uint32_t)S.lane < MA) ? ((const uint32_t*)S.win)[lt * MA + (uint32_t)S.lane] : 0u;
        for (uint32_t j = 0; j < wn; ++j) {
            const float w = (i == slot) ? delay : __uint_as_float(rdl(wl, i));
            sum += (double)w;
            i = (i + 1 == MA) ? 0 : i + 1;
        }
    } else {
        for (uint32_t j = 0; j < wn; ++j) {
            float w = (i == slot) ? delay : __uint_as_float(u_ld32((const uint32_t*)S.win + lt * MA + i));
            sum += (double)w;
            i = (i + 1 == MA) ? 0 : i + 1;
        }
    }
    ping_set_win(S, R, lt, pw_new, (uint64_t)__double_as_longlong(sum / (double)wn));
}

// ping-back delay slot of responder position pos on tunnel t (tunnelled overlays): one
// slot per overlay node on the tunnel
__device__ __forceinline__ uint32_t pbd_slot(const Sim& S, uint32_t t, uint32_t pos) {
    const uint32_t tr = S.T->tresp[t];
    return (tr & 0xffffu) + (uint32_t)__builtin_popcount((tr >> 16) & ((1u << pos) - 1u));
}

// returns 1 if a data decision needs an action
template <bool PRE = false, class RS>
__device__ __forceinline__ int on_arrive(const Sim& S, RS& R, Hot& H, uint32_t l, Decision& D, bool fused,
                                         MlpPre1& Mpre) {
    const LV& L = S.lv;
    if (S.mem) TP1_START();
    TP2_START();
    const uint32_t v = (uint32_t)t_ldst(S, l);
    LinkV k = link_get(R, l);
    const uint32_t wh = k.head & (uint32_t)(L.WCAP() - 1);
    const uint32_t x = S.mem ? wire_ent(S, k, wh)
                             : (S.tun ? u_ld32(&S.went[l * (uint32_t)L.WCAP() + wh])
                                      : u_ld32(&S.ring[ring_off(S, l) + k.head]));
    if (S.mem) TP1(0);
    TP2(0);
    const uint32_t type = ent_type(x);
    const bool tun = S.tun;
    if (relay_ip(S) && type == T_RELAY && rip_tgt(x) != v) {
        // a switch inside the packet's tunnel: IP-forwarded towards the tunnel's target
        // (packet-manager.cc:115 -> not valid, no Notify) on the entry alone
        wire_pop(S, R, H, l, k);
        const uint32_t d = H.dec, dist = relay_dist(S, d, x);
        if (dist >= L.log_cap()) fail(H, PRISMA_EBIT_LOGWRAP);
        // IpForward decrements the TTL first and drops at 0 (no trace, no counter)
        const uint32_t tt = rip_ttl(x);
        if (tt == 1u) return 0;
        const uint32_t xf = tt == kRipTtlSat ? x : x - (1u << 20);
        if (!link_send(S, R, H, ti_link(route(S, v, rip_tgt(x))), xf))
            relay_dropped(S, d - dist, (record_word(S, d - dist, 24) >> 8) & 255u, v);
        return 0;
    }
    if (ent_is_data(x)) {
        // PacketRoutingEnv::NotifyPktRcv -> Notify (packet-routing-gym.cc:231-267)
        // A forwarded packet's previous decision record (t_ns, uid, dst,
        // start, deciding node + action, TTL) comes from the HBM log -- the
        // temp_obs entry of forwarder.py:153-159.  The load is issued first
        // and consumed after the link update and the observation, which do
        // not depend on it (and only on this path, so no load is ever left
        // in flight across loop iterations).
        // (A fresh packet loads and ignores some record of its own log: the
        // load and its consumption are unconditional on this path.)
        const uint32_t d = H.dec;
        const uint32_t dist = relay_dist(S, d, x);
        const unsigned char* pr = S.logrep + (size_t)((d - dist) & (L.log_cap() - 1)) * L.rec_bytes();
        const uint4 ph = *(const uint4*)pr;
        const uint2 pw = *(const uint2*)(pr + 24);
        if constexpr (PRE) {                                        // the decision's weights ride along
            if (S.ctrl) {
                mlp_preload_node(Mpre, S, v, 0u, false);
            } else {
                // the entry names the destination (engine_layout.h): no weights for a
                // packet that has arrived, the one-hot row element with the others
                const uint32_t dst_e = (type == T_FRESH) ? f_dst(x) : r_dst(x);
                if (dst_e != v) mlp_preload_node(Mpre, S, v, dst_e, true);
            }
        }
        // memory-resident engine: the observation's gather goes out with the record
        // load, before the arrival link's update (it reads node v's out-links, which
        // nothing touches before the decision)
        const uint32_t obs_early = S.mem ? observe_links(S, R, H, v, ns_to_sec(H.now)) : 0u;
        if (S.mem) TP1(1);
        TP2(1);
        wire_pop(S, R, H, l, k);
        if (S.mem) TP1(2);
        TP2(2);
        uint32_t ttl = 255u;                                        // SetIpTtl(255) (poisson-application.cc:330)
        if (tun && type == T_RELAY) {
            // Tunnelled overlay: the packet's next hop is the target of the tunnel
            // the previous decision picked; anywhere else it is only IP-forwarded
            // (packet-manager.cc:115 -> not valid, no Notify).
            const uint32_t w6p = rfl(pw.x), w7p = rfl(pw.y);
            const uint32_t u = w6p & 255u;
            const uint32_t ti = S.T->tinfo[(uint32_t)t_ovrow(S, u) + (w7p & 255u)];
            const uint32_t ttl_prev = (w7p >> 16) & 255u;
            if (ti_tgt(ti) != v) {
                // (relay_ip: the entry named this node as the target, so the record is not this
                // packet's -- the log wrapped past the 18-bit decision index)
                if (relay_ip(S)) { fail(H, PRISMA_EBIT_LOGWRAP); return 0; }
                if (dist >= L.log_cap()) fail(H, PRISMA_EBIT_LOGWRAP);
                // IpForward decrements the TTL first and drops at 0 (no trace, no counter)
                if (ttl_prev == (route(S, u, v) >> 8)) return 0;
                if (!link_send(S, R, H, ti_link(route(S, v, ti_tgt(ti))), x))
                    relay_dropped(S, d - dist, (w6p >> 8) & 255u, v);
                return 0;
            }
            ttl = ttl_prev - (ti_len(ti) - 1u);
        }
        H.dec = d + 1u;
        int r0 = -1, deg = 0;
        if (!S.mem) { r0 = t_ovrow(S, v); deg = t_ovrow(S, v + 1) - r0; }
        const uint32_t obs_links = S.mem ? obs_early : observe_links(S, R, H, v, ns_to_sec(H.now), r0, deg);
        D.r0 = r0; D.deg = deg;
        const int64_t t_prev = mk64(rfl(ph.x), rfl(ph.y));
        const uint32_t uid_prev = rfl(ph.z), w_prev = rfl(pw.x);
        if (S.mem) TP1(3);
        TP2(3);
        double reward = 0.0;
        int32_t prev = -1;
        uint32_t dst, start, uid, last = 0u;
        if (type == T_FRESH) {
            // first notification: destination from the flow, uid and start
            // second rebuilt from their low bits (the packet left its app less
            // than 1 s and fewer than 2^20 injections ago)
            dst = f_dst(x);
            const uint32_t s0 = (uint32_t)(TSEC(H.now));
            start = s0 - ((s0 ^ f_parity(x)) & 1u);
            const uint32_t lu = H.uid - 1u;
            uid = lu - ((lu - f_uid(x)) & kUidMask);
        } else if (PRISMA_ABLATE & 1) {
            dst = (x >> 2) & 255u; start = x >> 10; uid = 0; prev = (int32_t)d - 1;
        } else {
            prev = (int32_t)(d - dist);
            if (dist >= L.log_cap()) fail(H, PRISMA_EBIT_LOGWRAP);
            uid = uid_prev;
            dst = (w_prev >> 8) & 255u;
            start = w_prev >> 16;
            last = w_prev & 255u;
            if (PRISMA_ABLATE & 32) {
                reward = (double)(uint32_t)(H.now - t_prev);                  // (diagnostic builds only)
            } else if (PRISMA_REWARD_LANES) {
                // the reward's two clock terms (forwarder.py:360) in lanes 0 and 1 of one vector
                // evaluation -- now in even lanes, the previous decision's time in odd ones -- and
                // lane 0 takes the difference with lane 1's term brought over by a DPP move
                const uint32_t m = S.m1;                                      // -(lane & 1)
                const int64_t tt = mk64((lo32(t_prev) & m) | (lo32(H.now) & ~m), (hi32(t_prev) & m) | (hi32(H.now) & ~m));
                const double us = us_to_sec(py_micros(tt));
                const uint64_t ub = (uint64_t)__double_as_longlong(us);
                const double up = __longlong_as_double((long long)mk64(dpp_u32<0xB1, 0xF>((uint32_t)ub),
                                                                       dpp_u32<0xB1, 0xF>((uint32_t)(ub >> 32))));
                const uint64_t rb = (uint64_t)__double_as_longlong(us - up);
                reward = __longlong_as_double((long long)mk64(rfl((uint32_t)rb), rfl((uint32_t)(rb >> 32))));
            } else {
                reward = us_to_sec(py_micros(H.now)) - us_to_sec(py_micros(t_prev));   // forwarder.py:360
            }
            CNT_ADD(S, reward_sum, reward);
        }
        // obs[0] = m_map_overlay_array[dst] (the identity on identity overlays)
        const uint32_t o = (S.lane == 0) ? (tun ? (uint32_t)S.T->ovi[dst] : dst) : obs_links;
        CNT_ADD(S, decisions, 1u);
        // --train: the answer to this notification also echoes a small-signalling
        // packet to the last hop, unless this node is the packet's source (:303-306)
        const uint32_t echo = (S.ctrl && L.train() && v != ent_src(x, v)) ? PEND_ECHO : 0u;
        D.x = x; D.dst = dst; D.start = start; D.uid = uid; D.v = v; D.d = d; D.reward = reward; D.prev = prev;
        D.obs = o; D.flags = echo; D.last = last; D.ttl = ttl;
        if (dst == v) {                                             // getGameOver
            write_record(S, H, d, reward, uid, prev, v, dst, start, -1, PRISMA_ST_DESTINATION, o, ttl);
            if (!fused && S.ctrl && L.notify_dest()) {              // the agent is notified (done=True)
                D.flags |= PEND_DEST;
                return 1;
            }
            if (echo) send_echo(S, R, H, (uint32_t)t_lrev(S, l), uid, last);
            receive_counters(S, R, H, x, true, start, 0u);
            return 0;
        }
        if (!fused) write_record(S, H, d, reward, uid, prev, v, dst, start, -1, PRISMA_ST_PENDING, o, ttl);
        if (S.mem) TP1(4);
        TP2(4);
        return 1;
    }
    wire_pop(S, R, H, l, k);
    if (S.mem) TP1(5);
    TP2(5);
    if (S.ctrl && ent_is_big(x)) {                                  // (only with --signaling and --train)
        const uint32_t bp = t_bpair(S, g_gen(x));
        const uint32_t src = bp_src(bp), dst = bp_dst(bp);
        if (v == src) {                  // from the traffic node: IP-forwarded towards its destination
            if (!link_send(S, R, H, bp_link(bp), x)) CNT_ADD(S, ctrl_dropped, 1u);
            return 0;
        }
        if (tun && v != dst) { ctrl_forward(S, R, H, v, dst, x); return 0; }
        // BigSignalingPacketManager::receivePacket (big-signaling-packet-manager.cc:93-108):
        // at its destination, not its source -> Notify; obs [1000] (+ NN / segment index, sender)
        if (!fused && L.notify_dest()) {
            const uint32_t n = g_n(x), ns = t_bs_nseg(S);
            const uint32_t nn = ns <= 1u ? n : n / ns, seg = ns <= 1u ? 0u : n % ns;
            const uint32_t so = 0x10000u | (tun ? (uint32_t)S.T->ovi[src] : src);
            D.x = x; D.v = v; D.uid = 0u; D.flags = PEND_CTRL; D.last = 0u;
            D.obs = (S.lane == 0) ? 1000u : ((S.lane == 1) ? nn : ((S.lane == 2) ? seg : ((S.lane == 3) ? so : 0u)));
            return 1;
        }
        receive_counters(S, R, H, x, false, 0u, l);
        return 0;
    }
    if (S.ctrl && ent_is_echo(x)) {                                 // (echoes exist only with --train)
        const uint32_t to = e_to(x);
        if (tun && to != v) { ctrl_forward(S, R, H, v, to, x); return 0; }
        // SmallSignalingPacketManager::receivePacket (small-signaling-packet-manager.cc:86-94):
        // addressed to this node, so valid -> Notify; the agent sees obs [1000]
        if (!fused && S.ctrl && L.notify_dest()) {
            D.x = x; D.v = v; D.uid = e_uid(x); D.flags = PEND_CTRL; D.last = 0u;
            const uint32_t sz = ent_size(S, x, l);
            D.obs = (S.lane == 0) ? 1000u : ((S.lane == 1) ? e_uid(x) : ((S.lane == 2) ? sz : 0u));
            return 1;
        }
        receive_counters(S, R, H, x, false, 0u, l);
        return 0;
    }
    // pings.  NotifyPktRcv hands every ping seen on an overlay node's devices to
    // its managers, addressed to it or not (packet-routing-gym.cc:254-259); the
    // packet itself continues to its addressee (IP forwarding).
    const uint32_t t = p_tunnel(x), rnd = p_round(x);
    const uint32_t ti = tun ? (uint32_t)S.T->tinfo[t] : 0u;
    const bool ovl = !tun || S.T->ovi[v] >= 0;
    if (type == T_PFWD) {                                           // ping-forward-packet-manager.cc:94-156
        const uint32_t tgt = tun ? ti_tgt(ti) : v;
        if (ovl) {
            // responder position on the tunnel: its own delay slot
            const uint32_t pos = tun ? (route(S, ti_org(ti), v) >> 8) - 1u : 0u;
            const float delay = (float)(ns_to_sec(H.now) - ping_send_s(L, rnd));
            const uint32_t slot = tun ? pbd_slot(S, t, pos) : t;
            st_rep(S, &S.pbd[slot * L.PBK() + (rnd & (L.PBK() - 1))], delay);
            if (!link_send(S, R, H, (uint32_t)t_lrev(S, l), p_make(T_PBACK, t, pos, rnd))) CNT_ADD(S, ctrl_dropped, 1u);
        }
        if (tgt != v) { ctrl_forward(S, R, H, v, tgt, x); return 0; }
    } else {                                                        // ping-back-packet-manager.cc:120-144
        const uint32_t org = tun ? ti_org(ti) : v;
        if (ovl) {
            const uint32_t slot = tun ? pbd_slot(S, t, p_pos(x)) : t;
            const float delay = __uint_as_float(u_ld32((const uint32_t*)S.pbd + slot * L.PBK() + (rnd & (L.PBK() - 1))));
            if (!tun) {
                ping_ack(S, R, H, t, rnd, delay);                  // identity: tunnel == link
            } else {
                // the ORIGIN's tunnel index applied to this node's own tunnel list
                const uint32_t idx = t - (uint32_t)t_ovrow(S, org);
                const uint32_t v0 = (uint32_t)t_ovrow(S, v);
                if (idx >= (uint32_t)t_ovrow(S, v + 1) - v0) fail(H, PRISMA_EBIT_PINGIDX);
                else ping_ack(S, R, H, v0 + idx, rnd, delay);
            }
        }
        if (org != v) { ctrl_forward(S, R, H, v, org, x); return 0; }
    }
    receive_counters(S, R, H, x, false, 0u, l);
    if (S.mem) TP1(6);
    TP2(6);
    return 0;
}

// ---------------------------------------------------------------------------
// replica (re)initialisation: LDS image zeroed, registers set (all lanes)
// ---------------------------------------------------------------------------
// keep_totals: carry the header's hops_total / events_total over (auto-reset)
template <int FS, int LS>
// rng / r: the ns-3 stream table and the replica's local index (null: Philox streams)
__device__ __forceinline__ void init_replica(Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t episode, bool keep_totals,
                                             const uint32_t* rng, uint32_t r) {
    const LV& L = S.lv;
    const int lane = S.lane;
    uint32_t dec = H.dec, hl = H.hops_launch, el = H.ev_launch;
    const uint64_t ht = keep_totals ? (uint64_t)u_ld64((const int64_t*)&S.h->hops_total) : 0u;
    const uint64_t et = keep_totals ? (uint64_t)u_ld64((const int64_t*)&S.h->events_total) : 0u;
    __syncthreads();
    uint4* st4 = (uint4*)S.base;
    for (uint32_t i = (uint32_t)lane; i < L.lds_state_bytes() / 16u; i += kWave) st4[i] = make_uint4(0, 0, 0, 0);
    const uint32_t* rep = rng ? rng + 18u * kMrgPowers + kMrgRepWords * r : nullptr;
    if (rng) {
        __syncthreads();
        ns3_init_lds(S, rng, rep);
    }
    // big-signalling generators: flow slot F (on_bsig), each generator started right after its
    // flow (sim.cc:599-647: the start events in install order, fseq)
    const bool bsig = S.ctrl && !S.mem;
    const uint32_t nbs = bsig ? S.T->n_bsig : 0u;
#pragma unroll
    for (int j = 0; j < FS; ++j) {
        uint32_t f = (uint32_t)lane + 64u * j;
        int64_t t = INT64_MAX;
        uint32_t s = 0xffffffffu;
        if (f < (uint32_t)L.F()) {
            double U;
            if (rng) {
                U = ns3_start_u01(rng, rep, f);
            } else {
                uint32_t c[4] = { f, 0u, episode, 0u };
                philox4x32_10(c, L.seed_lo(), S.gid);
                uint64_t u53 = ((uint64_t)(c[0] >> 5) << 26) | (uint64_t)(c[1] >> 6);
                U = (double)u53 * (1.0 / 9007199254740992.0);
            }
            t = sec_to_ns(0.0001 + U);                              // sim.cc:610-630
            s = bsig ? S.T->fseq[f] : (uint32_t)L.NO() + f;    // after the NO ping timers
        } else if (nbs && f == (uint32_t)L.F()) {
            t = sec_to_ns(0.0001);                                  // AppStartTime (sim.cc:244, 645)
            s = S.T->fseq[f];                                       // generator 0's start
        }
        R.fk_lo.v[j] = lo32(t); R.fk_hi.v[j] = hi32(t); R.fk_seq.v[j] = s; R.f_draw.v[j] = 0;
    }
#pragma unroll
    for (int j = 0; j < LS; ++j) {
        R.cp_t.v[j] = 0; R.cp_seq.v[j] = 0; R.wh_t.v[j] = 0; R.wh_seq.v[j] = 0;
        R.p0.v[j] = 0; R.p1.v[j] = 0; R.p2.v[j] = 0; R.qb.v[j] = 0;
        R.pm_lo.v[j] = 0; R.pm_mlo.v[j] = 0; R.pm_mhi.v[j] = 0; R.pm_win.v[j] = 0;
        R.pav_lo.v[j] = 0; R.pav_hi.v[j] = 0;
        uint64_t od = __double_as_longlong(ping_send_s(L, 0));
        R.od_lo.v[j] = (uint32_t)od; R.od_hi.v[j] = (uint32_t)(od >> 32);
    }
    H.now = 0;
    H.ping_t = L.ping_period();                                       // data-packet-manager.cc:118-121
    H.ping_seq = 0;
    H.seq = (uint32_t)L.NO() + (uint32_t)L.F() + nbs;
    H.uid = 0; H.ping_rounds = 0; H.pend = 0; H.over = 0; H.error = 0; H.stop = 0;
    H.dec = dec; H.hops_launch = hl; H.ev_launch = el;
    H.episode = episode;
    if (lane == 0) {
        S.c->episode = episode;
        S.h->hops_total = ht;
        S.h->events_total = et;
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// wave-wide reductions to lane 63 (DPP row/bank steps)
// ---------------------------------------------------------------------------
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROW_MASK, 0xf, false);
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int64_t dpp_min_i64(int64_t v) {
    uint32_t lo = dpp_u32<CTRL, ROW_MASK>(lo32(v));
    uint32_t hi = dpp_u32<CTRL, ROW_MASK>(hi32(v));
    int64_t o = mk64(lo, hi);
    return o < v ? o : v;
}

__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
    v = dpp_min_i64<0xB1, 0xF>(v);      // quad_perm [1,0,3,2]
    v = dpp_min_i64<0x4E, 0xF>(v);      // quad_perm [2,3,0,1]
    v = dpp_min_i64<0x141, 0xF>(v);     // row_half_mirror
    v = dpp_min_i64<0x140, 0xF>(v);     // row_mirror
    v = dpp_min_i64<0x142, 0xA>(v);     // row_bcast:15
    v = dpp_min_i64<0x143, 0xC>(v);     // row_bcast:31
    return mk64(rdl(lo32(v), 63), rdl(hi32(v), 63));
}

// One DPP step of an unsigned min, folded by the compiler into v_min_u32
// with a DPP source: rows outside ROW_MASK see the identity (~0u).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_umin(uint32_t v) {
    uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, CTRL, ROW_MASK, 0xf, false);
    return o < v ? o : v;
}

__device__ __forceinline__ uint32_t wave_umin_fast(uint32_t v) {
    v = dpp_umin<0xB1, 0xF>(v);
    v = dpp_umin<0x4E, 0xF>(v);
    v = dpp_umin<0x141, 0xF>(v);
    v = dpp_umin<0x140, 0xF>(v);
    v = dpp_umin<0x142, 0xA>(v);
    v = dpp_umin<0x143, 0xC>(v);
    return rdl(v, 63);
}

// Next event = min (time, seq) over every source of the replica, as 32-bit
// offsets from the clock: each lane reduces the sources it owns
// lexicographically on (offset, seq), the wave reduces the lane minima with
// fused DPP min steps.  Link events are always < 2^31 ns ahead; a flow or the
// ping timer further than 2^32-2 ns ahead saturates, and if every source
// saturates the exact 64-bit reduction over flows and ping runs instead.
__device__ __forceinline__ void key_take(uint32_t k, uint32_t s, uint32_t c, uint32_t& bk, uint32_t& bs,
                                         uint32_t& bc) {
    // (offset, seq) as one 64-bit key: one compare and three selects.  Written as
    // `k < bk || (k == bk && s < bs)` the short-circuit became exec-mask branches, ~20 scalar
    // instructions per event selection (A/B: +3.7 % at the headline, +2.3 % at configs 3 and 4)
    const bool t = (((uint64_t)k << 32) | s) < (((uint64_t)bk << 32) | bs);
    bk = t ? k : bk;
    bs = t ? s : bs;
    bc = t ? c : bc;
}

__device__ __forceinline__ uint32_t sat_offset(int64_t t, int64_t now) {
    const uint64_t dt = (uint64_t)(t - now);
    return (dt >> 32) ? 0xffffffffu : (uint32_t)dt;
}

template <int FS, int LS>
__device__ __forceinline__ void select_event(const Sim& S, const Regs<FS, LS>& R, const Hot& H, int lane, int64_t& bt,
                                             uint32_t& bc, uint32_t& bs) {
    // flows and the ping timer: each lane's cached earliest (flow_min_refresh), then one offset
    int64_t ft = R.fm_t;
    uint32_t s = R.fm_s, c = R.fm_c;
    uint32_t k = sat_offset(ft, H.now);
    // links: 32-bit offsets
    const uint32_t n0 = lo32(H.now);
#pragma unroll
    for (int j = 0; j < LS; ++j) {
        // each lane derives its links' candidates from their state: the completion while
        // packets wait behind the transmitter (elided otherwise, lazy_due), the wire head's
        // arrival while the wire holds packets -- no stored key to maintain in link_put
        // (A/B: +5.4 % at the headline, +6 % at config 3)
        const uint32_t p2 = R.p2.v[j];
        const bool cpv = (p2 >> 16) != 0u && (p2 & 0xffffu) != 0u;
        const bool whv = (R.p1.v[j] >> 16) != 0u;
        const uint32_t oc = cpv ? R.cp_t.v[j] - n0 : 0xffffffffu;
        const uint32_t ow = whv ? R.wh_t.v[j] - n0 : 0xffffffffu;
        const uint32_t code = (uint32_t)(lane + 64 * j);
        key_take(oc, R.cp_seq.v[j], (K_COMPLETE << 28) | code, k, s, c);
        key_take(ow, R.wh_seq.v[j], (K_ARRIVE << 28) | code, k, s, c);
    }
    const uint32_t kmin = wave_umin_fast(k);
    if (kmin != 0xffffffffu) {
        bt = H.now + (int64_t)kmin;
        const bool tie = (k == kmin);
        const uint64_t tied = __ballot(tie);
        uint32_t win;
        if (__builtin_popcountll(tied) == 1) {
            win = (uint32_t)__builtin_ctzll(tied);
        } else {                                                    // same-ns events: ns-3 uid order
            const uint32_t smin = wave_umin_fast(tie ? s : 0xffffffffu);
            win = (uint32_t)__builtin_ctzll(__ballot(tie && s == smin));
        }
        bc = rdl(c, win);
        bs = rdl(s, win);
        return;
    }
    // every source is >= 2^32-1 ns away (or none is pending): exact 64-bit path
    int64_t t = INT64_MAX;
    uint32_t s2 = 0xffffffffu, c2 = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < FS; ++j) {
        int64_t tj = mk64(R.fk_lo.v[j], R.fk_hi.v[j]);
        uint32_t sj = R.fk_seq.v[j];
        if (key_less(tj, sj, t, s2)) { t = tj; s2 = sj; c2 = (K_FLOW << 28) | (uint32_t)(lane + 64 * j); }
    }
    if (lane == 0 && key_less(H.ping_t, H.ping_seq, t, s2)) { t = H.ping_t; s2 = H.ping_seq; c2 = K_PING << 28; }
    bt = wave_min_i64(t);
    const bool tie = (t == bt);
    const uint64_t tied = __ballot(tie);
    uint32_t win;
    if ((tied & (tied - 1)) == 0) {
        win = (uint32_t)__builtin_ctzll(tied);
    } else {
        const uint32_t smin = wave_umin_fast(tie ? s2 : 0xffffffffu);
        win = (uint32_t)__builtin_ctzll(__ballot(tie && s2 == smin));
    }
    bc = rdl(c2, win);
    bs = rdl(s2, win);
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// the [N][N] action table (table policy) sits in LDS after the state image, or in HBM
__device__ __forceinline__ int table_action(const Sim& S, uint32_t i) {
    return (int)rfl(S.tab_lds ? (uint32_t)S.table[i] : (uint32_t)S.table_g[i]);
}

__device__ __forceinline__ void stage_table(unsigned char* lds, const KParams& P, int lane) {
    CLayout& LC = *(CLayout*)P.lay;
    if (P.table && LC.table_in_lds) {
        uint8_t* dstp = lds + LC.lds_state_bytes;
        const uint32_t nt = (uint32_t)(LC.N * LC.N);
        for (uint32_t i = (uint32_t)lane; i < nt; i += kWave) dstp[i] = P.table[i];
    }
}

template <int FS, int LS>
__device__ __forceinline__ void stage_in(unsigned char* lds, const KParams& P, int r, int lane, Regs<FS, LS>& R) {
    CLayout& LC = *(CLayout*)P.lay;
    stage_table(lds, P, lane);
    const unsigned char* img = P.state + (size_t)r * LC.state_bytes;
    const uint4* s4 = (const uint4*)img;
    uint4* d4 = (uint4*)lds;
    for (uint32_t i = (uint32_t)lane; i < LC.lds_state_bytes / 16u; i += kWave) d4[i] = s4[i];
    regs_io(R, (uint32_t*)(const_cast<unsigned char*>(img) + LC.s_regs), lane, false);
}

template <int FS, int LS>
__device__ __forceinline__ void stage_out(unsigned char* lds, const KParams& P, int r, int lane, Regs<FS, LS>& R) {
    CLayout& LC = *(CLayout*)P.lay;
    unsigned char* img = P.state + (size_t)r * LC.state_bytes;
    uint4* s4 = (uint4*)img;
    const uint4* d4 = (const uint4*)lds;
    for (uint32_t i = (uint32_t)lane; i < LC.lds_state_bytes / 16u; i += kWave) s4[i] = d4[i];
    regs_io(R, (uint32_t*)(img + LC.s_regs), lane, true);
}

__device__ __forceinline__ void publish_counters(const Sim& S, const KParams& P, int r, int lane) {
    const uint32_t* src = (const uint32_t*)S.c;
    uint32_t* dst = (uint32_t*)(P.cnt_out + r);
    if (lane < (int)(sizeof(prisma_counters_t) / 4)) dst[lane] = src[lane];
}

// ---------------------------------------------------------------------------
// Episode boundaries inside a fused launch (prisma_run with auto_reset, register-resident
// engine): main.py:111-114 runs the episodes back to back, so a replica whose episode ends
// (Simulator::Stop at simTime, sim.cc:703) with hop budget left starts its next episode in the
// same launch and spends the rest of its budget there.  The next episode's fresh image (LDS
// part + register part) is built ahead of time by the reset kernel into P.spare, so the restart
// is a copy: the LDS image and the registers are reloaded from it, and the log position and
// the running totals carried over.  The step kernel then runs a second inlined copy of the
// event loop (step_kernel.h).  Restarting inside the first loop instead -- its clock and
// sequence numbers then get a second incoming value -- cost the hot loop ~20 VGPRs and 13 %
// (A/B, profiles/r03a); so did Philox draws in the loop, an outer loop around it or an
// out-of-line call (scripts/asm_headline.sh: 24-60 VGPR spills).  Without a valid spare (a
// second episode end in one launch) the replica stops at the end and the reset kernel after
// the launch starts its next episode.
// ---------------------------------------------------------------------------
template <int FS, int LS>
__device__ __forceinline__ bool spare_restart(const KParams& P, Sim& S, Regs<FS, LS>& R, int r, uint32_t done,
                                              uint32_t& budget) {
    CLayout& LC = *(CLayout*)P.lay;
    if (!P.spare || !LC.auto_reset || (P.mode != 2 && P.mode != 4) || done >= budget) return false;
    if (!u_ld32(&S.h->over) || u_ld32(&S.h->error)) return false;
    const unsigned char* sp = P.spare + (size_t)r * LC.state_bytes;
    if (rfl(((const Hdr*)(sp + kOffHdr))->episode) != u_ld32(&S.h->episode) + 1u) return false;
    const int lane = S.lane;
    // carried over: the log position and the running totals (hot_store has added this launch's)
    const uint32_t dec = u_ld32(&S.h->dec_count);
    const uint64_t ht = (uint64_t)u_ld64((const int64_t*)&S.h->hops_total);
    const uint64_t et = (uint64_t)u_ld64((const int64_t*)&S.h->events_total);
    __syncthreads();
    const uint4* s4 = (const uint4*)sp;
    uint4* d4 = (uint4*)S.base;
    for (uint32_t i = (uint32_t)lane; i < LC.lds_state_bytes / 16u; i += kWave) d4[i] = s4[i];
    regs_io(R, (uint32_t*)(const_cast<unsigned char*>(sp) + LC.s_regs), lane, false);
    __syncthreads();
    if (lane == 0) {
        S.h->dec_count = dec; S.h->hops_total = ht; S.h->events_total = et;
        S.c->dec_count = dec; S.c->hops_total = ht; S.c->events_total = et;
    }
    __syncthreads();
    budget -= done;
    return true;
}
template <class RS>
__device__ __forceinline__ bool spare_restart(const KParams&, Sim&, RS&, int, uint32_t, uint32_t&) { return false; }

// ---------------------------------------------------------------------------
// the event loop of one launch (both engines): finish the pending decision,
// then one discrete event per iteration until max_hops hops, a decision that
// needs an external action, or the end of the episode; publish the outputs.
// ---------------------------------------------------------------------------
template <bool MLP, int MB, class RS>
__device__ __forceinline__ uint32_t event_loop(const KParams& P, Sim& S, RS& R, int r, uint32_t max_hops) {
    const int lane = S.lane;
    const LV& L = S.lv;
    const bool mlp_mode = MLP;
    S.mlp_inst = MLP;
    const bool table_mode = (P.mode == 2) || mlp_mode;            // fused in-kernel policy
    S.mlp = P.mlp;
    S.mlp_rp = P.mlp_rp;
    S.table_g = P.table;
    S.tab_lds = S.tab_lds && ((CLayout*)P.lay)->table_in_lds != 0u;
    const uint32_t NN = (uint32_t)L.N();
    Hot H;
    hot_load(S, H);
    flow_min_refresh(S, R, H);

    H.stop = 0;
    H.hops_launch = 0;
    if (PRISMA_PRIO && S.prio_total) prio_update(S, 0u);
    if (H.pend && !H.over) {
        if (table_mode) {
            uint32_t pn = u_ld32(&S.h->pend_node), pd = u_ld32(&S.h->pend_ent[1]);
            MlpPre1 M0;
            const int a = mlp_mode ? mlp_action<MB>(S, pn, (lane < L.W()) ? S.obs[lane] : 0u, M0)
                                   : table_action(S, pn * NN + pd);
            H.hops_launch += finish_pending(S, R, H, a);
        } else if (P.actions) {
            finish_pending(S, R, H, (int)rfl((uint32_t)P.actions[r]));
        } else {
            H.stop = 1;                                // nothing to apply: re-emit the pending obs
        }
    }
    if (H.over || (table_mode && H.hops_launch >= max_hops)) H.stop = 1;

    // Drain the stage-in loads here: otherwise the waitcnt pass keeps them
    // "possibly pending" at the loop header and emits vmcnt waits there that,
    // on every later iteration, also wait for the previous event's record
    // stores.
    __builtin_amdgcn_s_waitcnt(0);
#if PRISMA_TIMING
    uint64_t tm_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t tm_cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tm_a = 0, tm_b = 0;
    S.tsub[0] = 0; S.tsub[1] = 0; S.tlast = 0;
    S.tmlp[0] = 0; S.tmlp[1] = 0; S.tmlp[2] = 0; S.tmlp[3] = 0;
    S.tflow[0] = 0; S.tflow[1] = 0; S.tflow[2] = 0; S.tflow[3] = 0; S.tfl = 0;
    for (int i = 0; i < 16; ++i) { S.tp[i] = 0; S.tpn[i] = 0; }
    S.tpl = 0;
#define TM_MARK(i) do { tm_b = TM_NOW(); tm_acc[i] += tm_b - tm_a; tm_cnt[i]++; tm_a = tm_b; } while (0)
#else
#define TM_MARK(i) do { } while (0)
#endif
    constexpr bool kPre = MLP && RS::kMem;               // memory-resident engine + MLP: weights prefetched
    while (!H.stop) {
        int64_t bt;
        uint32_t bc, bs;
#if PRISMA_TIMING
        tm_a = TM_NOW();
#endif
        select_event(S, R, H, lane, bt, bc, bs);
        if (bt >= L.t_end()) {                           // Simulator::Stop(simTime) (sim.cc:703)
            lazy_resolve(S, R, H, true);                 // here, not after the loop: there it costs registers
            H.over = 1;
            H.stop = 1;
            break;
        }
        H.now = bt;
        H.cur_seq = bs;
#if PRISMA_TRACE
        if (lane == 0 && r < 8 && g_prisma_trace) {
            const unsigned int i = g_prisma_trace_n[r]++;
            if (i < g_prisma_trace_cap) {
                long long* q = g_prisma_trace + ((size_t)r * g_prisma_trace_cap + i) * 3;
                q[0] = bt; q[1] = bc >> 28; q[2] = bc & 0x0fffffffu;
            }
        }
#endif
        H.ev_launch++;                                   // added to the events counter at exit
        const uint32_t kind = bc >> 28, id = bc & 0x0fffffffu;
        TM_MARK(0);
        if (kind == K_ARRIVE) {
            Decision D;
            D.r0 = -1; D.deg = 0;
            MlpPre1 Mp;                                  // (kPre) the decision's first weights, fetched on arrival
            const int need = on_arrive<kPre>(S, R, H, id, D, table_mode, Mp);
            TM_MARK(1);
            if (need) {
                if (table_mode) {
                    const int a = mlp_mode ? mlp_action<MB, kPre>(S, D.v, D.obs, Mp)
                                           : table_action(S, D.v * NN + D.dst);
                    // (the row handoff: headline +2.1 % in A/B; config 4's MLP instance -2 %, so
                    // the MLP instances read the row again)
                    apply_decision<!RS::kMem && !MLP>(S, R, H, D.x, D.dst, D.start, D.uid, D.v, D.d, a, true,
                                   D.reward, D.prev, D.obs,
                                   (D.flags & PEND_ECHO) ? (uint32_t)t_lrev(S, id) : kNoLink, D.last, D.ttl,
                                   D.r0, D.deg);
                    H.hops_launch++;
                    if (H.hops_launch >= max_hops) H.stop = 1;
                    if (PRISMA_PRIO && H.hops_launch == S.prio_next) prio_update(S, H.hops_launch);
                    TM_MARK(2);
                } else {
                    if (lane == 0) {
                        Hdr& h = *S.h;
                        h.pend_link = id; h.pend_node = D.v; h.pend_dec = D.d;
                        h.pend_ent[0] = D.x; h.pend_ent[1] = D.dst; h.pend_ent[2] = D.start; h.pend_ent[3] = D.flags;
                        h.pend_uid = D.uid; h.pend_last = D.last;
                    }
                    if (lane < L.W()) S.obs[lane] = D.obs;
                    H.pend = 1;
                    H.stop = 1;
                }
            }
        } else if (kind == K_COMPLETE) {
            on_complete(S, R, H, id);
            TM_MARK(3);
        } else if (kind == K_FLOW) {
            on_flow(S, R, H, id);
            TM_MARK(4);
        } else {
            on_ping_round(S, R, H);
            TM_MARK(5);
        }
        if (H.error) { H.over = 1; H.stop = 1; }
        if (!MLP) {
            // the loop's exit flags as provably uniform values: the loop then exits with a
            // scalar branch instead of exec-mask bookkeeping (A/B: table instances +0.6 %, the
            // MLP instances -1 %, so only the former)
            H.stop = rfl(H.stop); H.over = rfl(H.over); H.error = rfl(H.error);
        }
    }
#if PRISMA_TIMING
    tm_acc[6] = S.tsub[0]; tm_acc[7] = S.tsub[1];
    if (lane == 0) {
        for (int i = 0; i < 8; ++i) {
            atomicAdd(&g_prisma_timing[i], (unsigned long long)tm_acc[i]);
            atomicAdd(&g_prisma_timing[8 + i], (unsigned long long)tm_cnt[i]);
        }
        for (int i = 0; i < 4; ++i) atomicAdd(&g_prisma_timing[16 + i], (unsigned long long)S.tmlp[i]);
        for (int i = 0; i < 4; ++i) atomicAdd(&g_prisma_timing[20 + i], (unsigned long long)S.tflow[i]);
        for (int i = 0; i < 16; ++i) {
            atomicAdd(&g_prisma_timing[24 + i], (unsigned long long)S.tp[i]);
            atomicAdd(&g_prisma_timing[40 + i], (unsigned long long)S.tpn[i]);
        }
    }
#endif
    if (!H.error) lazy_resolve(S, R, H, false);      // elided completions up to where the launch stopped

    hot_store(S, R, H);
    __syncthreads();
    const bool pending = H.pend && !H.over;
    if (P.mask_out && lane == 0) P.mask_out[r] = pending ? 1 : 0;
    if (P.node_out && lane == 0) P.node_out[r] = pending ? (int32_t)S.h->pend_node : -1;
    if (P.obs_out && lane < L.W()) P.obs_out[(size_t)r * L.W() + lane] = pending ? (int32_t)S.obs[lane] : 0;
    publish_counters(S, P, r, lane);
    return H.hops_launch;
}
