// prisma_engine.hip — MI355X (gfx950) packet-hop engine behind include/prisma.h.
//
// Design: one 64-lane wavefront (= one workgroup) owns one
// topology replica of PRISMA's ns-3 scenario and runs its discrete-event
// loop for a whole launch.
//   * Link and flow state is lane-distributed in VGPRs: link l lives in lane
//     l % 64, register slot l / 64 (likewise flows).  Every lane keeps the
//     next-event key (time, seq) of the sources it owns, so choosing the next
//     event is a register-only per-lane min plus a DPP wave reduction (the
//     ns-3 MapScheduler (time, uid) order) — no LDS, no barrier.
//   * The selected handler runs as uniform code on all lanes: scalars live in
//     SGPRs, a link's fields are read with v_readlane and written back with
//     v_writelane into the owning lane.
//   * Packet FIFOs (per-link rings of 16-B entries), wire arrival times and the
//     ping windows live in LDS; the replica image is staged HBM -> LDS/VGPR at
//     launch and written back at exit (16-B coalesced).
//   * Every data notification appends a 32+4W-byte decision record to the
//     replica's HBM log with one coalesced wave store.
// Results are bit-identical to the CPU oracle (oracle/), the independent
// restatement of the reference ns-3 semantics.
//
// Compile: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <new>
#include <string>
#include <vector>

#include "../../include/prisma.h"
#include "engine_layout.h"
#include "numerics.h"

using namespace prisma;

#define HIP_OK(x) ((x) == hipSuccess)

// Diagnostic timing builds only (scripts/ablate.sh; results are NOT the
// reference's): bit 0 skips the previous-record read (relay entries carry
// dst/start), bit 1 skips the decision-record stores, bit 2 skips observe().
#ifndef PRISMA_ABLATE
#define PRISMA_ABLATE 0
#endif
// Diagnostic timing build (-DPRISMA_TIMING=1, scripts/timing.py): s_memtime
// cycle totals per loop phase, summed over waves into g_prisma_timing.
#ifndef PRISMA_TIMING
#define PRISMA_TIMING 0
#endif
#if PRISMA_TIMING
__device__ unsigned long long g_prisma_timing[16];
#define TM_NOW() ((uint64_t)__builtin_amdgcn_s_memtime())
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
    int32_t R;
    int32_t max_hops;
    uint32_t episode;            // reset kernel only
    int32_t mode;                // 0 reset, 1 external step, 2 table run
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
    // t = now + (uint32)(t_lo - lo32(now))
    LA<LS> lk_t, lk_seq, lk_kind;                // link next event key: kind 0 none / K_COMPLETE / K_ARRIVE
    LA<LS> cp_t, cp_seq;                         // tx completion event (valid while busy)
    LA<LS> wh_t, wh_seq;                         // arrival event of the wire head (valid while n_wire > 0)
    LA<LS> p0, p1, p2, qb;                       // head|txp<<16, tail|n_wire<<16, n_queue|busy<<16, queued bytes
    // per TUNNEL t (lane t % 64, slot t / 64; tunnel == link on identity overlays):
    LA<LS> pm_lo, pm_mlo, pm_mhi;                // ping: oldest unacked round, acked bits of rounds lo+1..lo+64
    LA<LS> pm_win;                               // win_n | win_head << 16 | saturated << 31
    LA<LS> pav_lo, pav_hi;                       // ping window mean (double), refreshed per ping-back
    LA<LS> od_lo, od_hi;                         // send time (s) of round lo
    static constexpr int NF = 4, NL = 19;
};

template <int FS, int LS>
__device__ __forceinline__ void regs_io(Regs<FS, LS>& R, uint32_t* img, int lane, bool store) {
    uint32_t* fb = img;
    uint32_t* lb = img + 4 * 64 * FS;
#define RIO_F(fld, a) if (store) R.fld.store(fb + (a) * 64 * FS, lane); else R.fld.load(fb + (a) * 64 * FS, lane);
#define RIO_L(fld, a) if (store) R.fld.store(lb + (a) * 64 * LS, lane); else R.fld.load(lb + (a) * 64 * LS, lane);
    RIO_F(fk_lo, 0) RIO_F(fk_hi, 1) RIO_F(fk_seq, 2) RIO_F(f_draw, 3)
    RIO_L(lk_t, 0) RIO_L(wh_t, 1) RIO_L(lk_seq, 2) RIO_L(lk_kind, 3) RIO_L(cp_t, 4) RIO_L(wh_seq, 5)
    RIO_L(cp_seq, 6) RIO_L(p0, 7) RIO_L(p1, 8) RIO_L(p2, 9) RIO_L(qb, 10) RIO_L(pm_lo, 11)
    RIO_L(pm_mlo, 12) RIO_L(pm_mhi, 13) RIO_L(pm_win, 14) RIO_L(pav_lo, 15) RIO_L(pav_hi, 16)
    RIO_L(od_lo, 17) RIO_L(od_hi, 18)
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
static_assert(sizeof(Layout) <= 4 * kWave, "Layout must fit one VGPR");
struct LV {
    uint32_t w;
    __device__ __forceinline__ void load(const Layout* lay, int lane) {
        w = (lane < (int)(sizeof(Layout) / 4)) ? ((const uint32_t*)lay)[lane] : 0u;
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
    __device__ __forceinline__ uint32_t table_bytes() const { return (uint32_t)u(offsetof(Layout, table_bytes) / 4); }
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
};


// LDS views of one replica + its topology
struct Sim {
    LV lv;                                  // scenario constants (one VGPR)
    unsigned char* base;
    Hdr* h;
    prisma_counters_t* c;
    uint32_t* obs;
    uint32_t* wt; uint32_t* wseq;           // wire: arrival time (low 32 bits) and seq
    uint32_t* ring;
    float* win;
    float* pbd;                             // ping-back delays [responder slot][PBK]
    const CAS TopoImage* T;                 // topology (scalar loads at fixed offsets)
    const uint8_t* table;
    const float* mlp;                       // DQN-buffer weights (HBM) or null
    float* hbuf;                            // 64 floats of LDS: a layer's activations
    unsigned char* logrep;
    uint32_t gid;
    int lane;
    bool tun;                               // tunnelled overlay: a compile-time constant in the
                                            // step kernels (template TUN), folded after inlining
#if PRISMA_TIMING
    mutable uint64_t tsub[2], tlast;             // sub-phase cycles inside apply_decision
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
    S.ring = (uint32_t*)(lds + L.s_ring());
    S.win = (float*)(lds + L.s_win());
    S.pbd = (float*)(lds + L.s_pbd());
    S.T = (const CAS TopoImage*)topo;
    S.table = (const uint8_t*)(lds + L.lds_state_bytes());
    S.hbuf = (float*)(lds + L.s_mlp());
    S.mlp = nullptr;
    S.logrep = logrep;
    S.gid = gid;
    S.lane = lane;
    S.tun = L.tunnels() != 0u;
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
}

template <int FS, int LS>
__device__ inline void hot_store(Sim& S, const Regs<FS, LS>& R, const Hot& H) {
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

__device__ __forceinline__ uint32_t ent_size(const LV& L, uint32_t x) {
    return ent_is_data(x) ? L.data_size() : (ent_is_echo(x) ? L.echo_size() : L.ping_size());
}
// FIFO ring of link l: uniform capacities on identity overlays, per-link (sized by the
// control traffic crossing each link) on tunnelled ones
__device__ __forceinline__ uint32_t ring_off(const Sim& S, uint32_t l) {
    const LV& L = S.lv;
    if (S.tun) return S.T->rinfo[l] & 0xffffu;
    return l < (uint32_t)L.E() ? l * L.qcap_s() : (uint32_t)L.E() * L.qcap_s() + (l - (uint32_t)L.E()) * L.qcap_a();
}
__device__ __forceinline__ uint32_t ring_cap(const Sim& S, uint32_t l) {
    const LV& L = S.lv;
    if (S.tun) return S.T->rinfo[l] >> 16;
    return l < (uint32_t)L.E() ? L.qcap_s() : L.qcap_a();
}

// one link's fields as uniform scalars
struct LinkV {
    uint32_t head, txp, tail, n_wire, n_queue, busy, qb;
    uint32_t cp_t, cp_seq;       // completion time (low 32 bits), seq
    uint32_t wh_t, wh_seq;       // wire-head arrival time (low 32 bits), seq
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
template <int FS, int LS>
__device__ __forceinline__ void link_put(const Sim& S, Regs<FS, LS>& R, const Hot& H, uint32_t l, const LinkV& k) {
    R.p0.set(l, k.head | (k.txp << 16));
    R.p1.set(l, k.tail | (k.n_wire << 16));
    R.p2.set(l, k.n_queue | (k.busy << 16));
    R.qb.set(l, k.qb);
    R.cp_t.set(l, k.cp_t);
    R.cp_seq.set(l, k.cp_seq);
    R.wh_t.set(l, k.wh_t);
    R.wh_seq.set(l, k.wh_seq);
    const uint32_t n0 = lo32(H.now);
    uint32_t t = 0, s = 0xffffffffu, kind = 0;
    if (k.busy) { t = k.cp_t; s = k.cp_seq; kind = K_COMPLETE; }
    if (k.n_wire) {
        const uint32_t rw = k.wh_t - n0, rt = t - n0;
        if (kind == 0 || rw < rt || (rw == rt && k.wh_seq < s)) { t = k.wh_t; s = k.wh_seq; kind = K_ARRIVE; }
    }
    R.lk_t.set(l, t);
    R.lk_seq.set(l, s);
    R.lk_kind.set(l, kind);
}

// ---- link FIFO / transmitter (point-to-point-net-device.cc:273-336, 595-666)
__device__ __forceinline__ void transmit_start(const Sim& S, Hot& H, uint32_t l, LinkV& k, uint32_t ring_idx,
                                               uint32_t x) {
    const LV& L = S.lv;
    const bool sw = l < (uint32_t)L.E();
    int64_t tx = sw ? (ent_is_data(x) ? L.sw_txd() : (ent_is_echo(x) ? L.sw_txe() : L.sw_txp()))
                    : S.T->acctx[l - (uint32_t)L.E()];
    int64_t prop = sw ? L.sw_prop() : 0;
    k.busy = 1;
    k.cp_t = lo32(H.now + tx);
    k.cp_seq = H.seq++;                                        // TransmitComplete
    uint32_t w = l * (uint32_t)L.WCAP() + (ring_idx & (uint32_t)(L.WCAP() - 1));
    const uint32_t at = lo32(H.now + tx + prop);
    const uint32_t as = H.seq++;                               // channel Receive
    if (S.lane == 0) { S.wt[w] = at; S.wseq[w] = as; }
    if (k.n_wire == 1) { k.wh_t = at; k.wh_seq = as; }        // the wire was empty: new head
    if (k.n_wire > (uint32_t)L.WCAP()) fail(H, PRISMA_EBIT_WIRE);
}

// returns 1 if enqueued, 0 if dropped (a ring overflow fails the replica)
template <int FS, int LS>
__device__ __forceinline__ int link_send(const Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t l, uint32_t e) {
    const LV& L = S.lv;
    LinkV k = link_get(R, l);
    uint32_t size = ent_size(L, e);
    bool ok = l < (uint32_t)L.E() ? (k.qb + size <= L.qmax_bytes()) : (k.n_queue + 1u <= L.acc_qmax_pkts());
    if (!ok) return 0;
    uint32_t cap = ring_cap(S, l), off = ring_off(S, l);
    if (k.n_wire + k.n_queue + 1u > cap) { fail(H, PRISMA_EBIT_RING); return 0; }
    if (S.lane == 0) S.ring[off + k.tail] = e;
    k.tail = (k.tail + 1 == cap) ? 0 : k.tail + 1;
    k.n_queue++;
    k.qb += size;
    if (!k.busy) {                                              // :643-650
        uint32_t xi = k.txp;
        uint32_t hx = (k.n_queue == 1) ? e : u_ld32(&S.ring[off + xi]);
        k.txp = (xi + 1 == cap) ? 0 : xi + 1;
        k.n_queue--;
        k.n_wire++;
        k.qb -= ent_size(L, hx);
        transmit_start(S, H, l, k, xi, hx);
    }
    link_put(S, R, H, l, k);
    return 1;
}

template <int FS, int LS>
__device__ __forceinline__ void on_complete(const Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t l) {   // :305-336
    const LV& L = S.lv;
    LinkV k = link_get(R, l);
    k.busy = 0;
    if (k.n_queue) {
        uint32_t cap = ring_cap(S, l);
        uint32_t xi = k.txp;
        uint32_t hx = u_ld32(&S.ring[ring_off(S, l) + xi]);
        k.txp = (xi + 1 == cap) ? 0 : xi + 1;
        k.n_queue--;
        k.n_wire++;
        k.qb -= ent_size(L, hx);
        transmit_start(S, H, l, k, xi, hx);
    }
    link_put(S, R, H, l, k);
}

// ---- observation (data-packet-manager.cc:171-206)
// send time in seconds of ping round k as the ping-back manager stores it:
// (double)GetMilliSeconds() * 0.001 (ping-back-packet-manager.cc:98-116)
__device__ __forceinline__ double ping_send_s(const LV& L, int64_t k) {
    uint64_t ms = (uint64_t)(((k + 1) * L.ping_period()) / 1000000);
    return (double)ms * 0.001;
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
template <int FS, int LS>
__device__ __forceinline__ uint32_t observe_links(const Sim& S, const Regs<FS, LS>& R, const Hot& H, uint32_t v,
                                                  double now_s) {
    if (PRISMA_ABLATE & 4) return 0u;
    const int r0 = S.T->ovrow[v], deg = S.T->ovrow[v + 1] - r0;
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
        if (pobs)
            val = ping_value_lane(ld_d(R.pav_lo.v[j], R.pav_hi.v[j]), R.pm_lo.v[j], ld_d(R.od_lo.v[j], R.od_hi.v[j]),
                                  H.ping_rounds, now_s);
        else
            val = R.qb.v[j];
        const uint32_t g = (uint32_t)__shfl((int)val, (int)(src & 63u));
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
    uint32_t hw;
    switch (lane) {
    case 0: hw = lo32(H.now); break;
    case 1: hw = hi32(H.now); break;
    case 2: hw = uid; break;
    case 3: hw = (uint32_t)prev; break;
    case 4: hw = (uint32_t)rb; break;
    case 5: hw = (uint32_t)(rb >> 32); break;
    case 6: hw = node | (dst << 8) | (start << 16); break;
    default: hw = w7; break;
    }
    uint32_t ob = (uint32_t)__shfl((int)obs_reg, (lane - 8) & 63);
    uint32_t word = lane < 8 ? hw : ob;
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
template <int FS, int LS>
__device__ __forceinline__ void receive_counters(const Sim& S, Regs<FS, LS>& R, const Hot& H, uint32_t x, bool arrived,
                                                 uint32_t start) {
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
    if (!ent_is_data(x)) CNT_ADD(S, bytes_signaling, ent_size(L, x) - 2u);
    if (ent_type(x) == T_FRESH) {
        CNT_ADD(S, ov_injected, 1u);
        CNT_ADD(S, bytes_data, L.data_size() - 2u);
    }
}

constexpr uint32_t kNoLink = 0xffffffffu;

// source node of a data entry (MyTag source)
__device__ __forceinline__ uint32_t ent_src(const Sim& S, uint32_t x) {
    return ent_type(x) == T_FRESH ? (uint32_t)S.T->fsrc[f_flow(x)] : r_src(x);
}

// DataPacketManager::sendSmallSignalingPacket (data-packet-manager.cc:301-347): a 0-B
// payload (30 B on the wire, signalling type "ideal") back on the arrival device,
// addressed to the data packet's last hop `to`
template <int FS, int LS>
__device__ __forceinline__ void send_echo(const Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t link, uint32_t uid,
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

// DataPacketManager::sendPacket (data-packet-manager.cc:251-299) for decision
// d at node v, then the Receive tail.  x is the arriving entry (for the
// counters); fused: the record is written here once, with the final status
// (table policy).
template <int FS, int LS>
__device__ __forceinline__ void apply_decision(const Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t x, uint32_t dst,
                                               uint32_t start, uint32_t uid, uint32_t v, uint32_t d, int action,
                                               bool fused, double reward, int32_t prev, uint32_t obs_reg,
                                               uint32_t echo_link, uint32_t last, uint32_t ttl) {
    const LV& L = S.lv;
#if PRISMA_TIMING
    S.tlast = TM_NOW();
#endif
    // ExecuteActions (packet-routing-gym.cc:203-208): the --train echo goes first
    if (echo_link != kNoLink) send_echo(S, R, H, echo_link, uid, last);
    int r0 = S.T->ovrow[v], deg = S.T->ovrow[v + 1] - r0;
    uint32_t status;
    if (action >= 0 && action < deg) {
        const uint32_t l = tunnel_link(S, (uint32_t)(r0 + action));   // RouteOutput (:281-287)
        CNT_ADD(S, hops, 1u);
        CNT_ADD(S, hop_deg_sum, (uint64_t)deg);
        const uint32_t src = ent_src(S, x);
        const uint32_t fwd = (PRISMA_ABLATE & 1) ? (T_RELAY | (dst << 2) | (start << 10) | (src << 24)) : r_make(d, src);
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
    if (fused) write_record(S, H, d, reward, uid, prev, v, dst, start, action, status, obs_reg, ttl);
    else patch_record(S, H, d, action, status);
    receive_counters(S, R, H, x, false, 0u);
#if PRISMA_TIMING
    { const uint64_t t = TM_NOW(); S.tsub[1] += t - S.tlast; S.tlast = t; }
#endif
}

// Answer to the pending notification.  Returns 1 if a hop was executed (0 for a
// destination or control notification, whose action is ignored: sendPacket at
// the destination does nothing (:256-260), ExecuteActions sends nothing for a
// small-signalling packet).
template <int FS, int LS>
__device__ __forceinline__ int finish_pending(const Sim& S, Regs<FS, LS>& R, Hot& H, int action) {
    const Hdr& h = *S.h;
    H.pend = 0;
    const uint32_t x = u_ld32(&h.pend_ent[0]), flags = u_ld32(&h.pend_ent[3]);
    if (flags & PEND_CTRL) {
        receive_counters(S, R, H, x, false, 0u);
        return 0;
    }
    const uint32_t echo_link = (flags & PEND_ECHO) ? (uint32_t)S.T->lrev[u_ld32(&h.pend_link)] : kNoLink;
    const uint32_t last = u_ld32(&h.pend_last);
    if (flags & PEND_DEST) {
        if (echo_link != kNoLink) send_echo(S, R, H, echo_link, u_ld32(&h.pend_uid), last);
        receive_counters(S, R, H, x, true, u_ld32(&h.pend_ent[2]));
        return 0;
    }
    apply_decision(S, R, H, x, 0u, 0u, u_ld32(&h.pend_uid), u_ld32(&h.pend_node), u_ld32(&h.pend_dec), action,
                   false, 0.0, 0, 0u, echo_link, last, 0u);
    return 1;
}

// ---- handlers (uniform) ------------------------------------------------------
template <int FS, int LS>
__device__ __forceinline__ void on_ping_round(const Sim& S, Regs<FS, LS>& R, Hot& H) {   // data-packet-manager.cc:350-413
    const LV& L = S.lv;
    uint32_t k = H.ping_rounds;
    uint32_t first_rearm = 0;
    for (int i = 0; i < L.NO(); ++i) {                            // timers in overlay order (sim.cc:528-546)
        const int u = S.tun ? S.T->ovnode[i] : i;
        const int r0 = S.T->ovrow[u], r1 = S.T->ovrow[u + 1];
        for (int t = r0; t < r1; ++t) {
            if (!link_send(S, R, H, tunnel_link(S, (uint32_t)t), p_make(T_PFWD, (uint32_t)t, 0u, k)))
                CNT_ADD(S, ctrl_dropped, 1u);
        }
        uint32_t s = H.seq++;                                    // re-arm of node u
        if (i == 0) first_rearm = s;
    }
    H.ping_rounds = k + 1;
    // one ns-3 event per overlay node timer (the round is NO consecutive events)
    CNT_ADD(S, events, (uint64_t)(L.NO() - 1));
    H.ev_launch += (uint32_t)(L.NO() - 1);
    H.ping_t = H.now + L.ping_period();
    H.ping_seq = first_rearm;
}

template <int FS, int LS>
__device__ __forceinline__ void flow_next(const Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t f, uint32_t draw) {
    uint32_t c[4] = { f, draw, H.episode, 1u };                   // poisson-application.cc:265-295
    philox4x32_10(c, S.lv.seed_lo(), S.gid);
    uint64_t u53 = ((uint64_t)(c[0] >> 5) << 26) | (uint64_t)(c[1] >> 6);
    double U = ((double)u53 + 1.0) * (1.0 / 9007199254740992.0);
    double delay = -S.T->fmean[f] * det_log(U);
    int64_t t = H.now + sec_to_ns(delay);
    R.fk_lo.set(f, lo32(t));
    R.fk_hi.set(f, hi32(t));
    R.fk_seq.set(f, H.seq++);
    R.f_draw.set(f, draw + 1);
}

template <int FS, int LS>
__device__ __forceinline__ void on_flow(const Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t f) {
    uint32_t draw = R.f_draw.get(f);
    if (draw != 0) {                                                // SendPacket :297-358
        uint32_t src = (uint32_t)S.T->fsrc[f];
        uint32_t par = (uint32_t)(H.now / 1000000000) & 1u;         // start second (its parity)
        link_send(S, R, H, (uint32_t)S.lv.E() + src, f_make(f, par, H.uid & kUidMask));   // access link
        H.uid++;
    }
    flow_next(S, R, H, f, draw);                                    // StartSending / ScheduleNextTx
}

// ---- in-kernel DQN_buffer_model (models.py:258-306; fixed fp32 operation order,
// DESIGN.md §2, restated by the oracle's mlp_action): lane j computes unit j of
// each layer, activations are broadcast through 64 floats of LDS, weights are
// read per lane from HBM (L2-resident, shared by every replica).
__device__ __forceinline__ float hb_ld(const Sim& S, int i) { return S.hbuf[i]; }

__device__ __forceinline__ float mlp_dense64(const Sim& S, const float* __restrict__ W, int lane, int stride) {
    float acc = 0.0f;
#pragma unroll 16
    for (int i = 0; i < 64; ++i) acc = __builtin_fmaf(hb_ld(S, i), W[i * stride + lane], acc);
    return acc;
}

// one-hot input: obs[0] (the destination's overlay index, lane 0 of obs_reg)
__device__ __forceinline__ int mlp_action(const Sim& S, uint32_t v, uint32_t obs_reg) {
    const LV& L = S.lv;
    const int lane = S.lane;
    const int N = L.N(), D = L.max_deg();
    const float* __restrict__ W1 = S.mlp;
    const float* __restrict__ b1 = W1 + N * N * 32;
    const float* __restrict__ Wb = b1 + N * 32;
    const float* __restrict__ bb = Wb + N * D * 32;
    const float* __restrict__ W2 = bb + N * 32;
    const float* __restrict__ b2 = W2 + N * 64 * 64;
    const float* __restrict__ W3 = b2 + N * 64;
    const float* __restrict__ b3 = W3 + N * 64 * 64;
    const float* __restrict__ W4 = b3 + N * 64;
    const float* __restrict__ b4 = W4 + N * 64 * D;
    const int deg = S.T->ovrow[v + 1] - S.T->ovrow[v];
    const uint32_t dst = rdl(obs_reg, 0);
    // LayerNormalization of the deg buffer values (population variance, epsilon 1e-3)
    float sum = 0.0f;
    for (int k = 0; k < deg; ++k) sum = __fadd_rn(sum, (float)rdl(obs_reg, (uint32_t)(k + 1)));
    const float mean = __fdiv_rn(sum, (float)deg);
    float var = 0.0f;
    for (int k = 0; k < deg; ++k) {
        const float d = __fsub_rn((float)rdl(obs_reg, (uint32_t)(k + 1)), mean);
        var = __fadd_rn(var, __fmul_rn(d, d));
    }
    var = __fdiv_rn(var, (float)deg);
    const float den = __fsqrt_rn(__fadd_rn(var, 1e-3f));
    // layer 1: one-hot(dst) branch in lanes 0-31, buffers branch in lanes 32-63
    float h;
    if (lane < 32) {
        h = det_elu(__fadd_rn(W1[((int)v * N + (int)dst) * 32 + lane], b1[(int)v * 32 + lane]));
    } else {
        const int j = lane - 32;
        float acc = 0.0f;
        for (int k = 0; k < deg; ++k) {
            const float xn = __fdiv_rn(__fsub_rn((float)rdl(obs_reg, (uint32_t)(k + 1)), mean), den);
            acc = __builtin_fmaf(xn, Wb[((int)v * D + k) * 32 + j], acc);
        }
        h = det_elu(__fadd_rn(acc, bb[(int)v * 32 + j]));
    }
    S.hbuf[lane] = h;
    __builtin_amdgcn_wave_barrier();
    h = det_elu(__fadd_rn(mlp_dense64(S, W2 + (int)v * 64 * 64, lane, 64), b2[(int)v * 64 + lane]));
    __builtin_amdgcn_wave_barrier();
    S.hbuf[lane] = h;
    __builtin_amdgcn_wave_barrier();
    h = det_elu(__fadd_rn(mlp_dense64(S, W3 + (int)v * 64 * 64, lane, 64), b3[(int)v * 64 + lane]));
    __builtin_amdgcn_wave_barrier();
    S.hbuf[lane] = h;
    __builtin_amdgcn_wave_barrier();
    float q = 0.0f;
    if (lane < deg) q = det_elu(__fadd_rn(mlp_dense64(S, W4 + (int)v * 64 * D, lane, D), b4[(int)v * D + lane]));
    __builtin_amdgcn_wave_barrier();
    // tf.argmin: first minimum (learner.py:145)
    int best = 0;
    float bq = __uint_as_float(rdl(__float_as_uint(q), 0));
    for (int a = 1; a < deg; ++a) {
        const float qa = __uint_as_float(rdl(__float_as_uint(q), (uint32_t)a));
        if (qa < bq) { bq = qa; best = a; }
    }
    return best;
}

// the head packet leaves the wire of link l (arrival at the far end)
template <int FS, int LS>
__device__ __forceinline__ void wire_pop(const Sim& S, Regs<FS, LS>& R, const Hot& H, uint32_t l, LinkV& k) {
    const LV& L = S.lv;
    const uint32_t cap = ring_cap(S, l);
    k.head = (k.head + 1 == cap) ? 0 : k.head + 1;
    k.n_wire--;
    if (k.n_wire) {                                                 // next packet on the wire
        const uint32_t w = l * (uint32_t)L.WCAP() + (k.head & (uint32_t)(L.WCAP() - 1));
        k.wh_t = u_ld32(S.wt + w);
        k.wh_seq = u_ld32(S.wseq + w);
    }
    link_put(S, R, H, l, k);
}

struct Decision {
    uint32_t x, dst, start, uid, v, d; double reward; int32_t prev; uint32_t obs, flags, last, ttl;
};

// a control packet (or a data packet inside a tunnel) continues along the
// underlay route to `to` (Ipv4L3Protocol::IpForward through the patched
// Ipv4Interface::Send, ipv4-interface.cc:213-229)
template <int FS, int LS>
__device__ __forceinline__ void ctrl_forward(const Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t v, uint32_t to,
                                             uint32_t x) {
    if (!link_send(S, R, H, ti_link(route(S, v, to)), x)) CNT_ADD(S, ctrl_dropped, 1u);
}

// PingBackPacketManager::receivePacket (ping-back-packet-manager.cc:120-144) on
// tunnel lt with the one-hop delay the ping-back carries
template <int FS, int LS>
__device__ __forceinline__ void ping_ack(const Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t lt, uint32_t rnd,
                                         float delay) {
    const LV& L = S.lv;
    // the round itself (rounds in flight are less than 2^18 behind the last one sent)
    const uint32_t last = H.ping_rounds - 1u;
    const uint32_t k = last - ((last - rnd) & kRoundMask);
    // erase round k from the unacknowledged list (first match; none if already acked)
    uint32_t lo = R.pm_lo.get(lt);
    uint64_t mask = ((uint64_t)R.pm_mhi.get(lt) << 32) | R.pm_mlo.get(lt);
    uint32_t pw = R.pm_win.get(lt);
    if (k == lo) {
        if (pw >> 31) fail(H, PRISMA_EBIT_ACKORDER);               // acked bits were lost (see below)
        const uint32_t n = (uint32_t)__builtin_ctzll(~mask);       // rounds lo+1.. already acked
        lo += 1u + n;
        mask = (n >= 63u) ? 0ull : (mask >> (n + 1u));
        const uint64_t od = __double_as_longlong(ping_send_s(L, lo));
        R.pm_lo.set(lt, lo);
        R.od_lo.set(lt, (uint32_t)od);
        R.od_hi.set(lt, (uint32_t)(od >> 32));
        R.pm_mlo.set(lt, (uint32_t)mask);
        R.pm_mhi.set(lt, (uint32_t)(mask >> 32));
    } else if (k > lo) {
        const uint32_t b = k - lo - 1u;
        if (b < 64u) {
            mask |= 1ull << b;
            R.pm_mlo.set(lt, (uint32_t)mask);
            R.pm_mhi.set(lt, (uint32_t)(mask >> 32));
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
    R.pm_win.set(lt, wn | (wh << 16) | (pw & (1u << 31)));
    if (S.lane == 0) S.win[lt * MA + slot] = delay;
    // refresh the cached window mean (data-packet-manager.cc:55-65), summed oldest first
    double sum = 0.0;
    uint32_t i = wh;
    for (uint32_t j = 0; j < wn; ++j) {
        float w = (i == slot) ? delay : __uint_as_float(u_ld32((const uint32_t*)S.win + lt * MA + i));
        sum += (double)w;
        i = (i + 1 == MA) ? 0 : i + 1;
    }
    uint64_t avg = __double_as_longlong(sum / (double)wn);
    R.pav_lo.set(lt, (uint32_t)avg);
    R.pav_hi.set(lt, (uint32_t)(avg >> 32));
}

// ping-back delay slot of responder position pos on tunnel t (tunnelled overlays): one
// slot per overlay node on the tunnel
__device__ __forceinline__ uint32_t pbd_slot(const Sim& S, uint32_t t, uint32_t pos) {
    const uint32_t tr = S.T->tresp[t];
    return (tr & 0xffffu) + (uint32_t)__builtin_popcount((tr >> 16) & ((1u << pos) - 1u));
}

// returns 1 if a data decision needs an action
template <int FS, int LS>
__device__ __forceinline__ int on_arrive(const Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t l, Decision& D, bool fused) {
    const LV& L = S.lv;
    LinkV k = link_get(R, l);
    const uint32_t x = u_ld32(&S.ring[ring_off(S, l) + k.head]);
    const uint32_t type = ent_type(x);
    const uint32_t v = (uint32_t)S.T->ldst[l];
    const bool tun = S.tun;
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
        const uint32_t dist = (d - r_dec(x)) & kRelayMask;
        const unsigned char* pr = S.logrep + (size_t)((d - dist) & (L.log_cap() - 1)) * L.rec_bytes();
        const uint4 ph = *(const uint4*)pr;
        const uint2 pw = *(const uint2*)(pr + 24);
        wire_pop(S, R, H, l, k);
        uint32_t ttl = 255u;                                        // SetIpTtl(255) (poisson-application.cc:330)
        if (tun && type == T_RELAY) {
            // Tunnelled overlay: the packet's next hop is the target of the tunnel
            // the previous decision picked; anywhere else it is only IP-forwarded
            // (packet-manager.cc:115 -> not valid, no Notify).
            const uint32_t w6p = rfl(pw.x), w7p = rfl(pw.y);
            const uint32_t u = w6p & 255u;
            const uint32_t ti = S.T->tinfo[(uint32_t)S.T->ovrow[u] + (w7p & 255u)];
            const uint32_t ttl_prev = (w7p >> 16) & 255u;
            if (ti_tgt(ti) != v) {
                if (dist >= L.log_cap()) fail(H, PRISMA_EBIT_LOGWRAP);
                // IpForward decrements the TTL first and drops at 0 (no trace, no counter)
                if (ttl_prev == (route(S, u, v) >> 8)) return 0;
                if (!link_send(S, R, H, ti_link(route(S, v, ti_tgt(ti))), x)) {
                    // dropped on an intermediate FIFO: point-to-point-net-device.cc:655-664 at this
                    // node, MacTxDrop -> the sender's loss (data-packet-manager.cc:88-98,
                    // forwarder.py:214-244)
                    if (((w6p >> 8) & 255u) != v) {
                        CNT_ADD(S, ov_lost, 1u);
                        CNT_ADD(S, cost_sum, L.loss_penalty_f());
                        CNT_ADD(S, cost_n, 1u);
                    } else {
                        CNT_ADD(S, un_lost, 1u);
                        CNT_ADD(S, un_cost_sum, L.loss_penalty_f());
                        CNT_ADD(S, un_cost_n, 1u);
                    }
                    patch_status(S, d - dist, PRISMA_ST_DROPPED);
                    CNT_ADD(S, reward_sum, L.loss_penalty());
                }
                return 0;
            }
            ttl = ttl_prev - (ti_len(ti) - 1u);
        }
        H.dec = d + 1u;
        const uint32_t obs_links = observe_links(S, R, H, v, ns_to_sec(H.now));
        const int64_t t_prev = mk64(rfl(ph.x), rfl(ph.y));
        const uint32_t uid_prev = rfl(ph.z), w_prev = rfl(pw.x);
        double reward = 0.0;
        int32_t prev = -1;
        uint32_t dst, start, uid, last = 0u;
        if (type == T_FRESH) {
            // first notification: destination from the flow, uid and start
            // second rebuilt from their low bits (the packet left its app less
            // than 1 s and fewer than 2^20 injections ago)
            const uint32_t f = f_flow(x);
            dst = (uint32_t)S.T->fdst[f];
            const uint32_t s0 = (uint32_t)(H.now / 1000000000);
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
            reward = (double)py_micros(H.now) / 1e6 - (double)py_micros(t_prev) / 1e6;   // forwarder.py:360
            CNT_ADD(S, reward_sum, reward);
        }
        // obs[0] = m_map_overlay_array[dst] (the identity on identity overlays)
        const uint32_t o = (S.lane == 0) ? (tun ? (uint32_t)S.T->ovi[dst] : dst) : obs_links;
        CNT_ADD(S, decisions, 1u);
        // --train: the answer to this notification also echoes a small-signalling
        // packet to the last hop, unless this node is the packet's source (:303-306)
        const uint32_t echo = (L.train() && v != ent_src(S, x)) ? PEND_ECHO : 0u;
        D.x = x; D.dst = dst; D.start = start; D.uid = uid; D.v = v; D.d = d; D.reward = reward; D.prev = prev;
        D.obs = o; D.flags = echo; D.last = last; D.ttl = ttl;
        if (dst == v) {                                             // getGameOver
            write_record(S, H, d, reward, uid, prev, v, dst, start, -1, PRISMA_ST_DESTINATION, o, ttl);
            if (!fused && L.notify_dest()) {                        // the agent is notified (done=True)
                D.flags |= PEND_DEST;
                return 1;
            }
            if (echo) send_echo(S, R, H, (uint32_t)S.T->lrev[l], uid, last);
            receive_counters(S, R, H, x, true, start);
            return 0;
        }
        if (!fused) write_record(S, H, d, reward, uid, prev, v, dst, start, -1, PRISMA_ST_PENDING, o, ttl);
        return 1;
    }
    wire_pop(S, R, H, l, k);
    if (ent_is_echo(x)) {
        const uint32_t to = e_to(x);
        if (tun && to != v) { ctrl_forward(S, R, H, v, to, x); return 0; }
        // SmallSignalingPacketManager::receivePacket (small-signaling-packet-manager.cc:86-94):
        // addressed to this node, so valid -> Notify; the agent sees obs [1000]
        if (!fused && L.notify_dest()) {
            D.x = x; D.v = v; D.uid = e_uid(x); D.flags = PEND_CTRL; D.last = 0u;
            D.obs = (S.lane == 0) ? 1000u : ((S.lane == 1) ? e_uid(x) : 0u);
            return 1;
        }
        receive_counters(S, R, H, x, false, 0u);
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
            if (S.lane == 0) S.pbd[slot * L.PBK() + (rnd & (L.PBK() - 1))] = delay;
            if (!link_send(S, R, H, (uint32_t)S.T->lrev[l], p_make(T_PBACK, t, pos, rnd))) CNT_ADD(S, ctrl_dropped, 1u);
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
                const uint32_t idx = t - (uint32_t)S.T->ovrow[org];
                const uint32_t v0 = (uint32_t)S.T->ovrow[v];
                if (idx >= (uint32_t)S.T->ovrow[v + 1] - v0) fail(H, PRISMA_EBIT_PINGIDX);
                else ping_ack(S, R, H, v0 + idx, rnd, delay);
            }
        }
        if (org != v) { ctrl_forward(S, R, H, v, org, x); return 0; }
    }
    receive_counters(S, R, H, x, false, 0u);
    return 0;
}

// ---------------------------------------------------------------------------
// replica (re)initialisation: LDS image zeroed, registers set (all lanes)
// ---------------------------------------------------------------------------
// keep_totals: carry the header's hops_total / events_total over (auto-reset)
template <int FS, int LS>
__device__ __forceinline__ void init_replica(Sim& S, Regs<FS, LS>& R, Hot& H, uint32_t episode, bool keep_totals) {
    const LV& L = S.lv;
    const int lane = S.lane;
    uint32_t dec = H.dec, hl = H.hops_launch, el = H.ev_launch;
    const uint64_t ht = keep_totals ? (uint64_t)u_ld64((const int64_t*)&S.h->hops_total) : 0u;
    const uint64_t et = keep_totals ? (uint64_t)u_ld64((const int64_t*)&S.h->events_total) : 0u;
    __syncthreads();
    uint4* st4 = (uint4*)S.base;
    for (uint32_t i = (uint32_t)lane; i < L.lds_state_bytes() / 16u; i += kWave) st4[i] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < FS; ++j) {
        uint32_t f = (uint32_t)lane + 64u * j;
        int64_t t = INT64_MAX;
        uint32_t s = 0xffffffffu;
        if (f < (uint32_t)L.F()) {
            uint32_t c[4] = { f, 0u, episode, 0u };
            philox4x32_10(c, L.seed_lo(), S.gid);
            uint64_t u53 = ((uint64_t)(c[0] >> 5) << 26) | (uint64_t)(c[1] >> 6);
            double U = (double)u53 * (1.0 / 9007199254740992.0);
            t = sec_to_ns(0.0001 + U);                              // sim.cc:610-630
            s = (uint32_t)L.NO() + f;                          // after the NO ping timers
        }
        R.fk_lo.v[j] = lo32(t); R.fk_hi.v[j] = hi32(t); R.fk_seq.v[j] = s; R.f_draw.v[j] = 0;
    }
#pragma unroll
    for (int j = 0; j < LS; ++j) {
        R.lk_t.v[j] = 0; R.lk_seq.v[j] = 0xffffffffu; R.lk_kind.v[j] = 0;
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
    H.seq = (uint32_t)L.NO() + (uint32_t)L.F();
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
    if (k < bk || (k == bk && s < bs)) { bk = k; bs = s; bc = c; }
}

__device__ __forceinline__ uint32_t sat_offset(int64_t t, int64_t now) {
    const uint64_t dt = (uint64_t)(t - now);
    return (dt >> 32) ? 0xffffffffu : (uint32_t)dt;
}

template <int FS, int LS>
__device__ __forceinline__ void select_event(const Regs<FS, LS>& R, const Hot& H, int lane, int64_t& bt, uint32_t& bc) {
    // flows and the ping timer: exact 64-bit per-lane minimum, then one offset
    int64_t ft = INT64_MAX;
    uint32_t s = 0xffffffffu, c = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < FS; ++j) {
        const int64_t tj = mk64(R.fk_lo.v[j], R.fk_hi.v[j]);
        const uint32_t sj = R.fk_seq.v[j];
        if (key_less(tj, sj, ft, s)) { ft = tj; s = sj; c = (K_FLOW << 28) | (uint32_t)(lane + 64 * j); }
    }
    if (lane == 0 && key_less(H.ping_t, H.ping_seq, ft, s)) { ft = H.ping_t; s = H.ping_seq; c = K_PING << 28; }
    uint32_t k = sat_offset(ft, H.now);
    // links: 32-bit offsets
    const uint32_t n0 = lo32(H.now);
#pragma unroll
    for (int j = 0; j < LS; ++j) {
        const uint32_t kind = R.lk_kind.v[j];
        const uint32_t kj = kind ? R.lk_t.v[j] - n0 : 0xffffffffu;
        key_take(kj, R.lk_seq.v[j], (kind << 28) | (uint32_t)(lane + 64 * j), k, s, c);
    }
    const uint32_t kmin = wave_umin_fast(k);
    if (kmin != 0xffffffffu) {
        bt = H.now + (int64_t)kmin;
        const bool tie = (k == kmin);
        const uint64_t tied = __ballot(tie);
        uint32_t win;
        if ((tied & (tied - 1)) == 0) {
            win = (uint32_t)__builtin_ctzll(tied);
        } else {                                                    // same-ns events: ns-3 uid order
            const uint32_t smin = wave_umin_fast(tie ? s : 0xffffffffu);
            win = (uint32_t)__builtin_ctzll(__ballot(tie && s == smin));
        }
        bc = rdl(c, win);
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
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// the [N][N] action table (table policy) sits in LDS after the state image
__device__ __forceinline__ void stage_table(unsigned char* lds, const KParams& P, int lane) {
    CLayout& LC = *(CLayout*)P.lay;
    if (P.table) {
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

// mode 0: (re)build every replica at episode P.episode.
// mode 3 (auto-reset, launched after each step when auto_reset is set): a
// replica whose episode ended (and did not fail) starts episode + 1, keeping
// its decision-log position and running totals.  The event loop itself never
// resets, so a launch never crosses an episode boundary.
template <int FS, int LS>
__global__ void __launch_bounds__(64) prisma_reset_kernel_t(KParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int r = blockIdx.x, lane = threadIdx.x;
    CLayout& LC = *(CLayout*)P.lay;
    const unsigned char* img = P.state + (size_t)r * LC.state_bytes;
    const Hdr* gh = (const Hdr*)(img + kOffHdr);
    uint32_t episode = P.episode;
    Hot H;
    memset(&H, 0, sizeof(H));
    const bool keep = (P.mode == 3);
    if (keep) {
        if (!rfl(gh->over) || rfl(gh->error)) return;           // replica still running (or failed)
        episode = rfl(gh->episode) + 1u;
        H.dec = rfl(gh->dec_count);
        if (lane < (int)(sizeof(Hdr) / 4)) ((uint32_t*)(lds + kOffHdr))[lane] = ((const uint32_t*)gh)[lane];
        __syncthreads();
    }
    LV lv;
    lv.load(P.lay, lane);
    Sim S;
    sim_bind(S, lv, lds, P.topo, P.log + (size_t)r * LC.log_cap * LC.rec_bytes, LC.replica_base + (uint32_t)r, lane);
    Regs<FS, LS> R;
    init_replica(S, R, H, episode, keep);
    hot_store(S, R, H);
    __syncthreads();
    publish_counters(S, P, r, lane);
    stage_out(lds, P, r, lane, R);
}

// waves per SIMD the register allocator must leave room for: 4 (<= 128
// VGPRs) for small replicas so 4096 of them are resident on 256 CUs at
// once, 2 (<= 256) up to 512 flows x 128 links
template <int FS, int LS> struct StepOcc {
    static constexpr int waves = (FS <= 2 && LS == 1) ? 4 : (LS <= 2 ? 2 : 1);
};

// MLP: the in-kernel DQN-buffer policy is compiled in (mode 4 only); the table /
// external instances carry none of its code or registers.
template <int FS, int LS, bool MLP, bool TUN>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(StepOcc<FS, LS>::waves)))
prisma_step_kernel_t(KParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int r = blockIdx.x, lane = threadIdx.x;
    CLayout& LC = *(CLayout*)P.lay;
    LV lv;
    lv.load(P.lay, lane);
    Regs<FS, LS> R;
    stage_in(lds, P, r, lane, R);
    __syncthreads();
    Sim S;
    sim_bind(S, lv, lds, P.topo, P.log + (size_t)r * LC.log_cap * LC.rec_bytes, LC.replica_base + (uint32_t)r, lane);
    S.tun = TUN;
    const LV& L = S.lv;
    const bool mlp_mode = MLP;
    const bool table_mode = (P.mode == 2) || mlp_mode;            // fused in-kernel policy
    S.mlp = P.mlp;
    const uint32_t max_hops = (uint32_t)P.max_hops;
    const uint32_t NN = (uint32_t)L.N();
    Hot H;
    hot_load(S, H);

    H.stop = 0;
    H.hops_launch = 0;
    if (H.pend && !H.over) {
        if (table_mode) {
            uint32_t pn = u_ld32(&S.h->pend_node), pd = u_ld32(&S.h->pend_ent[1]);
            const int a = mlp_mode ? mlp_action(S, pn, (lane < L.W()) ? S.obs[lane] : 0u)
                                   : (int)rfl((uint32_t)S.table[pn * NN + pd]);
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
#define TM_MARK(i) do { tm_b = TM_NOW(); tm_acc[i] += tm_b - tm_a; tm_cnt[i]++; tm_a = tm_b; } while (0)
#else
#define TM_MARK(i) do { } while (0)
#endif
    while (!H.stop) {
        int64_t bt;
        uint32_t bc;
#if PRISMA_TIMING
        tm_a = TM_NOW();
#endif
        select_event(R, H, lane, bt, bc);
        if (bt >= L.t_end()) {                           // Simulator::Stop(simTime) (sim.cc:703)
            H.over = 1;
            H.stop = 1;
            break;
        }
        H.now = bt;
        CNT_ADD(S, events, 1u);
        H.ev_launch++;
        const uint32_t kind = bc >> 28, id = bc & 0x0fffffffu;
        TM_MARK(0);
        if (kind == K_ARRIVE) {
            Decision D;
            const int need = on_arrive(S, R, H, id, D, table_mode);
            TM_MARK(1);
            if (need) {
                if (table_mode) {
                    const int a = mlp_mode ? mlp_action(S, D.v, D.obs)
                                           : (int)rfl((uint32_t)S.table[D.v * NN + D.dst]);
                    apply_decision(S, R, H, D.x, D.dst, D.start, D.uid, D.v, D.d, a, true,
                                   D.reward, D.prev, D.obs,
                                   (D.flags & PEND_ECHO) ? (uint32_t)S.T->lrev[id] : kNoLink, D.last, D.ttl);
                    H.hops_launch++;
                    if (H.hops_launch >= max_hops) H.stop = 1;
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
    }
#if PRISMA_TIMING
    tm_acc[6] = S.tsub[0]; tm_acc[7] = S.tsub[1];
    if (lane == 0) {
        for (int i = 0; i < 8; ++i) {
            atomicAdd(&g_prisma_timing[i], (unsigned long long)tm_acc[i]);
            atomicAdd(&g_prisma_timing[8 + i], (unsigned long long)tm_cnt[i]);
        }
    }
#endif

    hot_store(S, R, H);
    __syncthreads();
    const bool pending = H.pend && !H.over;
    if (P.mask_out && lane == 0) P.mask_out[r] = pending ? 1 : 0;
    if (P.node_out && lane == 0) P.node_out[r] = pending ? (int32_t)S.h->pend_node : -1;
    if (P.obs_out && lane < L.W()) P.obs_out[(size_t)r * L.W() + lane] = pending ? (int32_t)S.obs[lane] : 0;
    publish_counters(S, P, r, lane);
    stage_out(lds, P, r, lane, R);
}

// instantiations: flow slots FS in {1,2,4,8} (F <= 512), link slots LS in {1,2,4} (L <= 256)
typedef void (*kernel_fn)(KParams);
template <int FS, int LS> struct KPair {
    static const void* step(bool tun) {
        return tun ? (const void*)prisma_step_kernel_t<FS, LS, false, true>
                   : (const void*)prisma_step_kernel_t<FS, LS, false, false>;
    }
    static const void* step_mlp(bool tun) {
        return tun ? (const void*)prisma_step_kernel_t<FS, LS, true, true>
                   : (const void*)prisma_step_kernel_t<FS, LS, true, false>;
    }
    static const void* reset() { return (const void*)prisma_reset_kernel_t<FS, LS>; }
};

// which: 0 step (table / external), 1 reset, 2 step with the DQN-buffer policy;
// tun: tunnelled-overlay instance (identity overlays run code without the tunnel paths)
static const void* pick_kernel(int fs, int ls, int which, bool tun) {
#define PK(F_, L_) if (fs == F_ && ls == L_) \
    return which == 1 ? KPair<F_, L_>::reset() : (which == 2 ? KPair<F_, L_>::step_mlp(tun) : KPair<F_, L_>::step(tun));
    PK(1, 1) PK(1, 2) PK(1, 4) PK(2, 1) PK(2, 2) PK(2, 4) PK(4, 1) PK(4, 2) PK(4, 4) PK(8, 1) PK(8, 2) PK(8, 4)
#undef PK
    return nullptr;
}

// Gather records (replica[i], dec[i]) into a dense array: one lane per 4-byte
// word, a wave per group of records (record rows are 48-64 B, so a wave
// writes 1 KiB contiguous destination rows).
// writes 1 KiB contiguous destination rows).
extern "C" __global__ void __launch_bounds__(256) prisma_gather_kernel(
        const unsigned char* log, uint32_t log_cap, uint32_t rec_bytes, const int32_t* replica,
        const uint32_t* dec, int32_t n, uint32_t* dst) {
    const uint32_t words = rec_bytes / 4u;
    const uint64_t total = (uint64_t)n * words;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = i / words;
        uint32_t w = (uint32_t)(i - k * words);
        const uint32_t* src = (const uint32_t*)(log + ((size_t)replica[k] * log_cap + (dec[k] & (log_cap - 1))) * rec_bytes);
        dst[i] = src[w];
    }
}

// ===========================================================================
// host side: sizing, validation, C-ABI
// ===========================================================================
struct prisma_env {
    int device;
    int32_t R;
    Layout lay;
    unsigned char* d_state = nullptr;
    unsigned char* d_topo = nullptr;
    unsigned char* d_log = nullptr;
    prisma_counters_t* d_cnt = nullptr;
    Layout* d_lay = nullptr;
    const void* k_step = nullptr;
    const void* k_step_mlp = nullptr;
    const void* k_reset = nullptr;
    bool reset_done = false;
};

static thread_local std::string g_err;
static int set_err(int code, const std::string& msg) { g_err = msg; return code; }

extern "C" int prisma_abi_version(void) { return PRISMA_ABI_VERSION; }

#if PRISMA_TIMING
// diagnostic build only: read and clear the per-phase cycle totals
extern "C" int prisma_debug_timing(unsigned long long* out16) {
    if (!HIP_OK(hipDeviceSynchronize()) ||
        !HIP_OK(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_prisma_timing), 16 * sizeof(unsigned long long)))) return -1;
    unsigned long long z[16] = {0};
    return HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_prisma_timing), z, sizeof(z))) ? 0 : -1;
}
#endif
extern "C" const char* prisma_last_error(void) { return g_err.c_str(); }

static uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }
static uint32_t next_pow2(uint32_t x) { uint32_t p = 1; while (p < x) p <<= 1; return p; }

// Overlay of a topology (host): tunnels, routing, control-packet load per link.
struct OverlayPlan {
    bool tunnels = false;                // false: identity overlay (tunnel t == link t)
    int T = 0, NO = 0, maxdeg = 0, plen = 1;
    std::vector<int32_t> ovrow, ovi, ovnode;
    std::vector<uint32_t> tinfo, route;  // route: [N][N] next link | hops << 8
    std::vector<uint32_t> tresp;         // pbd slot base | responder position mask << 16
    int n_resp = 0;                      // ping responders over all tunnels (pbd slots)
    // control-packet routes (links in order), each starting when its ping round
    // (or, for echoes, the data arrival) fires: pings, ping-backs, echoes
    std::vector<std::vector<int>> cpaths, epaths;
};

// ns-3 global routing restated for unit link metrics: the SPF
// pops equal-distance candidates first-in-first-out and scans link records in
// device order (ascending neighbour id), and without RandomEcmpRouting the
// first root exit direction is used -- so x forwards towards y through the
// lowest-id neighbour that lies on a shortest path.  Identical rule in
// prisma_amd/topology.py:route_tables (the oracle's routing).
static int plan_overlay(const prisma_topology_t* T, OverlayPlan& OP) {
    const int N = T->n_nodes, E = T->n_links;
    std::vector<int32_t> adj((size_t)N * N, -1);             // link id u -> v
    for (int u = 0; u < N; ++u)
        for (int l = T->row_ptr[u]; l < T->row_ptr[u + 1]; ++l) adj[(size_t)u * N + T->link_dst[l]] = l;
    std::vector<int32_t> dist((size_t)N * N, -1);
    for (int y = 0; y < N; ++y) {
        std::vector<int> fr(1, y), nx;
        dist[(size_t)y * N + y] = 0;
        while (!fr.empty()) {
            nx.clear();
            for (int u : fr)
                for (int l = T->row_ptr[u]; l < T->row_ptr[u + 1]; ++l) {
                    const int w = T->link_dst[l];
                    if (dist[(size_t)w * N + y] < 0) { dist[(size_t)w * N + y] = dist[(size_t)u * N + y] + 1; nx.push_back(w); }
                }
            fr.swap(nx);
        }
    }
    for (size_t i = 0; i < dist.size(); ++i)
        if (dist[i] < 0) return set_err(PRISMA_ERR_CONFIG, "the physical topology must be connected");
    std::vector<int32_t> hop((size_t)N * N, -1);
    for (int x = 0; x < N; ++x)
        for (int y = 0; y < N; ++y) {
            if (x == y) continue;
            for (int l = T->row_ptr[x]; l < T->row_ptr[x + 1]; ++l)   // ascending neighbour id
                if (dist[(size_t)T->link_dst[l] * N + y] == dist[(size_t)x * N + y] - 1) { hop[(size_t)x * N + y] = l; break; }
        }
    // overlay nodes and adjacency
    const int NO = T->n_overlay > 0 ? T->n_overlay : N;
    if (NO < 2 || NO > N) return set_err(PRISMA_ERR_CONFIG, "n_overlay must be 0 or in [2, n_nodes]");
    if (T->n_overlay > 0 && (!T->overlay_nodes || !T->overlay_adj)) return set_err(PRISMA_ERR_ARG, "null overlay array");
    OP.NO = NO;
    OP.ovi.assign(N, -1);
    OP.ovnode.resize(NO);
    for (int i = 0; i < NO; ++i) {
        const int u = T->n_overlay > 0 ? T->overlay_nodes[i] : i;
        if (u < 0 || u >= N || OP.ovi[u] >= 0) return set_err(PRISMA_ERR_CONFIG, "bad overlay_nodes");
        OP.ovi[u] = i;
        OP.ovnode[i] = u;
    }
    auto oadj = [&](int i, int j) -> bool {
        return T->n_overlay > 0 ? T->overlay_adj[(size_t)i * NO + j] != 0 : adj[(size_t)i * N + j] >= 0;
    };
    for (int i = 0; i < NO; ++i)
        for (int j = 0; j < NO; ++j)
            if (oadj(i, j) != oadj(j, i) || (i == j && oadj(i, i)))
                return set_err(PRISMA_ERR_CONFIG, "overlay adjacency must be symmetric without self-loops");
    // tunnels grouped by underlay id, each node's in ascending overlay index (sim.cc:469-476)
    OP.ovrow.assign(N + 1, 0);
    std::vector<int> tsrc, tdst;
    for (int u = 0; u < N; ++u) {
        const int i = OP.ovi[u];
        int deg = 0;
        if (i >= 0)
            for (int j = 0; j < NO; ++j)
                if (oadj(i, j)) { tsrc.push_back(u); tdst.push_back(OP.ovnode[j]); ++deg; }
        if (i >= 0 && deg == 0) return set_err(PRISMA_ERR_CONFIG, "an overlay node has no overlay neighbour");
        OP.maxdeg = deg > OP.maxdeg ? deg : OP.maxdeg;
        OP.ovrow[u + 1] = (int32_t)tsrc.size();
    }
    OP.T = (int)tsrc.size();
    if (OP.T > 256) return set_err(PRISMA_ERR_CONFIG, "more than 256 tunnels (8-bit tunnel ids)");
    bool ident = (NO == N);
    for (int t = 0; t < OP.T && ident; ++t) ident = (dist[(size_t)tsrc[t] * N + tdst[t]] == 1);
    for (int i = 0; i < NO && ident; ++i) ident = (OP.ovnode[i] == i);
    OP.tunnels = !ident;
    OP.tinfo.resize(OP.T);
    OP.tresp.resize(OP.T);
    auto route_links = [&](int x, int y, std::vector<int>& out) {   // append the route x -> y
        while (x != y) { const int l = hop[(size_t)x * N + y]; out.push_back(l); x = T->link_dst[l]; }
    };
    for (int t = 0; t < OP.T; ++t) {
        const int u = tsrc[t], w = tdst[t];
        const int len = dist[(size_t)u * N + w];
        if (len > 8) return set_err(PRISMA_ERR_CONFIG, "tunnel longer than 8 links (3-bit responder position)");
        OP.plen = len > OP.plen ? len : OP.plen;
        const int l0 = ident ? t : hop[(size_t)u * N + w];
        OP.tinfo[t] = (uint32_t)l0 | ((uint32_t)w << 8) | ((uint32_t)u << 16) | ((uint32_t)len << 24);
        // forward path of the pings; a ping-back from every overlay node on it
        // (reverse of the arrival link, then routed to the origin); the --train
        // echo from the target likewise
        std::vector<int> fwd;
        route_links(u, w, fwd);
        OP.cpaths.push_back(fwd);
        uint32_t mask = 0;
        int x = u;
        for (int i = 0; i < len; ++i) {
            const int l = fwd[i], nxt = T->link_dst[l];
            if (OP.ovi[nxt] >= 0) {
                mask |= 1u << i;
                std::vector<int> rp(fwd.begin(), fwd.begin() + i + 1);
                rp.push_back(T->link_rev[l]);
                route_links(x, u, rp);
                OP.cpaths.push_back(rp);
                if (nxt == w) {
                    std::vector<int> ep(1, T->link_rev[l]);
                    route_links(x, u, ep);
                    OP.epaths.push_back(ep);
                }
            }
            x = nxt;
        }
        OP.tresp[t] = (uint32_t)OP.n_resp | (mask << 16);
        OP.n_resp += __builtin_popcount(mask);
    }
    if (OP.tunnels) {
        OP.route.assign((size_t)N * N, 0u);
        for (int x = 0; x < N; ++x)
            for (int y = 0; y < N; ++y)
                OP.route[(size_t)x * N + y] = (x == y ? 255u : (uint32_t)hop[(size_t)x * N + y]) |
                                              ((uint32_t)dist[(size_t)x * N + y] << 8);
    }
    return PRISMA_OK;
}

static int build_layout(const prisma_topology_t* T, const prisma_params_t* P, Layout& L,
                        std::vector<unsigned char>& topo) {
    const int N = T->n_nodes, E = T->n_links, F = T->n_flows;
    if (N < 2 || N > 255) return set_err(PRISMA_ERR_CONFIG, "n_nodes must be in [2, 255] (8-bit node ids)");
    if (E < 1 || F < 1) return set_err(PRISMA_ERR_CONFIG, "need at least one link and one flow");
    if (!T->row_ptr || !T->link_dst || !T->link_rev || !T->flow_src || !T->flow_dst || !T->flow_rate_bps)
        return set_err(PRISMA_ERR_ARG, "null topology array");
    if (T->row_ptr[0] != 0 || T->row_ptr[N] != E) return set_err(PRISMA_ERR_CONFIG, "row_ptr must span [0, n_links]");
    int maxdeg = 0;
    for (int u = 0; u < N; ++u) {
        int d = T->row_ptr[u + 1] - T->row_ptr[u];
        if (d < 1) return set_err(PRISMA_ERR_CONFIG, "every node needs at least one link");
        if (d > maxdeg) maxdeg = d;
        for (int l = T->row_ptr[u]; l < T->row_ptr[u + 1]; ++l) {
            int v = T->link_dst[l], rv = T->link_rev[l];
            if (v < 0 || v >= N || v == u) return set_err(PRISMA_ERR_CONFIG, "bad link_dst");
            if (l > T->row_ptr[u] && T->link_dst[l - 1] >= v) return set_err(PRISMA_ERR_CONFIG, "neighbours must be ascending");
            if (rv < 0 || rv >= E || T->link_dst[rv] != u || rv < T->row_ptr[v] || rv >= T->row_ptr[v + 1])
                return set_err(PRISMA_ERR_CONFIG, "bad link_rev");
        }
    }
    (void)maxdeg;
    // ---- overlay: tunnels along ns-3 global routing (sim.cc:455-476, 683)
    OverlayPlan OP;
    int rc = plan_overlay(T, OP);
    if (rc) return rc;
    if (OP.maxdeg != T->max_deg) return set_err(PRISMA_ERR_CONFIG, "max_deg mismatch (largest overlay degree)");
    if (OP.maxdeg > 127) return set_err(PRISMA_ERR_CONFIG, "degree above 127");
    for (int f = 0; f < F; ++f) {
        if (T->flow_src[f] < 0 || T->flow_src[f] >= N || T->flow_dst[f] < 0 || T->flow_dst[f] >= N ||
            T->flow_src[f] == T->flow_dst[f] || T->flow_rate_bps[f] == 0 ||
            OP.ovi[T->flow_src[f]] < 0 || OP.ovi[T->flow_dst[f]] < 0)
            return set_err(PRISMA_ERR_CONFIG, "bad flow (flows run between overlay nodes)");
    }
    const int maxdeg_o = OP.maxdeg;
    if (P->link_bps == 0 || P->link_delay_ns < 0 || P->max_buffer_bytes == 0 || P->packet_size == 0 ||
        P->ma_size == 0 || P->ma_size > 64 || !(P->ping_interval_s > 0.0f))
        return set_err(PRISMA_ERR_CONFIG, "bad link / ping parameters");
    if (!(P->sim_time_s > 0.0) || P->sim_time_s > 4095.0)
        return set_err(PRISMA_ERR_CONFIG, "sim_time_s must be in (0, 4095] (12-bit packet start second)");
    if (P->sim_time_s / (double)P->ping_interval_s >= (double)(1u << 17))
        return set_err(PRISMA_ERR_CONFIG, "more than 2^17 ping rounds per episode (18-bit round field)");
    if (P->log_capacity < 1024 || P->log_capacity > (1u << 22) || (P->log_capacity & (P->log_capacity - 1)))
        return set_err(PRISMA_ERR_CONFIG, "log_capacity must be a power of two >= 1024");

    memset(&L, 0, sizeof(L));
    const int Lk = E + N;
    L.N = N; L.E = E; L.L = Lk; L.F = F; L.max_deg = maxdeg_o;
    L.T = OP.T; L.NO = OP.NO; L.tunnels = OP.tunnels ? 1u : 0u; L.PLEN = (uint32_t)OP.plen;
    L.W = (1 + maxdeg_o + 3) & ~3;                  // obs width: multiple of 4 (16-B record rows)
    L.MA = (int)P->ma_size;
    L.data_size = P->packet_size + 30u;             // UDP 8 + IP 20 + PPP 2
    L.ping_size = 8u + 30u;
    L.echo_size = 0u + 30u;                         // signalling type "ideal": 0-B payload (sim.cc:371-391)
    L.train = P->train ? 1u : 0u;
    // link constants (sim.cc:398-433): switch links share rate, delay and queue
    L.sw_txd = sec_to_ns((double)L.data_size * 8 / (double)P->link_bps);
    L.sw_txp = sec_to_ns((double)L.ping_size * 8 / (double)P->link_bps);
    L.sw_txe = sec_to_ns((double)L.echo_size * 8 / (double)P->link_bps);
    L.sw_prop = P->link_delay_ns;
    L.qmax_bytes = P->max_buffer_bytes;
    L.acc_qmax_pkts = 1000u;                        // "1000p" packet-mode access queue
    std::vector<int64_t> acctx(N);
    std::vector<int32_t> ldst(Lk);
    for (int u = 0; u < N; ++u)
        for (int l = T->row_ptr[u]; l < T->row_ptr[u + 1]; ++l) ldst[l] = T->link_dst[l];
    for (int u = 0; u < N; ++u) {
        uint64_t bps = (uint64_t)1000000 * P->link_bps * (uint64_t)(T->row_ptr[u + 1] - T->row_ptr[u]);
        acctx[u] = sec_to_ns((double)L.data_size * 8 / (double)bps);
        ldst[E + u] = u;
    }
    // wire capacity: packets whose transmission ended within the last
    // propagation delay, plus the one being transmitted
    const int64_t min_tx = L.train ? L.sw_txe : L.sw_txp;      // shortest packet on a switch link
    if (min_tx < 1) return set_err(PRISMA_ERR_CONFIG, "link too fast for the wire model");
    uint32_t wire = (uint32_t)(P->link_delay_ns / min_tx) + 2u;
    L.WCAP = (int)next_pow2(wire < 2 ? 2 : wire);
    if (L.WCAP > 64) return set_err(PRISMA_ERR_CONFIG, "propagation delay too long for the wire model");
    // ring capacity: full byte-limited FIFO of data + the control packets that
    // can be queued at once + the packets on the wire.
    double drain_s = (double)P->max_buffer_bytes * 8.0 / (double)P->link_bps + (double)L.sw_txd * 1e-9;
    const double tx_s = (double)L.sw_txd * 1e-9, ival = (double)P->ping_interval_s;
    const uint32_t data_max = P->max_buffer_bytes / L.data_size;
    std::vector<uint32_t> rcap(E);
    double span;
    if (!OP.tunnels) {
        // identity: per round one ping and one ping-back cross a link, each within
        // two FIFOs and wires of its round; echoes answer data packets that crossed
        // the reverse link, at least one data transmission apart
        span = 2.0 * (drain_s + (double)P->link_delay_ns * 1e-9);
        const uint32_t ctrl = 2u * ((uint32_t)(span / ival) + 3u);
        const uint32_t echoes = L.train ? (uint32_t)(drain_s / tx_s) + 2u : 0u;
        uint32_t qs = data_max + ctrl + echoes + (uint32_t)L.WCAP;
        qs = (qs + (uint32_t)L.WCAP - 1) / (uint32_t)L.WCAP * (uint32_t)L.WCAP;
        for (int l = 0; l < E; ++l) rcap[l] = qs;
    } else {
        // tunnelled: per link, every control route through it contributes the
        // rounds (echoes: data arrivals, >= one transmission apart) whose packets
        // can still sit in its FIFO: a packet at the d-th FIFO of its route left
        // its round's start at most d * (drain + 2 tx + propagation) before
        const double hop_s = (double)P->max_buffer_bytes * 8.0 / (double)P->link_bps + 2.0 * tx_s +
                             (double)P->link_delay_ns * 1e-9;
        std::vector<double> c(E, 0.0);
        for (const auto& pth : OP.cpaths)
            for (size_t i = 0; i < pth.size(); ++i) c[pth[i]] += (double)((uint32_t)((double)(i + 1) * hop_s / ival) + 1u);
        if (L.train)
            for (const auto& pth : OP.epaths)
                for (size_t i = 0; i < pth.size(); ++i) c[pth[i]] += (double)((uint32_t)((double)(i + 1) * hop_s / tx_s) + 1u);
        for (int l = 0; l < E; ++l) {
            uint32_t qs = data_max + (uint32_t)c[l] + (uint32_t)L.WCAP;
            rcap[l] = (qs + (uint32_t)L.WCAP - 1) / (uint32_t)L.WCAP * (uint32_t)L.WCAP;
        }
        span = 2.0 * (double)OP.plen * hop_s;
    }
    L.qcap_s = 0;
    uint32_t tot = 0;
    for (int l = 0; l < E; ++l) {
        if (rcap[l] > 65535u) return set_err(PRISMA_ERR_CONFIG, "queue too deep");
        L.qcap_s = rcap[l] > L.qcap_s ? rcap[l] : L.qcap_s;
        tot += rcap[l];
    }
    L.qcap_a = (uint32_t)(L.WCAP < 8 ? 8 : L.WCAP);
    tot += (uint32_t)N * L.qcap_a;
    if (tot > 65535u) return set_err(PRISMA_ERR_CONFIG, "ring entries exceed the LDS image");
    L.ring_total = tot;
    // ping-back delay slots per responder: round k's slot is reused by round
    // k + PBK, whose forward ping arrives after round k's ping-back (at most
    // span after k's send) has been consumed
    L.PBK = next_pow2((uint32_t)(span / ival) + 2u);
    // wire arrival times are kept as their low 32 bits relative to the clock
    int64_t max_acc = 0;
    for (int u = 0; u < N; ++u) max_acc = acctx[u] > max_acc ? acctx[u] : max_acc;
    if ((L.sw_txd > max_acc ? L.sw_txd : max_acc) + L.sw_prop >= ((int64_t)1 << 31))
        return set_err(PRISMA_ERR_CONFIG, "transmission + propagation delay above 2^31 ns");

    // topology image
    uint32_t o = 0;
    auto take = [&](uint32_t bytes) { uint32_t r = o; o = align16(o + bytes); return r; };
    L.table_bytes = (uint32_t)(N * N);
    L.topo_bytes = (uint32_t)sizeof(TopoImage) + (OP.tunnels ? 4u * (uint32_t)(N * N) : 0u);
    if (Lk > 256 || E > 256 || F > 512 || OP.T > 256) return set_err(PRISMA_ERR_CONFIG, "topology image limits exceeded");
    topo.assign(L.topo_bytes, 0);
    TopoImage& TI = *(TopoImage*)topo.data();
    memcpy(TI.rowptr, T->row_ptr, 4u * (N + 1));
    memcpy(TI.ldst, ldst.data(), 4u * Lk);
    memcpy(TI.lrev, T->link_rev, 4u * E);
    memcpy(TI.acctx, acctx.data(), 8u * N);
    memcpy(TI.fsrc, T->flow_src, 4u * F);
    memcpy(TI.fdst, T->flow_dst, 4u * F);
    for (int f = 0; f < F; ++f)                      // poisson-application.cc:280-283
        TI.fmean[f] = (double)(P->packet_size * 8u) / (double)T->flow_rate_bps[f];
    memcpy(TI.ovrow, OP.ovrow.data(), 4u * (N + 1));
    memcpy(TI.tinfo, OP.tinfo.data(), 4u * OP.T);
    for (int x = 0; x < N; ++x) TI.ovi[x] = OP.ovi[x];
    memcpy(TI.ovnode, OP.ovnode.data(), 4u * OP.NO);
    if (OP.tunnels) {
        uint32_t off = 0;
        for (int l = 0; l < Lk; ++l) {
            const uint32_t cap = l < E ? rcap[l] : L.qcap_a;
            TI.rinfo[l] = off | (cap << 16);
            off += cap;
        }
        memcpy(TI.tresp, OP.tresp.data(), 4u * OP.T);
    }
    if (OP.tunnels) memcpy(topo.data() + sizeof(TopoImage), OP.route.data(), 4u * (size_t)N * N);

    // state image: LDS part (staged into LDS) then register part (staged into VGPRs)
    int fs = 1, ls = 1;
    while (64 * fs < F) fs *= 2;
    while (64 * ls < (Lk > OP.T ? Lk : OP.T)) ls *= 2;
    if (fs > 8 || ls > 4)
        return set_err(PRISMA_ERR_CONFIG,
                       "more than 512 flows or 256 links / tunnels per replica (register-resident engine)");
    L.FS = fs; L.LS = ls;
    o = 0;
    L.s_hdr = take(sizeof(Hdr));
    L.s_cnt = take(sizeof(prisma_counters_t));
    L.s_obs = take(4u * L.W);
    if (L.s_hdr != kOffHdr || L.s_cnt != kOffCnt || L.s_obs != kOffObs)
        return set_err(PRISMA_ERR_CONFIG, "internal: LDS header offsets");
    L.s_wt = take(4u * Lk * L.WCAP);
    L.s_wseq = take(4u * Lk * L.WCAP);
    L.s_ring = take(4u * tot);
    L.s_win = take(4u * (uint32_t)OP.T * L.MA);
    L.s_pbd = take(4u * (uint32_t)(OP.tunnels ? OP.n_resp : OP.T) * L.PBK);
    L.lds_state_bytes = o;
    L.s_regs = take(4u * (4u * 64u * (uint32_t)fs + 19u * 64u * (uint32_t)ls));
    L.state_bytes = o;
    L.lds_bytes = L.lds_state_bytes + align16(L.table_bytes);
    L.s_mlp = L.lds_bytes;                          // + 256 B of DQN-buffer activations (MLP launches only)
    if (L.lds_bytes + 256u > 160u * 1024u)
        return set_err(PRISMA_ERR_CONFIG, "replica state exceeds the 160 KiB LDS of a gfx950 CU");

    L.t_end = sec_to_ns(P->sim_time_s);
    L.ping_period = sec_to_ns((double)P->ping_interval_s);     // Seconds(float) (sim.cc:173)
    L.ma = P->ma_size;
    L.ping_as_obs = P->ping_as_obs ? 1u : 0u;
    L.auto_reset = P->auto_reset ? 1u : 0u;
    L.notify_dest = P->notify_dest ? 1u : 0u;
    L.seed_lo = (uint32_t)P->seed;
    L.replica_base = P->replica_base;
    L.log_cap = P->log_capacity;
    L.rec_bytes = 32u + 4u * (uint32_t)L.W;
    L.loss_penalty = P->loss_penalty;
    L.loss_penalty_f = (float)P->loss_penalty;
    return PRISMA_OK;
}

extern "C" int prisma_create(const prisma_topology_t* topo, const prisma_params_t* params, int32_t n_replicas,
                             int32_t device, prisma_env_t** out) {
    if (!topo || !params || !out || n_replicas < 1) return set_err(PRISMA_ERR_ARG, "null argument or n_replicas < 1");
    *out = nullptr;
    Layout L;
    std::vector<unsigned char> img;
    int rc = build_layout(topo, params, L, img);
    if (rc) return rc;
    int ndev = 0;
    if (!HIP_OK(hipGetDeviceCount(&ndev)) || ndev == 0) return set_err(PRISMA_ERR_DEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return set_err(PRISMA_ERR_DEVICE, "device index out of range");
    if (!HIP_OK(hipSetDevice(device))) return set_err(PRISMA_ERR_DEVICE, "hipSetDevice failed");
    hipDeviceProp_t prop;
    if (!HIP_OK(hipGetDeviceProperties(&prop, device))) return set_err(PRISMA_ERR_DEVICE, "hipGetDeviceProperties failed");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_err(PRISMA_ERR_DEVICE, std::string("engine is built for gfx950, device is ") + prop.gcnArchName);
    prisma_env* e = new (std::nothrow) prisma_env();
    if (!e) return set_err(PRISMA_ERR_NOMEM, "host allocation failed");
    e->device = device;
    e->R = n_replicas;
    e->lay = L;
    size_t sb = (size_t)L.state_bytes * n_replicas;
    size_t lb = (size_t)L.log_cap * L.rec_bytes * n_replicas;
    if (!HIP_OK(hipMalloc(&e->d_state, sb)) || !HIP_OK(hipMalloc(&e->d_topo, L.topo_bytes)) ||
        !HIP_OK(hipMalloc(&e->d_log, lb)) ||
        !HIP_OK(hipMalloc((void**)&e->d_cnt, sizeof(prisma_counters_t) * n_replicas)) ||
        !HIP_OK(hipMalloc((void**)&e->d_lay, sizeof(Layout)))) {
        prisma_destroy(e);
        return set_err(PRISMA_ERR_NOMEM, "hipMalloc failed");
    }
    if (!HIP_OK(hipMemcpy(e->d_topo, img.data(), L.topo_bytes, hipMemcpyHostToDevice)) ||
        !HIP_OK(hipMemcpy(e->d_lay, &L, sizeof(Layout), hipMemcpyHostToDevice)) ||
        !HIP_OK(hipMemset(e->d_log, 0, lb)) ||
        !HIP_OK(hipMemset(e->d_cnt, 0, sizeof(prisma_counters_t) * n_replicas))) {
        prisma_destroy(e);
        return set_err(PRISMA_ERR_DEVICE, "device initialisation failed");
    }
    e->k_step = pick_kernel(L.FS, L.LS, 0, L.tunnels != 0u);
    e->k_reset = pick_kernel(L.FS, L.LS, 1, false);
    e->k_step_mlp = pick_kernel(L.FS, L.LS, 2, L.tunnels != 0u);
    (void)hipFuncSetAttribute(e->k_step_mlp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds_bytes + 256);
    (void)hipFuncSetAttribute(e->k_step, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds_bytes);
    (void)hipFuncSetAttribute(e->k_reset, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds_bytes);
    *out = e;
    return PRISMA_OK;
}

static KParams base_params(prisma_env_t* e) {
    KParams P;
    memset(&P, 0, sizeof(P));
    P.lay = e->d_lay;
    P.state = e->d_state;
    P.topo = e->d_topo;
    P.log = e->d_log;
    P.cnt_out = e->d_cnt;
    P.R = e->R;
    return P;
}

static int launch(prisma_env_t* e, const void* kern, KParams P, void* stream) {
    (void)hipSetDevice(e->device);
    void* args[] = { &P };
    const size_t lds = e->lay.lds_bytes + (kern == e->k_step_mlp ? 256u : 0u);
    hipError_t err = hipLaunchKernel(kern, dim3((unsigned)e->R), dim3(kWave), args, lds, (hipStream_t)stream);
    if (err == hipSuccess) err = hipGetLastError();
    if (err != hipSuccess) return set_err(PRISMA_ERR_LAUNCH, std::string("kernel launch failed: ") + hipGetErrorString(err));
    return PRISMA_OK;
}

// with auto_reset, replicas whose episode ended in the last launch start the next one
static int auto_reset(prisma_env_t* e, void* stream) {
    if (!e->lay.auto_reset) return PRISMA_OK;
    KParams P = base_params(e);
    P.mode = 3;
    return launch(e, e->k_reset, P, stream);
}

extern "C" int prisma_reset(prisma_env_t* e, uint32_t episode, void* stream) {
    if (!e) return set_err(PRISMA_ERR_ARG, "null env");
    KParams P = base_params(e);
    P.mode = 0;
    P.episode = episode;
    int rc = launch(e, e->k_reset, P, stream);
    if (!rc) e->reset_done = true;
    return rc;
}

extern "C" int prisma_step(prisma_env_t* e, const int32_t* actions, int32_t* obs_out, uint8_t* mask_out,
                           int32_t* node_out, void* stream) {
    if (!e) return set_err(PRISMA_ERR_ARG, "null env");
    if (!e->reset_done) return set_err(PRISMA_ERR_STATE, "prisma_reset must be called first");
    KParams P = base_params(e);
    P.mode = 1;
    P.actions = actions;
    P.obs_out = obs_out;
    P.mask_out = mask_out;
    P.node_out = node_out;
    P.max_hops = 0x7fffffff;
    int rc = launch(e, e->k_step, P, stream);
    return rc ? rc : auto_reset(e, stream);
}

extern "C" int prisma_run(prisma_env_t* e, int32_t policy, const void* policy_data, int32_t max_hops, void* stream) {
    if (!e) return set_err(PRISMA_ERR_ARG, "null env");
    if (!e->reset_done) return set_err(PRISMA_ERR_STATE, "prisma_reset must be called first");
    if ((policy != PRISMA_POLICY_TABLE && policy != PRISMA_POLICY_DQN_BUFFER) || !policy_data)
        return set_err(PRISMA_ERR_ARG, "policy must be PRISMA_POLICY_TABLE (uint8 table) or "
                                       "PRISMA_POLICY_DQN_BUFFER (fp32 weights), with device data");
    if (max_hops < 1) return set_err(PRISMA_ERR_ARG, "max_hops must be >= 1");
    KParams P = base_params(e);
    if (policy == PRISMA_POLICY_TABLE) {
        P.mode = 2;
        P.table = (const uint8_t*)policy_data;
    } else {
        P.mode = 4;
        P.mlp = (const float*)policy_data;
    }
    P.max_hops = max_hops;
    int rc = launch(e, P.mode == 4 ? e->k_step_mlp : e->k_step, P, stream);
    return rc ? rc : auto_reset(e, stream);
}

extern "C" int prisma_read_counters(prisma_env_t* e, prisma_counters_t* host_out, void* stream) {
    if (!e || !host_out) return set_err(PRISMA_ERR_ARG, "null argument");
    (void)hipSetDevice(e->device);
    if (!HIP_OK(hipMemcpyAsync(host_out, e->d_cnt, sizeof(prisma_counters_t) * e->R, hipMemcpyDeviceToHost,
                               (hipStream_t)stream)) ||
        !HIP_OK(hipStreamSynchronize((hipStream_t)stream)))
        return set_err(PRISMA_ERR_DEVICE, "counter copy failed");
    return PRISMA_OK;
}

extern "C" int prisma_counters_device(prisma_env_t* e, void** dev_ptr) {
    if (!e || !dev_ptr) return set_err(PRISMA_ERR_ARG, "null argument");
    *dev_ptr = e->d_cnt;
    return PRISMA_OK;
}

extern "C" int prisma_log_view(prisma_env_t* e, prisma_log_view_t* out) {
    if (!e || !out) return set_err(PRISMA_ERR_ARG, "null argument");
    out->records = e->d_log;
    out->record_bytes = e->lay.rec_bytes;
    out->log_capacity = e->lay.log_cap;
    out->obs_width = e->lay.W;
    out->n_replicas = e->R;
    return PRISMA_OK;
}

extern "C" int prisma_copy_log(prisma_env_t* e, void* dst_device, uint64_t bytes, void* stream) {
    if (!e || !dst_device) return set_err(PRISMA_ERR_ARG, "null argument");
    uint64_t total = (uint64_t)e->lay.log_cap * e->lay.rec_bytes * (uint64_t)e->R;
    if (bytes < total) return set_err(PRISMA_ERR_ARG, "destination smaller than the log");
    (void)hipSetDevice(e->device);
    if (!HIP_OK(hipMemcpyAsync(dst_device, e->d_log, total, hipMemcpyDeviceToDevice, (hipStream_t)stream)))
        return set_err(PRISMA_ERR_DEVICE, "log copy failed");
    return PRISMA_OK;
}

extern "C" int prisma_copy_counters(prisma_env_t* e, void* dst_device, void* stream) {
    if (!e || !dst_device) return set_err(PRISMA_ERR_ARG, "null argument");
    (void)hipSetDevice(e->device);
    if (!HIP_OK(hipMemcpyAsync(dst_device, e->d_cnt, sizeof(prisma_counters_t) * e->R, hipMemcpyDeviceToDevice,
                               (hipStream_t)stream)))
        return set_err(PRISMA_ERR_DEVICE, "counter copy failed");
    return PRISMA_OK;
}

extern "C" int prisma_gather_records(prisma_env_t* e, const int32_t* replica, const uint32_t* dec, int32_t n,
                                     void* dst_device, void* stream) {
    if (!e || (n > 0 && (!replica || !dec || !dst_device))) return set_err(PRISMA_ERR_ARG, "null argument");
    if (n <= 0) return PRISMA_OK;
    (void)hipSetDevice(e->device);
    uint64_t total = (uint64_t)n * (e->lay.rec_bytes / 4u);
    unsigned grid = (unsigned)((total + 255) / 256);
    if (grid > 8192u) grid = 8192u;
    hipLaunchKernelGGL(prisma_gather_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const unsigned char*)e->d_log, e->lay.log_cap, e->lay.rec_bytes, replica, dec, n,
                       (uint32_t*)dst_device);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return set_err(PRISMA_ERR_LAUNCH, std::string("gather launch failed: ") + hipGetErrorString(err));
    return PRISMA_OK;
}

extern "C" int prisma_state_bytes(prisma_env_t* e, uint32_t* state_bytes, uint32_t* lds_bytes) {
    if (!e) return set_err(PRISMA_ERR_ARG, "null env");
    if (state_bytes) *state_bytes = e->lay.state_bytes;
    if (lds_bytes) *lds_bytes = e->lay.lds_bytes;
    return PRISMA_OK;
}

extern "C" int prisma_plan(const prisma_topology_t* topo, const prisma_params_t* params, prisma_plan_t* out) {
    if (!topo || !params || !out) return set_err(PRISMA_ERR_ARG, "null argument");
    Layout L;
    std::vector<unsigned char> img;
    int rc = build_layout(topo, params, L, img);
    if (rc) return rc;
    out->state_bytes = L.state_bytes;
    out->lds_bytes = L.lds_bytes;
    out->lds_state_bytes = L.lds_state_bytes;
    out->ring_entries = L.ring_total;
    out->record_bytes = L.rec_bytes;
    out->obs_width = L.W;
    out->flow_slots = L.FS;
    out->link_slots = L.LS;
    return PRISMA_OK;
}

extern "C" void prisma_destroy(prisma_env_t* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->d_state) (void)hipFree(e->d_state);
    if (e->d_topo) (void)hipFree(e->d_topo);
    if (e->d_log) (void)hipFree(e->d_log);
    if (e->d_cnt) (void)hipFree(e->d_cnt);
    if (e->d_lay) (void)hipFree(e->d_lay);
    delete e;
}
