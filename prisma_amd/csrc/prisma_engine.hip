// prisma_engine.hip — MI355X (gfx950) packet-hop engine behind include/prisma.h.
//
// Design: one 64-lane wavefront (= one workgroup) owns one
// topology replica.  At launch the replica's state image is staged from HBM
// into LDS with 16-byte coalesced loads; the wavefront then runs the
// replica's discrete-event loop out of LDS:
//   * next event = wave-wide min over (time_ns, seq) of every pending
//     candidate — flow injections, link tx-completions, wire heads and the
//     ping round — each lane scanning the candidates it owns, then a
//     64-lane shuffle reduction (the ns-3 MapScheduler order);
//   * the selected handler runs on lane 0 against LDS (FIFO push/pop in
//     per-link rings, drop-on-overflow, link-delay accumulation, the
//     Q-routing reward of forwarder.py:360);
//   * each data notification appends one decision record to the replica's
//     HBM transition log.
// At exit the image is written back to HBM.  Results are bit-identical to
// the CPU oracle (oracle/), which restates the reference ns-3 semantics.
//
// Compile: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared
// (-ffp-contract=off keeps every double/float expression identical to the
// oracle's; the reference quantities involved are cited where computed).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <new>
#include <string>
#include <vector>

#include "../../include/prisma.h"
#include "engine_layout.h"

using namespace prisma;

#define HIP_OK(x) ((x) == hipSuccess)

// ---------------------------------------------------------------------------
// numeric building blocks (device + host, identical IEEE sequences)
// ---------------------------------------------------------------------------
__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    uint32_t c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    c[0] = c0; c[1] = c1; c[2] = c2; c[3] = c3;
}

// ln(x) for x > 0 normal: range reduction to [sqrt(1/2), sqrt(2)] and the
// atanh series; + - * / only.
__host__ __device__ inline double det_log(double x) {
    uint64_t bits = __builtin_bit_cast(uint64_t, x);
    int e = (int)((bits >> 52) & 0x7ff) - 1023;
    double m = __builtin_bit_cast(double, (bits & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL);
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double z = s * s;
    double p = 2.0 / 19.0;
    p = p * z + 2.0 / 17.0;
    p = p * z + 2.0 / 15.0;
    p = p * z + 2.0 / 13.0;
    p = p * z + 2.0 / 11.0;
    p = p * z + 2.0 / 9.0;
    p = p * z + 2.0 / 7.0;
    p = p * z + 2.0 / 5.0;
    p = p * z + 2.0 / 3.0;
    double logm = 2.0 * s + s * (z * p);
    double de = (double)e;
    return de * 6.93147180369123816490e-01 + (de * 1.90821492927058770002e-10 + logm);
}

// ns-3 Seconds(double) -> int64 ns (round to nearest)
__host__ __device__ inline int64_t sec_to_ns(double s) { return (int64_t)(s * 1e9 + 0.5); }
// ns-3 Time::GetSeconds()
__host__ __device__ inline double ns_to_sec(int64_t t) { return (double)t / 1e9; }

// microseconds of std::to_string(GetSeconds()) (%f, ties-to-even on the
// exact binary value) as Python reads them back (packet-manager.cc:127-128).
__host__ __device__ inline uint64_t py_micros(int64_t t) {
    uint64_t u = (uint64_t)(t / 1000);
    int64_t r = t - (int64_t)u * 1000;
    if (r != 500) return r < 500 ? u : u + 1;
    double x = ns_to_sec(t);
    uint64_t b = __builtin_bit_cast(uint64_t, x);
    int ex = (int)((b >> 52) & 0x7ff);
    uint64_t mant = (b & 0x000fffffffffffffULL) | (ex ? 0x0010000000000000ULL : 0);
    if (!ex) ex = 1;
    int sh = 1075 - ex;                      // x = mant * 2^-sh, sh > 0 here
    // lhs = mant * 2e6 (< 2^75), rhs = (2u+1) << sh, compared as 128-bit
    const uint64_t k = 2000000ull;
    uint64_t lo = mant * k;
#ifdef __HIP_DEVICE_COMPILE__
    uint64_t hi = __umul64hi(mant, k);
#else
    uint64_t hi = (uint64_t)(((unsigned __int128)mant * k) >> 64);
#endif
    uint64_t v = 2 * u + 1, rhi, rlo;
    if (sh >= 64) { rhi = v << (sh - 64); rlo = 0; }
    else if (sh == 0) { rhi = 0; rlo = v; }
    else { rhi = v >> (64 - sh); rlo = v << sh; }
    if (hi != rhi) return hi > rhi ? u + 1 : u;
    if (lo != rlo) return lo > rlo ? u + 1 : u;
    return (u & 1) ? u + 1 : u;
}

__host__ __device__ inline double py_reward(int64_t t_now, uint32_t us_prev) {
    return (double)py_micros(t_now) / 1e6 - (double)us_prev / 1e6;
}

// ---------------------------------------------------------------------------
// device-side replica view
// ---------------------------------------------------------------------------
struct KParams {
    Layout lay;
    unsigned char* state;        // [R][state_bytes]
    const unsigned char* topo;   // [topo_bytes]
    unsigned char* log;          // [R][log_cap][rec_bytes]
    prisma_counters_t* cnt_out;  // [R]
    const int32_t* actions;      // [R] or null
    int32_t* obs_out;            // [R][W] or null
    uint8_t* mask_out;           // [R] or null
    int32_t* node_out;           // [R] or null
    const uint8_t* table;        // [N][N] or null
    int32_t R;
    int32_t max_hops;
    uint32_t episode;            // reset kernel only
    int32_t mode;                // 0 reset, 1 external step, 2 table run
};

// candidate key of one event source: 16 bytes, read with one ds_read_b128
struct __attribute__((aligned(16))) CKey {
    int64_t  t;
    uint32_t seq;
    uint32_t code;               // kind << 28 | index
};

// Lane-0 scalar state kept in registers for the whole event loop; it is
// loaded from / stored to the Hdr + counters of the LDS image at the loop
// boundaries only.
struct Hot {
    int64_t  now, ping_t;
    uint32_t ping_seq, seq, uid, dec, ping_rounds, episode;
    uint32_t pend, over, error, stop, hops_launch;
    uint64_t hops_total, events_total;
    prisma_counters_t c;
};

struct Sim {
    const Layout* L;
    unsigned char* base;         // LDS base
    Hdr* h;
    prisma_counters_t* c;
    uint32_t* obs;
    CKey* fkey; uint32_t* fdraw;
    CKey* lkey; LinkState* ln;
    int64_t* wt; uint32_t* wseq;
    uint4* ring;
    float* win; PingMeta* pm;
    const int32_t* rowptr; const int32_t* ldst; const int32_t* lrev;
    const int64_t* acctx;
    const int32_t* fsrc; const int32_t* fdst; const double* fmean;
    const uint8_t* table;
    unsigned char* logrep;       // this replica's log ring (HBM)
    uint32_t gid;                // global replica id
};

__device__ inline void sim_bind(Sim& S, const Layout& L, unsigned char* lds, unsigned char* logrep, uint32_t gid) {
    S.L = &L;
    S.base = lds;
    unsigned char* st = lds + L.topo_bytes;
    S.h = (Hdr*)(st + L.s_hdr);
    S.c = (prisma_counters_t*)(st + L.s_cnt);
    S.obs = (uint32_t*)(st + L.s_obs);
    S.fkey = (CKey*)(st + L.s_fkey);
    S.fdraw = (uint32_t*)(st + L.s_fdraw);
    S.lkey = (CKey*)(st + L.s_lkey);
    S.ln = (LinkState*)(st + L.s_link);
    S.wt = (int64_t*)(st + L.s_wt);
    S.wseq = (uint32_t*)(st + L.s_wseq);
    S.ring = (uint4*)(st + L.s_ring);
    S.win = (float*)(st + L.s_win);
    S.pm = (PingMeta*)(st + L.s_pmeta);
    S.rowptr = (const int32_t*)(lds + L.t_rowptr);
    S.ldst = (const int32_t*)(lds + L.t_ldst);
    S.lrev = (const int32_t*)(lds + L.t_lrev);
    S.acctx = (const int64_t*)(lds + L.t_acctx);
    S.fsrc = (const int32_t*)(lds + L.t_fsrc);
    S.fdst = (const int32_t*)(lds + L.t_fdst);
    S.fmean = (const double*)(lds + L.t_fmean);
    S.table = (const uint8_t*)(lds + L.t_table);
    S.logrep = logrep;
    S.gid = gid;
}

__device__ inline void hot_load(const Sim& S, Hot& H) {
    const Hdr& h = *S.h;
    H.now = h.now; H.ping_t = h.ping_t; H.ping_seq = h.ping_seq; H.seq = h.seq; H.uid = h.uid;
    H.dec = h.dec_count; H.ping_rounds = h.ping_rounds; H.episode = h.episode; H.pend = h.pend;
    H.over = h.over; H.error = h.error; H.stop = h.stop; H.hops_launch = h.hops_launch;
    H.hops_total = h.hops_total; H.events_total = h.events_total;
    H.c = *S.c;
}

__device__ inline void hot_store(Sim& S, const Hot& H) {
    Hdr& h = *S.h;
    h.now = H.now; h.ping_t = H.ping_t; h.ping_seq = H.ping_seq; h.seq = H.seq; h.uid = H.uid;
    h.dec_count = H.dec; h.ping_rounds = H.ping_rounds; h.episode = H.episode; h.pend = H.pend;
    h.over = H.over; h.error = H.error; h.stop = H.stop; h.hops_launch = H.hops_launch;
    h.hops_total = H.hops_total; h.events_total = H.events_total;
    prisma_counters_t c = H.c;
    c.now_ns = H.now; c.episode = H.episode; c.ping_rounds = H.ping_rounds; c.seq = H.seq; c.uid = H.uid;
    c.dec_count = H.dec; c.error = H.error; c.episode_over = H.over;
    c.hops_total = H.hops_total; c.events_total = H.events_total;
    *S.c = c;
}

__device__ inline void fail(Hot& H, uint32_t bit) {
    H.error |= bit;
    H.over = 1;
    H.stop = 1;
}

__device__ inline bool key_less(int64_t t, uint32_t s, int64_t bt, uint32_t bs) {
    return t < bt || (t == bt && s < bs);
}

// ---- link FIFO / transmitter (point-to-point-net-device.cc:273-336, 595-666)
__device__ inline uint32_t ent_size(const Layout& L, uint32_t x) {
    return ent_type(x) == T_DATA ? L.data_size : L.ping_size;
}
__device__ inline uint32_t ring_off(const Layout& L, int l) {
    return l < L.E ? (uint32_t)l * L.qcap_s : (uint32_t)L.E * L.qcap_s + (uint32_t)(l - L.E) * L.qcap_a;
}
__device__ inline uint32_t ring_cap(const Layout& L, int l) { return l < L.E ? L.qcap_s : L.qcap_a; }

// recompute the candidate key of link l: next tx completion or wire head
__device__ inline void relink(Sim& S, int l) {
    const LinkState& k = S.ln[l];
    CKey key;
    key.t = INT64_MAX; key.seq = 0xffffffffu; key.code = 0xffffffffu;
    if (k.busy) { key.t = k.complete_t; key.seq = k.complete_seq; key.code = (K_COMPLETE << 28) | (uint32_t)l; }
    if (k.n_wire) {
        uint32_t w = (uint32_t)l * S.L->WCAP + ((uint32_t)k.head & (uint32_t)(S.L->WCAP - 1));
        int64_t t = S.wt[w]; uint32_t s = S.wseq[w];
        if (key_less(t, s, key.t, key.seq)) { key.t = t; key.seq = s; key.code = (K_ARRIVE << 28) | (uint32_t)l; }
    }
    S.lkey[l] = key;
}

__device__ inline void transmit_start(Sim& S, Hot& H, int l, uint32_t ring_idx, uint32_t x) {
    const Layout& L = *S.L;
    LinkState& k = S.ln[l];
    int64_t tx = l < L.E ? (ent_type(x) == T_DATA ? L.sw_txd : L.sw_txp) : S.acctx[l - L.E];
    int64_t prop = l < L.E ? L.sw_prop : 0;
    k.busy = 1;
    k.complete_t = H.now + tx;
    k.complete_seq = H.seq++;                                  // TransmitComplete
    uint32_t w = (uint32_t)l * L.WCAP + (ring_idx & (uint32_t)(L.WCAP - 1));
    S.wt[w] = H.now + tx + prop;
    S.wseq[w] = H.seq++;                                       // channel Receive
    if (k.n_wire > (uint32_t)L.WCAP) fail(H, PRISMA_EBIT_WIRE);
}

// returns 1 if enqueued, 0 if dropped (or on ring overflow, which fails the replica)
__device__ inline int link_send(Sim& S, Hot& H, int l, uint4 e) {
    const Layout& L = *S.L;
    LinkState& k = S.ln[l];
    uint32_t size = ent_size(L, e.x);
    bool ok = l < L.E ? (k.q_bytes + size <= L.qmax_bytes) : ((uint32_t)k.n_queue + 1u <= L.acc_qmax_pkts);
    if (!ok) return 0;
    uint32_t cap = ring_cap(L, l), off = ring_off(L, l);
    if ((uint32_t)k.n_wire + k.n_queue + 1u > cap) { fail(H, PRISMA_EBIT_RING); return 0; }
    uint32_t ti = k.tail;
    S.ring[off + ti] = e;
    k.tail = (uint16_t)(ti + 1 == cap ? 0 : ti + 1);
    k.n_queue++;
    k.q_bytes += size;
    if (!k.busy) {                                              // :643-650
        uint32_t xi = k.txp;
        uint4 hd = S.ring[off + xi];
        k.txp = (uint16_t)(xi + 1 == cap ? 0 : xi + 1);
        k.n_queue--;
        k.n_wire++;
        k.q_bytes -= ent_size(L, hd.x);
        transmit_start(S, H, l, xi, hd.x);
        relink(S, l);
    }
    return 1;
}

__device__ inline void on_complete(Sim& S, Hot& H, int l) {         // :305-336
    const Layout& L = *S.L;
    LinkState& k = S.ln[l];
    k.busy = 0;
    if (k.n_queue) {
        uint32_t cap = ring_cap(L, l);
        uint32_t xi = k.txp;
        uint4 hd = S.ring[ring_off(L, l) + xi];
        k.txp = (uint16_t)(xi + 1 == cap ? 0 : xi + 1);
        k.n_queue--;
        k.n_wire++;
        k.q_bytes -= ent_size(L, hd.x);
        transmit_start(S, H, l, xi, hd.x);
    }
    relink(S, l);
}

// ---- observation (data-packet-manager.cc:171-206)
__device__ inline uint32_t ping_value(const Sim& S, const Hot& H, int l) {
    const PingMeta& m = S.pm[l];
    double avg = 0.0;
    if (m.win_n > 0) {
        double sum = 0.0;
        uint32_t MA = S.L->ma;
        uint32_t i = m.win_head;
        for (uint32_t j = 0; j < m.win_n; ++j) {
            sum += (double)S.win[(uint32_t)l * MA + i];
            i = (i + 1 == MA) ? 0 : i + 1;
        }
        avg = sum / (double)m.win_n;
    }
    // oldest unacknowledged ping (ping-back-packet-manager.cc:110-116):
    // acknowledgements of one tunnel arrive in index order, so the oldest
    // pending entry is the first hole below the last ack, else the ping
    // after the last ack if it was sent.
    int64_t oldest = -1;
    if (m.first_hole >= 0) oldest = m.first_hole;
    else if ((int64_t)m.acked_last + 1 < (int64_t)H.ping_rounds) oldest = (int64_t)m.acked_last + 1;
    float mt = 0.0f;
    if (oldest >= 0) {
        uint64_t ms = (uint64_t)(((oldest + 1) * S.L->ping_period) / 1000000);
        double a = ns_to_sec(H.now) - (double)ms * 0.001;
        double b = 2.60;
        mt = (float)((b < a) ? b : a);
    }
    double mx = (avg < (double)mt) ? (double)mt : avg;
    return (uint32_t)(1000 * mx);
}

__device__ inline void observe(Sim& S, const Hot& H, int v, uint32_t dst) {
    const int W = S.L->W;
    int r0 = S.rowptr[v], r1 = S.rowptr[v + 1];
    S.obs[0] = dst;
    for (int i = 1; i < W; ++i) {
        int l = r0 + i - 1;
        S.obs[i] = l < r1 ? (S.L->ping_as_obs ? ping_value(S, H, l) : S.ln[l].q_bytes) : 0u;
    }
}

__device__ inline unsigned char* rec_ptr(const Sim& S, uint32_t d) {
    return S.logrep + (size_t)(d & (S.L->log_cap - 1)) * S.L->rec_bytes;
}

__device__ inline void write_record(Sim& S, const Hot& H, uint32_t d, double reward, uint32_t uid, int32_t prev,
                                    uint32_t node, uint32_t dst, int action, uint32_t status) {
    unsigned char* p = rec_ptr(S, d);
    uint4 a, b;
    a.x = (uint32_t)H.now; a.y = (uint32_t)((uint64_t)H.now >> 32);
    uint64_t rb = __double_as_longlong(reward);
    a.z = (uint32_t)rb; a.w = (uint32_t)(rb >> 32);
    b.x = uid; b.y = (uint32_t)prev; b.z = node | (dst << 16);
    b.w = (uint32_t)(uint8_t)(int8_t)action | (status << 8) | ((H.episode & 0xffffu) << 16);
    *(uint4*)(p + 0) = a;
    *(uint4*)(p + 16) = b;
    const uint4* o = (const uint4*)S.obs;
    for (int i = 0; i < S.L->W / 4; ++i) ((uint4*)(p + 32))[i] = o[i];
    if (S.L->W & 2) *(uint2*)(p + 32 + 16 * (S.L->W / 4)) = *(const uint2*)(S.obs + 4 * (S.L->W / 4));
}

__device__ inline void patch_record(Sim& S, const Hot& H, uint32_t d, int action, uint32_t status) {
    unsigned char* p = rec_ptr(S, d);
    *(uint32_t*)(p + 28) = (uint32_t)(uint8_t)(int8_t)action | (status << 8) | ((H.episode & 0xffffu) << 16);
}

// Receive tail after the MacRx trace (point-to-point-net-device.cc:430-463)
__device__ inline void receive_counters(const Layout& L, Hot& H, uint32_t x, int v) {
    prisma_counters_t& c = H.c;
    uint32_t type = ent_type(x);
    if (type == T_DATA && ent_dst(x) == (uint32_t)v) {
        // valable, nextHop == finalDest on identity overlays
        c.ov_arrived++;
        float cost = (float)(ns_to_sec(H.now) - (double)ent_aux(x));
        c.cost_sum += cost; c.cost_n++;
        c.e2e_sum += cost; c.e2e_n++;
    }
    if (type > 0 && ent_dst(x) == (uint32_t)v) c.bytes_signaling += (int32_t)(L.ping_size - 2);
    if (type == T_DATA && ent_fresh(x)) {
        c.ov_injected++;
        c.bytes_data += (int32_t)(L.data_size - 2);
    }
}

// DataPacketManager::sendPacket (data-packet-manager.cc:251-299) for the
// decision held in (e, v, d), then the Receive tail.  `fused` = the record
// was not written yet (table policy: one record write per decision).
__device__ inline void apply_decision(Sim& S, Hot& H, uint4 e, int v, uint32_t d, int action, bool fused,
                                      double reward, int32_t prev) {
    const Layout& L = *S.L;
    int r0 = S.rowptr[v], deg = S.rowptr[v + 1] - r0;
    uint32_t status;
    if (action >= 0 && action < deg) {
        int l = r0 + action;
        uint4 f;
        f.x = ent_make(T_DATA, ent_src(e.x), ent_dst(e.x), 0u, 1u, ent_aux(e.x));
        f.y = e.y;                                   // uid
        f.z = d;                                     // decision of this hop
        f.w = (uint32_t)py_micros(H.now);            // temp_obs time
        H.c.hops++;
        H.c.hop_deg_sum += (uint64_t)deg;
        if (link_send(S, H, l, f)) {
            status = PRISMA_ST_ENQUEUED;
        } else {
            status = PRISMA_ST_DROPPED;              // :655-664 + forwarder.py:214-244
            H.c.ov_lost++;
            H.c.cost_sum += L.loss_penalty_f;
            H.c.cost_n++;
            H.c.reward_sum += L.loss_penalty;
        }
    } else {
        status = PRISMA_ST_DISCARDED;
    }
    if (fused) write_record(S, H, d, reward, e.y, prev, (uint32_t)v, ent_dst(e.x), action, status);
    else patch_record(S, H, d, action, status);
    receive_counters(L, H, e.x, v);
}

__device__ inline void finish_pending(Sim& S, Hot& H, int action) {
    Hdr& h = *S.h;
    uint4 e = make_uint4(h.pend_ent[0], h.pend_ent[1], h.pend_ent[2], h.pend_ent[3]);
    apply_decision(S, H, e, (int)h.pend_node, h.pend_dec, action, false, 0.0, 0);
    H.pend = 0;
}

// ---- handlers (lane 0) ------------------------------------------------------
__device__ inline void on_ping_round(Sim& S, Hot& H) {              // data-packet-manager.cc:350-413
    const Layout& L = *S.L;
    uint32_t k = H.ping_rounds;
    uint32_t ms = (uint32_t)(H.now / 1000000);
    uint32_t first_rearm = 0;
    for (int u = 0; u < L.N; ++u) {
        int r0 = S.rowptr[u], r1 = S.rowptr[u + 1];
        for (int l = r0; l < r1; ++l) {
            uint4 e;
            e.x = ent_make(T_PING_FWD, (uint32_t)u, (uint32_t)S.ldst[l], 0u, 0u, (uint32_t)(l - r0));
            e.y = k;
            e.z = ms;
            e.w = 0;
            if (!link_send(S, H, l, e)) H.c.ctrl_dropped++;
        }
        uint32_t s = H.seq++;                                    // re-arm of node u
        if (u == 0) first_rearm = s;
    }
    H.ping_rounds = k + 1;
    // one ns-3 event per node timer (the round is N consecutive events)
    H.c.events += (uint64_t)(L.N - 1);
    H.events_total += (uint64_t)(L.N - 1);
    H.ping_t = H.now + L.ping_period;
    H.ping_seq = first_rearm;
}

__device__ inline void flow_next(Sim& S, Hot& H, int f) {           // poisson-application.cc:265-295
    uint32_t draw = S.fdraw[f];
    uint32_t c[4] = { (uint32_t)f, draw, H.episode, 1u };
    philox4x32_10(c, S.L->seed_lo, S.gid);
    uint64_t u53 = ((uint64_t)(c[0] >> 5) << 26) | (uint64_t)(c[1] >> 6);
    double U = ((double)u53 + 1.0) * (1.0 / 9007199254740992.0);
    double delay = -S.fmean[f] * det_log(U);
    S.fdraw[f] = draw + 1;
    CKey key;
    key.t = H.now + sec_to_ns(delay);
    key.seq = H.seq++;
    key.code = (K_FLOW << 28) | (uint32_t)f;
    S.fkey[f] = key;
}

__device__ inline void on_flow(Sim& S, Hot& H, int f) {
    if (S.fdraw[f] != 0) {                                          // SendPacket :297-358
        uint32_t src = (uint32_t)S.fsrc[f];
        uint4 e;
        e.x = ent_make(T_DATA, src, (uint32_t)S.fdst[f], 1u, 1u, (uint32_t)(H.now / 1000000000));
        e.y = H.uid++;
        e.z = 0xffffffffu;
        e.w = 0;
        link_send(S, H, S.L->E + (int)src, e);                      // access link
    }
    flow_next(S, H, f);                                             // StartSending / ScheduleNextTx
}

// Returns 1 if a data decision needs an action (its entry/node/record in *pe/*pv/*pd).
__device__ inline int on_arrive(Sim& S, Hot& H, int l, uint4* pe, int* pv, uint32_t* pd, double* prew,
                                int32_t* pprev, bool fused) {
    const Layout& L = *S.L;
    LinkState& k = S.ln[l];
    uint32_t cap = ring_cap(L, l);
    uint32_t hi = k.head;
    uint4 e = S.ring[ring_off(L, l) + hi];
    k.head = (uint16_t)(hi + 1 == cap ? 0 : hi + 1);
    k.n_wire--;
    relink(S, l);
    int v = S.ldst[l];
    uint32_t type = ent_type(e.x);
    if (type == T_DATA) {
        // PacketRoutingEnv::NotifyPktRcv -> Notify (packet-routing-gym.cc:231-267)
        uint32_t dst = ent_dst(e.x);
        uint32_t d = H.dec++;
        double reward = 0.0;
        int32_t prev = -1;
        if (!ent_fresh(e.x)) {
            prev = (int32_t)e.z;
            reward = py_reward(H.now, e.w);                        // forwarder.py:360
            H.c.reward_sum += reward;
        }
        observe(S, H, v, dst);
        H.c.decisions++;
        if (dst == (uint32_t)v) {                                   // getGameOver
            write_record(S, H, d, reward, e.y, prev, (uint32_t)v, dst, -1, PRISMA_ST_DESTINATION);
            receive_counters(L, H, e.x, v);
            return 0;
        }
        if (!fused) write_record(S, H, d, reward, e.y, prev, (uint32_t)v, dst, -1, PRISMA_ST_PENDING);
        *pe = e; *pv = v; *pd = d; *prew = reward; *pprev = prev;
        return 1;
    }
    if (type == T_PING_FWD) {                                       // ping-forward-packet-manager.cc:94-156
        float delay = (float)(ns_to_sec(H.now) - ((double)e.z * 0.001));
        uint4 b;
        b.x = ent_make(T_PING_BACK, (uint32_t)v, ent_src(e.x), 0u, 0u, ent_aux(e.x));
        b.y = e.y;
        b.z = __float_as_uint(delay);
        b.w = 0;
        if (!link_send(S, H, S.lrev[l], b)) H.c.ctrl_dropped++;
    } else if (type == T_PING_BACK) {                               // ping-back-packet-manager.cc:120-144
        int lt = S.rowptr[v] + (int)ent_aux(e.x);
        PingMeta& m = S.pm[lt];
        int32_t idx = (int32_t)e.y;
        if (idx <= m.acked_last) {
            fail(H, PRISMA_EBIT_ACKORDER);
        } else {
            if (idx > m.acked_last + 1 && m.first_hole < 0) m.first_hole = m.acked_last + 1;
            m.acked_last = idx;
        }
        uint32_t MA = L.ma;
        uint32_t slot;
        if (m.win_n >= MA) {
            slot = m.win_head;
            m.win_head = (m.win_head + 1 == MA) ? 0 : m.win_head + 1;
        } else {
            slot = m.win_head + m.win_n;
            if (slot >= MA) slot -= MA;
            m.win_n++;
        }
        S.win[(uint32_t)lt * MA + slot] = __uint_as_float(e.z);
    }
    receive_counters(L, H, e.x, v);
    return 0;
}

// ---------------------------------------------------------------------------
// replica (re)initialisation: all lanes, operates on the LDS image
// ---------------------------------------------------------------------------
__device__ void init_replica(Sim& S, int lane, uint32_t episode) {
    const Layout& L = *S.L;
    uint32_t dec = S.h->dec_count;                 // monotonic across episodes
    uint64_t ht = S.h->hops_total, et = S.h->events_total;
    uint32_t hl = S.h->hops_launch;                // per-launch budget survives resets
    __syncthreads();
    uint4* st4 = (uint4*)(S.base + L.topo_bytes);
    for (uint32_t i = (uint32_t)lane; i < L.state_bytes / 16u; i += kWave) st4[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (int f = lane; f < L.F; f += kWave) {
        uint32_t c[4] = { (uint32_t)f, 0u, episode, 0u };
        philox4x32_10(c, L.seed_lo, S.gid);
        uint64_t u53 = ((uint64_t)(c[0] >> 5) << 26) | (uint64_t)(c[1] >> 6);
        double U = (double)u53 * (1.0 / 9007199254740992.0);
        CKey key;
        key.t = sec_to_ns(0.0001 + U);                             // sim.cc:610-630
        key.seq = (uint32_t)(L.N + f);
        key.code = (K_FLOW << 28) | (uint32_t)f;
        S.fkey[f] = key;
        S.fdraw[f] = 0;
    }
    for (int l = lane; l < L.E; l += kWave) {
        S.pm[l].acked_last = -1;
        S.pm[l].first_hole = -1;
    }
    for (int l = lane; l < L.L; l += kWave) {
        CKey key;
        key.t = INT64_MAX; key.seq = 0xffffffffu; key.code = 0xffffffffu;
        S.lkey[l] = key;
    }
    if (lane == 0) {
        Hdr& h = *S.h;
        h.now = 0;
        h.ping_t = L.ping_period;                                  // data-packet-manager.cc:118-121
        h.ping_seq = 0;
        h.seq = (uint32_t)(L.N + L.F);
        h.dec_count = dec;
        h.hops_total = ht;
        h.events_total = et;
        h.hops_launch = hl;
        h.episode = episode;
        S.c->episode = episode;
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// wave-wide event selection: per-lane min over owned candidate keys, then a
// DPP reduction of the 64-bit time to lane 63; the (rare) same-ns ties are
// resolved by a second reduction of seq over the tied lanes.
// ---------------------------------------------------------------------------
template <int CTRL, int ROW_MASK>
__device__ inline uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROW_MASK, 0xf, false);
}

template <int CTRL, int ROW_MASK>
__device__ inline int64_t dpp_min_i64(int64_t v) {
    uint32_t lo = dpp_u32<CTRL, ROW_MASK>((uint32_t)v);
    uint32_t hi = dpp_u32<CTRL, ROW_MASK>((uint32_t)((uint64_t)v >> 32));
    int64_t o = (int64_t)(((uint64_t)hi << 32) | lo);
    return o < v ? o : v;
}

template <int CTRL, int ROW_MASK>
__device__ inline uint32_t dpp_min_u32(uint32_t v) {
    uint32_t o = dpp_u32<CTRL, ROW_MASK>(v);
    return o < v ? o : v;
}

__device__ inline int64_t wave_min_i64(int64_t v) {
    v = dpp_min_i64<0xB1, 0xF>(v);      // quad_perm [1,0,3,2]
    v = dpp_min_i64<0x4E, 0xF>(v);      // quad_perm [2,3,0,1]
    v = dpp_min_i64<0x141, 0xF>(v);     // row_half_mirror
    v = dpp_min_i64<0x140, 0xF>(v);     // row_mirror
    v = dpp_min_i64<0x142, 0xA>(v);     // row_bcast:15
    v = dpp_min_i64<0x143, 0xC>(v);     // row_bcast:31
    uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), 63);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ inline uint32_t wave_min_u32(uint32_t v) {
    v = dpp_min_u32<0xB1, 0xF>(v);
    v = dpp_min_u32<0x4E, 0xF>(v);
    v = dpp_min_u32<0x141, 0xF>(v);
    v = dpp_min_u32<0x140, 0xF>(v);
    v = dpp_min_u32<0x142, 0xA>(v);
    v = dpp_min_u32<0x143, 0xC>(v);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ inline void select_event(const Sim& S, const Hot& H, int lane, int64_t& bt, uint32_t& bc) {
    const Layout& L = *S.L;
    int64_t t = INT64_MAX;
    uint32_t s = 0xffffffffu, c = 0xffffffffu;
    for (int f = lane; f < L.F; f += kWave) {
        CKey k = S.fkey[f];
        if (key_less(k.t, k.seq, t, s)) { t = k.t; s = k.seq; c = k.code; }
    }
    for (int l = lane; l < L.L; l += kWave) {
        CKey k = S.lkey[l];
        if (key_less(k.t, k.seq, t, s)) { t = k.t; s = k.seq; c = k.code; }
    }
    if (lane == 0 && key_less(H.ping_t, H.ping_seq, t, s)) { t = H.ping_t; s = H.ping_seq; c = K_PING << 28; }
    const int64_t tmin = wave_min_i64(t);
    uint64_t tied = __ballot(t == tmin);
    int win;
    if ((tied & (tied - 1)) == 0) {
        win = __builtin_ctzll(tied);
    } else {                                                        // same-ns events: ns-3 uid order
        uint32_t smin = wave_min_u32(t == tmin ? s : 0xffffffffu);
        win = __builtin_ctzll(__ballot(t == tmin && s == smin));
    }
    bt = tmin;
    bc = (uint32_t)__builtin_amdgcn_readlane((int)c, win);
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
__device__ inline void stage_in(unsigned char* lds, const KParams& P, int r, int lane) {
    const Layout& L = P.lay;
    const uint4* t4 = (const uint4*)P.topo;
    uint4* l4 = (uint4*)lds;
    for (uint32_t i = (uint32_t)lane; i < L.topo_bytes / 16u; i += kWave) l4[i] = t4[i];
    if (P.table && L.table_bytes) {
        uint8_t* dstp = lds + L.t_table;
        const uint32_t nt = (uint32_t)(L.N * L.N);
        for (uint32_t i = (uint32_t)lane; i < nt; i += kWave) dstp[i] = P.table[i];
    }
    const uint4* s4 = (const uint4*)(P.state + (size_t)r * L.state_bytes);
    uint4* d4 = (uint4*)(lds + L.topo_bytes);
    for (uint32_t i = (uint32_t)lane; i < L.state_bytes / 16u; i += kWave) d4[i] = s4[i];
}

__device__ inline void stage_out(unsigned char* lds, const KParams& P, int r, int lane) {
    const Layout& L = P.lay;
    uint4* s4 = (uint4*)(P.state + (size_t)r * L.state_bytes);
    const uint4* d4 = (const uint4*)(lds + L.topo_bytes);
    for (uint32_t i = (uint32_t)lane; i < L.state_bytes / 16u; i += kWave) s4[i] = d4[i];
}

__device__ inline void publish_counters(Sim& S, const KParams& P, int r, int lane) {
    const uint32_t* src = (const uint32_t*)S.c;
    uint32_t* dst = (uint32_t*)(P.cnt_out + r);
    if (lane < (int)(sizeof(prisma_counters_t) / 4)) dst[lane] = src[lane];
}

extern "C" __global__ void __launch_bounds__(64) prisma_reset_kernel(KParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int r = blockIdx.x, lane = threadIdx.x;
    const Layout& L = P.lay;
    const uint4* t4 = (const uint4*)P.topo;
    uint4* l4 = (uint4*)lds;
    for (uint32_t i = (uint32_t)lane; i < L.topo_bytes / 16u; i += kWave) l4[i] = t4[i];
    Sim S;
    sim_bind(S, L, lds, P.log + (size_t)r * L.log_cap * L.rec_bytes, L.replica_base + (uint32_t)r);
    if (lane == 0) { S.h->dec_count = 0; S.h->hops_total = 0; S.h->events_total = 0; S.h->hops_launch = 0; }
    init_replica(S, lane, P.episode);
    if (lane == 0) {
        Hot H;
        hot_load(S, H);
        hot_store(S, H);
    }
    __syncthreads();
    publish_counters(S, P, r, lane);
    stage_out(lds, P, r, lane);
}

extern "C" __global__ void __launch_bounds__(64) prisma_step_kernel(KParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int r = blockIdx.x, lane = threadIdx.x;
    const Layout& L = P.lay;
    stage_in(lds, P, r, lane);
    __syncthreads();
    Sim S;
    sim_bind(S, L, lds, P.log + (size_t)r * L.log_cap * L.rec_bytes, L.replica_base + (uint32_t)r);
    const bool table_mode = (P.mode == 2);
    const uint32_t max_hops = (uint32_t)P.max_hops;
    const uint32_t NN = (uint32_t)L.N;
    Hot H;
    hot_load(S, H);                                    // every lane holds a copy; lane 0 owns it

    if (lane == 0) {
        H.stop = 0;
        H.hops_launch = 0;
        if (H.pend && !H.over) {
            if (table_mode) {
                finish_pending(S, H, (int)S.table[S.h->pend_node * NN + ent_dst(S.h->pend_ent[0])]);
                H.hops_launch++;
                H.hops_total++;
            } else if (P.actions) {
                finish_pending(S, H, (int)P.actions[r]);
            } else {
                H.stop = 1;                            // nothing to apply: re-emit the pending obs
            }
        }
        if (H.over || (table_mode && H.hops_launch >= max_hops)) H.stop = 1;
    }
    __syncthreads();
    uint32_t stop = (uint32_t)__builtin_amdgcn_readfirstlane((int)H.stop);
    uint32_t resets = 0;
    while (!stop) {
        int64_t bt;
        uint32_t bc;
        select_event(S, H, lane, bt, bc);
        if (bt >= L.t_end) {                           // Simulator::Stop(simTime) (sim.cc:703)
            if (L.auto_reset && resets < 64u) {        // bounded: an empty scenario cannot spin forever
                ++resets;
                if (lane == 0) hot_store(S, H);
                init_replica(S, lane, H.episode + 1u);
                hot_load(S, H);
                continue;
            }
            if (lane == 0) { H.over = 1; H.stop = 1; }
            break;
        }
        if (lane == 0) {
            H.now = bt;
            H.c.events++;
            H.events_total++;
            const uint32_t kind = bc >> 28, id = bc & 0x0fffffffu;
            if (kind == K_ARRIVE) {
                uint4 e; int v; uint32_t d; double rw; int32_t pv;
                if (on_arrive(S, H, (int)id, &e, &v, &d, &rw, &pv, table_mode)) {
                    if (table_mode) {
                        apply_decision(S, H, e, v, d, (int)S.table[(uint32_t)v * NN + ent_dst(e.x)], true, rw, pv);
                        H.hops_launch++;
                        H.hops_total++;
                        if (H.hops_launch >= max_hops) H.stop = 1;
                    } else {
                        Hdr& h = *S.h;
                        h.pend_link = id; h.pend_node = (uint32_t)v; h.pend_dec = d;
                        h.pend_ent[0] = e.x; h.pend_ent[1] = e.y; h.pend_ent[2] = e.z; h.pend_ent[3] = e.w;
                        H.pend = 1;
                        H.stop = 1;
                    }
                }
            } else if (kind == K_COMPLETE) {
                on_complete(S, H, (int)id);
            } else if (kind == K_FLOW) {
                on_flow(S, H, (int)id);
            } else {
                on_ping_round(S, H);
            }
            if (H.error) { H.over = 1; H.stop = 1; }
        }
        __syncthreads();
        stop = (uint32_t)__builtin_amdgcn_readfirstlane((int)H.stop);
    }

    if (lane == 0) hot_store(S, H);
    __syncthreads();
    const bool pending = S.h->pend && !S.h->over;
    if (P.mask_out && lane == 0) P.mask_out[r] = pending ? 1 : 0;
    if (P.node_out && lane == 0) P.node_out[r] = pending ? (int32_t)S.h->pend_node : -1;
    if (P.obs_out && lane < L.W) P.obs_out[(size_t)r * L.W + lane] = pending ? (int32_t)S.obs[lane] : 0;
    publish_counters(S, P, r, lane);
    stage_out(lds, P, r, lane);
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
    bool reset_done = false;
};

static thread_local std::string g_err;
static int set_err(int code, const std::string& msg) { g_err = msg; return code; }

extern "C" int prisma_abi_version(void) { return PRISMA_ABI_VERSION; }
extern "C" const char* prisma_last_error(void) { return g_err.c_str(); }

static uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }
static uint32_t next_pow2(uint32_t x) { uint32_t p = 1; while (p < x) p <<= 1; return p; }

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
    if (maxdeg != T->max_deg) return set_err(PRISMA_ERR_CONFIG, "max_deg mismatch");
    if (maxdeg > 127) return set_err(PRISMA_ERR_CONFIG, "degree above 127");
    for (int f = 0; f < F; ++f) {
        if (T->flow_src[f] < 0 || T->flow_src[f] >= N || T->flow_dst[f] < 0 || T->flow_dst[f] >= N ||
            T->flow_src[f] == T->flow_dst[f] || T->flow_rate_bps[f] == 0)
            return set_err(PRISMA_ERR_CONFIG, "bad flow");
    }
    if (P->link_bps == 0 || P->link_delay_ns < 0 || P->max_buffer_bytes == 0 || P->packet_size == 0 ||
        P->ma_size == 0 || P->ma_size > 64 || !(P->ping_interval_s > 0.0f))
        return set_err(PRISMA_ERR_CONFIG, "bad link / ping parameters");
    if (!(P->sim_time_s > 0.0) || P->sim_time_s > 2047.0)
        return set_err(PRISMA_ERR_CONFIG, "sim_time_s must be in (0, 2047] (11-bit packet start second)");
    if (P->log_capacity < 64 || (P->log_capacity & (P->log_capacity - 1)))
        return set_err(PRISMA_ERR_CONFIG, "log_capacity must be a power of two >= 64");

    memset(&L, 0, sizeof(L));
    const int Lk = E + N;
    L.N = N; L.E = E; L.L = Lk; L.F = F; L.max_deg = maxdeg;
    L.W = (1 + maxdeg + 3) & ~3;                    // obs width: multiple of 4 (16-B record rows)
    L.MA = (int)P->ma_size;
    L.data_size = P->packet_size + 30u;             // UDP 8 + IP 20 + PPP 2
    L.ping_size = 8u + 30u;
    // link constants (sim.cc:398-433): switch links share rate, delay and queue
    L.sw_txd = sec_to_ns((double)L.data_size * 8 / (double)P->link_bps);
    L.sw_txp = sec_to_ns((double)L.ping_size * 8 / (double)P->link_bps);
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
    if (L.sw_txp < 1) return set_err(PRISMA_ERR_CONFIG, "link too fast for the wire model");
    uint32_t wire = (uint32_t)(P->link_delay_ns / L.sw_txp) + 2u;
    L.WCAP = (int)next_pow2(wire < 2 ? 2 : wire);
    if (L.WCAP > 64) return set_err(PRISMA_ERR_CONFIG, "propagation delay too long for the wire model");
    // ring capacity: full byte-limited FIFO of data + the control packets that
    // can be queued at once (<= 2 pings per round over the FIFO's drain time)
    double drain_s = (double)P->max_buffer_bytes * 8.0 / (double)P->link_bps + (double)L.sw_txd * 1e-9;
    double span = 2.0 * drain_s + 2.0 * (double)P->link_delay_ns * 1e-9;
    uint32_t ctrl = 2u * ((uint32_t)(span / (double)P->ping_interval_s) + 3u);
    uint32_t qs = P->max_buffer_bytes / L.data_size + ctrl + (uint32_t)L.WCAP;
    qs = (qs + (uint32_t)L.WCAP - 1) / (uint32_t)L.WCAP * (uint32_t)L.WCAP;
    if (qs > 65535u) return set_err(PRISMA_ERR_CONFIG, "queue too deep");
    L.qcap_s = qs;
    L.qcap_a = (uint32_t)(L.WCAP < 8 ? 8 : L.WCAP);
    uint32_t tot = (uint32_t)E * L.qcap_s + (uint32_t)N * L.qcap_a;

    // topology image
    uint32_t o = 0;
    auto take = [&](uint32_t bytes) { uint32_t r = o; o = align16(o + bytes); return r; };
    L.t_rowptr = take(4u * (N + 1));
    L.t_ldst = take(4u * Lk);
    L.t_lrev = take(4u * E);
    L.t_acctx = take(8u * N);
    L.t_fsrc = take(4u * F);
    L.t_fdst = take(4u * F);
    L.t_fmean = take(8u * F);
    L.t_table = take((uint32_t)(N * N));
    L.table_bytes = (uint32_t)(N * N);
    L.topo_bytes = o;
    topo.assign(o, 0);
    memcpy(&topo[L.t_rowptr], T->row_ptr, 4u * (N + 1));
    memcpy(&topo[L.t_ldst], ldst.data(), 4u * Lk);
    memcpy(&topo[L.t_lrev], T->link_rev, 4u * E);
    memcpy(&topo[L.t_acctx], acctx.data(), 8u * N);
    memcpy(&topo[L.t_fsrc], T->flow_src, 4u * F);
    memcpy(&topo[L.t_fdst], T->flow_dst, 4u * F);
    std::vector<double> fmean(F);
    for (int f = 0; f < F; ++f)                      // poisson-application.cc:280-283
        fmean[f] = (double)(P->packet_size * 8u) / (double)T->flow_rate_bps[f];
    memcpy(&topo[L.t_fmean], fmean.data(), 8u * F);

    // state image
    o = 0;
    L.s_hdr = take(sizeof(Hdr));
    L.s_cnt = take(sizeof(prisma_counters_t));
    L.s_obs = take(4u * L.W);
    L.s_fkey = take(16u * F);
    L.s_fdraw = take(4u * F);
    L.s_lkey = take(16u * Lk);
    L.s_link = take(sizeof(LinkState) * Lk);
    L.s_wt = take(8u * Lk * L.WCAP);
    L.s_wseq = take(4u * Lk * L.WCAP);
    L.s_ring = take(16u * tot);
    L.s_win = take(4u * E * L.MA);
    L.s_pmeta = take(sizeof(PingMeta) * E);
    L.state_bytes = o;
    L.lds_bytes = L.topo_bytes + L.state_bytes;
    if (L.lds_bytes > 160u * 1024u)
        return set_err(PRISMA_ERR_CONFIG, "replica state exceeds the 160 KiB LDS of a gfx950 CU");

    L.t_end = sec_to_ns(P->sim_time_s);
    L.ping_period = sec_to_ns((double)P->ping_interval_s);     // Seconds(float) (sim.cc:173)
    L.ma = P->ma_size;
    L.ping_as_obs = P->ping_as_obs ? 1u : 0u;
    L.auto_reset = P->auto_reset ? 1u : 0u;
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
        !HIP_OK(hipMalloc((void**)&e->d_cnt, sizeof(prisma_counters_t) * n_replicas))) {
        prisma_destroy(e);
        return set_err(PRISMA_ERR_NOMEM, "hipMalloc failed");
    }
    if (!HIP_OK(hipMemcpy(e->d_topo, img.data(), L.topo_bytes, hipMemcpyHostToDevice)) ||
        !HIP_OK(hipMemset(e->d_log, 0, lb)) ||
        !HIP_OK(hipMemset(e->d_cnt, 0, sizeof(prisma_counters_t) * n_replicas))) {
        prisma_destroy(e);
        return set_err(PRISMA_ERR_DEVICE, "device initialisation failed");
    }
    (void)hipFuncSetAttribute((const void*)prisma_step_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds_bytes);
    (void)hipFuncSetAttribute((const void*)prisma_reset_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds_bytes);
    *out = e;
    return PRISMA_OK;
}

static KParams base_params(prisma_env_t* e) {
    KParams P;
    memset(&P, 0, sizeof(P));
    P.lay = e->lay;
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
    hipError_t err = hipLaunchKernel(kern, dim3((unsigned)e->R), dim3(kWave), args, e->lay.lds_bytes, (hipStream_t)stream);
    if (err == hipSuccess) err = hipGetLastError();
    if (err != hipSuccess) return set_err(PRISMA_ERR_LAUNCH, std::string("kernel launch failed: ") + hipGetErrorString(err));
    return PRISMA_OK;
}

extern "C" int prisma_reset(prisma_env_t* e, uint32_t episode, void* stream) {
    if (!e) return set_err(PRISMA_ERR_ARG, "null env");
    KParams P = base_params(e);
    P.mode = 0;
    P.episode = episode;
    int rc = launch(e, (const void*)prisma_reset_kernel, P, stream);
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
    return launch(e, (const void*)prisma_step_kernel, P, stream);
}

extern "C" int prisma_run(prisma_env_t* e, int32_t policy, const uint8_t* table, int32_t max_hops, void* stream) {
    if (!e) return set_err(PRISMA_ERR_ARG, "null env");
    if (!e->reset_done) return set_err(PRISMA_ERR_STATE, "prisma_reset must be called first");
    if (policy != PRISMA_POLICY_TABLE || !table) return set_err(PRISMA_ERR_ARG, "policy must be PRISMA_POLICY_TABLE with a device table");
    if (max_hops < 1) return set_err(PRISMA_ERR_ARG, "max_hops must be >= 1");
    KParams P = base_params(e);
    P.mode = 2;
    P.table = table;
    P.max_hops = max_hops;
    return launch(e, (const void*)prisma_step_kernel, P, stream);
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

extern "C" void prisma_destroy(prisma_env_t* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->d_state) (void)hipFree(e->d_state);
    if (e->d_topo) (void)hipFree(e->d_topo);
    if (e->d_log) (void)hipFree(e->d_log);
    if (e->d_cnt) (void)hipFree(e->d_cnt);
    delete e;
}
