// prisma_engine_mem.hip — the memory-resident gfx950 engine.
//
// For topologies beyond the register-resident engine (more than 255 nodes,
// 256 links or 512 flows: the Erdos-Renyi 256-node config, 2 304 links and
// 65 280 flows per replica) the replica state lives in HBM and one 64-lane
// wavefront still owns one replica and runs the same event handlers
// (engine_core.h), over a different store (MemSt):
//   * one 128-byte record per link (FIFO pointers, queued bytes, completion and
//     wire-head keys, ping state of the link's tunnel, 8 wire slots), read and
//     written by every lane as uniform 16-B accesses;
//   * the next event of every source (links, then flows) as a 16-byte leaf key
//     {time lo, time hi, seq, aux} in HBM, under a 64-ary tournament tree whose
//     two upper levels (block and super-block minima) sit in LDS.  A source's
//     update re-reduces its 64-leaf block (one coalesced 1 KiB load + a DPP
//     reduction) only when the block minimum can change, and the level above
//     likewise; choosing the next event reduces <= 64 super-block minima;
//   * FIFO rings, ping windows and ping-back delays in HBM (ring offsets as in
//     the register-resident engine).
// The header, counters and pending observation stay in LDS (staged per launch).
#include "engine_core.h"

// ---------------------------------------------------------------------------
// store
// ---------------------------------------------------------------------------
struct MemSt {
    uint32_t* lrec;              // [L][kLRec]
    uint4* keys;                 // [n_leaf] {t lo, t hi, seq, aux}: aux = kind (links) / draw (flows)
    uint4* lv1;                  // LDS [n1] {t lo, t hi, seq, code}
    uint4* lv2;                  // LDS [n2]
    uint32_t L, n_leaf, n1, n2;
};

constexpr int64_t kInf = INT64_MAX;

__device__ __forceinline__ uint32_t leaf_of(const MemSt& R, uint32_t code) {
    return (code >> 28) == K_FLOW ? R.L + (code & 0x0fffffffu) : (code & 0x0fffffffu);
}

// uniform (t, seq, code) minimum over the lanes (lowest (t, seq); seqs are unique
// among finite keys, so the winner is unique unless every key is infinite)
struct Key { int64_t t; uint32_t s, c; };
__device__ __forceinline__ Key wave_min_key(int64_t t, uint32_t s, uint32_t c) {
    Key k;
    k.t = wave_min_i64(t);
    const bool tie = (t == k.t);
    const uint64_t tied = __ballot(tie);
    uint32_t win;
    if ((tied & (tied - 1)) == 0) {
        win = (uint32_t)__builtin_ctzll(tied);
    } else {
        const uint32_t smin = wave_umin_fast(tie ? s : 0xffffffffu);
        win = (uint32_t)__builtin_ctzll(__ballot(tie && s == smin));
    }
    k.s = rdl(s, win);
    k.c = rdl(c, win);
    return k;
}

__device__ __forceinline__ Key lds_key(const uint4* p) {
    const uint4 v = *p;
    Key k;
    k.t = mk64(rfl(v.x), rfl(v.y));
    k.s = rfl(v.z);
    k.c = rfl(v.w);
    return k;
}
__device__ __forceinline__ void lds_put_key(const Sim& S, uint4* p, const Key& k) {
    if (S.lane == 0) *p = make_uint4(lo32(k.t), hi32(k.t), k.s, k.c);
}

// minimum of leaf block b (64 leaves, one per lane)
__device__ __forceinline__ Key block_min(const Sim& S, const MemSt& R, uint32_t b) {
    const uint32_t leaf = b * 64u + (uint32_t)S.lane;
    int64_t t = kInf;
    uint32_t s = 0xffffffffu, c = 0u;
    if (leaf < R.n_leaf) {
        const uint4 k = R.keys[leaf];
        t = mk64(k.x, k.y);
        s = k.z;
        c = leaf < R.L ? ((k.w << 28) | leaf) : ((K_FLOW << 28) | (leaf - R.L));
    }
    return wave_min_key(t, s, c);
}
// minimum of level-1 group g (64 block minima)
__device__ __forceinline__ Key group_min(const Sim& S, const MemSt& R, uint32_t g) {
    const uint32_t i = g * 64u + (uint32_t)S.lane;
    int64_t t = kInf;
    uint32_t s = 0xffffffffu, c = 0u;
    if (i < R.n1) {
        const uint4 k = R.lv1[i];
        t = mk64(k.x, k.y);
        s = k.z;
        c = k.w;
    }
    return wave_min_key(t, s, c);
}

// A source's next event changed to (t, seq): store the leaf key and repair the
// two tree levels above it.  A block is re-reduced only if the leaf was its
// minimum and did not become smaller; a new smaller key just replaces it.
__device__ __forceinline__ void tree_touch(const Sim& S, MemSt& R, uint32_t leaf, int64_t t, uint32_t seq,
                                           uint32_t code, uint32_t aux) {
    st_rep(S, &R.keys[leaf], make_uint4(lo32(t), hi32(t), seq, aux));
    const uint32_t b = leaf >> 6;
    const Key cur = lds_key(&R.lv1[b]);
    Key nb;
    if (key_less(t, seq, cur.t, cur.s)) {
        nb.t = t; nb.s = seq; nb.c = code;
    } else if (leaf_of(R, cur.c) == leaf) {
        nb = block_min(S, R, b);
    } else {
        return;
    }
    lds_put_key(S, &R.lv1[b], nb);
    const uint32_t g = b >> 6;
    const Key cg = lds_key(&R.lv2[g]);
    Key ng;
    if (key_less(nb.t, nb.s, cg.t, cg.s)) {
        ng = nb;
    } else if (leaf_of(R, cg.c) == leaf_of(R, cur.c)) {
        ng = group_min(S, R, g);
    } else {
        return;
    }
    lds_put_key(S, &R.lv2[g], ng);
}

// ---- links: words 0-7 of the 128-B record, read and written by every lane as
// two 16-B accesses (each lane's later reads follow its own stores) ----
__device__ __forceinline__ LinkV link_get(const MemSt& R, uint32_t l) {
    const uint4* p = (const uint4*)(R.lrec + l * kLRec);
    const uint4 a = p[0], b = p[1];
    LinkV k;
    const uint32_t p0 = rfl(a.x), p1 = rfl(a.y), p2 = rfl(a.z);
    k.head = p0 & 0xffffu; k.txp = p0 >> 16;
    k.tail = p1 & 0xffffu; k.n_wire = p1 >> 16;
    k.n_queue = p2 & 0xffffu; k.busy = p2 >> 16;
    k.qb = rfl(a.w);
    k.cp_t = rfl(b.x);
    k.cp_seq = rfl(b.y);
    k.wh_t = rfl(b.z);
    k.wh_seq = rfl(b.w);
    return k;
}

__device__ __forceinline__ void link_put(const Sim& S, MemSt& R, const Hot& H, uint32_t l, const LinkV& k) {
    uint4* p = (uint4*)(R.lrec + l * kLRec);
    p[0] = make_uint4(k.head | (k.txp << 16), k.tail | (k.n_wire << 16), k.n_queue | (k.busy << 16), k.qb);
    p[1] = make_uint4(k.cp_t, k.cp_seq, k.wh_t, k.wh_seq);
    // next event of the link (register-resident link_put's rule), as an absolute key
    const uint32_t n0 = lo32(H.now);
    uint32_t t = 0, s = 0xffffffffu, kind = 0;
    if (k.busy) { t = k.cp_t; s = k.cp_seq; kind = K_COMPLETE; }
    if (k.n_wire) {
        const uint32_t rw = k.wh_t - n0, rt = t - n0;
        if (kind == 0 || rw < rt || (rw == rt && k.wh_seq < s)) { t = k.wh_t; s = k.wh_seq; kind = K_ARRIVE; }
    }
    const int64_t at = kind ? H.now + (int64_t)(uint32_t)(t - n0) : kInf;
    tree_touch(S, R, l, at, s, (kind << 28) | l, kind);
}

// ---- flows ----
__device__ __forceinline__ uint32_t flow_draw(const Sim& S, const MemSt& R, uint32_t f) {
    return u_ld32(&R.keys[R.L + f].w);
}
__device__ __forceinline__ void flow_set(const Sim& S, MemSt& R, const Hot& H, uint32_t f, int64_t t, uint32_t seq,
                                         uint32_t draw) {
    tree_touch(S, R, R.L + f, t, seq, (K_FLOW << 28) | f, draw);
}

// ---- ping state of tunnel t (== link t: identity overlays only) ----
__device__ __forceinline__ PingV ping_get(const Sim& S, const MemSt& R, uint32_t t) {
    const uint4 w = *(const uint4*)(R.lrec + t * kLRec + LR_PMLO);
    PingV p;
    p.lo = rfl(w.x); p.mlo = rfl(w.y); p.mhi = rfl(w.z); p.win = rfl(w.w);
    return p;
}
__device__ __forceinline__ void ping_set_lo(const Sim& S, MemSt& R, uint32_t t, uint32_t lo, uint64_t od) {
    uint32_t* p = R.lrec + t * kLRec;
    p[LR_PMLO] = lo;
    p[LR_ODLO] = (uint32_t)od;
    p[LR_ODHI] = (uint32_t)(od >> 32);
}
__device__ __forceinline__ void ping_set_mask(const Sim& S, MemSt& R, uint32_t t, uint64_t mask) {
    uint32_t* p = R.lrec + t * kLRec;
    p[LR_PMMLO] = (uint32_t)mask;
    p[LR_PMMHI] = (uint32_t)(mask >> 32);
}
__device__ __forceinline__ void ping_set_win(const Sim& S, MemSt& R, uint32_t t, uint32_t win, uint64_t avg) {
    uint32_t* p = R.lrec + t * kLRec;
    p[LR_PMWIN] = win;
    p[LR_PAVLO] = (uint32_t)avg;
    p[LR_PAVHI] = (uint32_t)(avg >> 32);
}

// observation of node v: lane i (1 <= i <= deg) evaluates link ovrow[v] + i - 1
__device__ __forceinline__ uint32_t observe_links(const Sim& S, const MemSt& R, const Hot& H, uint32_t v,
                                                  double now_s) {
    const int r0 = t_ovrow(S, v), deg = t_ovrow(S, v + 1) - r0;
    const int lane = S.lane;
    if (lane < 1 || lane > deg) return 0u;
    const uint32_t* p = R.lrec + (uint32_t)(r0 + lane - 1) * kLRec;
    if (S.lv.ping_as_obs())
        return ping_value_lane(ld_d(p[LR_PAVLO], p[LR_PAVHI]), p[LR_PMLO], ld_d(p[LR_ODLO], p[LR_ODHI]),
                               H.ping_rounds, now_s);
    return p[LR_QB];
}

// next event: minimum over the super-block minima and the ping timer
__device__ __forceinline__ void select_event(const Sim& S, const MemSt& R, const Hot& H, int lane, int64_t& bt,
                                             uint32_t& bc) {
    int64_t t = kInf;
    uint32_t s = 0xffffffffu, c = 0u;
    if ((uint32_t)lane < R.n2) {
        const uint4 k = R.lv2[lane];
        t = mk64(k.x, k.y);
        s = k.z;
        c = k.w;
    }
    if (lane == 0 && key_less(H.ping_t, H.ping_seq, t, s)) { t = H.ping_t; s = H.ping_seq; c = K_PING << 28; }
    const Key k = wave_min_key(t, s, c);
    bt = k.t;
    bc = k.c;
}

// ---------------------------------------------------------------------------
// binding, init, staging
// ---------------------------------------------------------------------------
__device__ __forceinline__ void mem_bind(Sim& S, MemSt& R, const KParams& P, const LV& lv, unsigned char* lds, int r,
                                         int lane) {
    CLayout& LC = *(CLayout*)P.lay;
    unsigned char* img = P.state + (size_t)r * LC.state_bytes;
    sim_bind(S, lv, lds, P.topo, P.log + (size_t)r * LC.log_cap * LC.rec_bytes, LC.replica_base + (uint32_t)r, lane);
    S.mem = true;
    S.tun = false;
    S.ring = (uint32_t*)(img + LC.s_ring);
    S.win = (float*)(img + LC.s_win);
    S.pbd = (float*)(img + LC.s_pbd);
    S.lrec = (uint32_t*)(img + LC.g_lrec);
    S.table = P.table;
    const CAS unsigned char* tb = (const CAS unsigned char*)P.topo;
    S.m_rowptr = (const CAS int32_t*)(tb + LC.t_rowptr);
    S.m_ldst = (const CAS int32_t*)(tb + LC.t_ldst);
    S.m_lrev = (const CAS int32_t*)(tb + LC.t_lrev);
    S.m_acctx = (const CAS int64_t*)(tb + LC.t_acctx);
    S.m_fsrc = (const CAS int32_t*)(tb + LC.t_fsrc);
    S.m_fdst = (const CAS int32_t*)(tb + LC.t_fdst);
    S.m_fmean = (const CAS double*)(tb + LC.t_fmean);
    R.lrec = S.lrec;
    R.keys = (uint4*)(img + LC.g_keys);
    R.lv1 = (uint4*)(lds + LC.s_lv1);
    R.lv2 = (uint4*)(lds + LC.s_lv2);
    R.L = (uint32_t)LC.L;
    R.n_leaf = LC.n_leaf;
    R.n1 = LC.n1;
    R.n2 = LC.n2;
}

// episode start (sim.cc:610-630, data-packet-manager.cc:118-121): LDS header,
// counters and obs zeroed; link records cleared (ping: round 0 pending from its
// send time on); link keys infinite; flow keys at their start offsets; tree built.
__device__ __forceinline__ void init_replica(Sim& S, MemSt& R, Hot& H, uint32_t episode, bool keep_totals) {
    const LV& L = S.lv;
    const int lane = S.lane;
    uint32_t dec = H.dec, hl = H.hops_launch, el = H.ev_launch;
    const uint64_t ht = keep_totals ? (uint64_t)u_ld64((const int64_t*)&S.h->hops_total) : 0u;
    const uint64_t et = keep_totals ? (uint64_t)u_ld64((const int64_t*)&S.h->events_total) : 0u;
    __syncthreads();
    uint4* st4 = (uint4*)S.base;
    for (uint32_t i = (uint32_t)lane; i < L.lds_state_bytes() / 16u; i += kWave) st4[i] = make_uint4(0, 0, 0, 0);
    const uint64_t od = (uint64_t)__double_as_longlong(ping_send_s(L, 0));
    const uint32_t NL = R.L;
    for (uint32_t i = (uint32_t)lane; i < NL * 16u; i += kWave) {          // words 0..15 of every record
        const uint32_t l = i >> 4, w = i & 15u;
        const uint32_t v = w == LR_ODLO ? (uint32_t)od : (w == LR_ODHI ? (uint32_t)(od >> 32) : 0u);
        R.lrec[l * kLRec + w] = v;
    }
    for (uint32_t i = (uint32_t)lane; i < R.n_leaf; i += kWave) {
        uint4 k;
        if (i < NL) {
            k = make_uint4(lo32(kInf), hi32(kInf), 0xffffffffu, 0u);
        } else {
            const uint32_t f = i - NL;
            uint32_t c[4] = { f, 0u, episode, 0u };
            philox4x32_10(c, L.seed_lo(), S.gid);
            uint64_t u53 = ((uint64_t)(c[0] >> 5) << 26) | (uint64_t)(c[1] >> 6);
            double U = (double)u53 * (1.0 / 9007199254740992.0);
            const int64_t t = sec_to_ns(0.0001 + U);
            k = make_uint4(lo32(t), hi32(t), (uint32_t)L.NO() + f, 0u);  // after the NO ping timers
        }
        R.keys[i] = k;
    }
    // leaf 64b + lane was written by this lane above: block_min reads its own stores
    for (uint32_t b = 0; b < R.n1; ++b) lds_put_key(S, &R.lv1[b], block_min(S, R, b));
    __syncthreads();
    for (uint32_t g = 0; g < R.n2; ++g) lds_put_key(S, &R.lv2[g], group_min(S, R, g));
    H.now = 0;
    H.ping_t = L.ping_period();
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

__device__ __forceinline__ void mem_stage(unsigned char* lds, const KParams& P, int r, int lane, bool out) {
    CLayout& LC = *(CLayout*)P.lay;
    uint4* g4 = (uint4*)(P.state + (size_t)r * LC.state_bytes);
    uint4* l4 = (uint4*)lds;
    for (uint32_t i = (uint32_t)lane; i < LC.lds_state_bytes / 16u; i += kWave) {
        if (out) g4[i] = l4[i];
        else l4[i] = g4[i];
    }
}

// ---------------------------------------------------------------------------
// kernels (modes as in prisma_engine.hip)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) prisma_mem_reset_kernel(KParams P) {
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
    MemSt R;
    mem_bind(S, R, P, lv, lds, r, lane);
    init_replica(S, R, H, episode, keep);
    hot_store(S, R, H);
    __syncthreads();
    publish_counters(S, P, r, lane);
    mem_stage(lds, P, r, lane, true);
}

template <bool MLP>
__global__ void __launch_bounds__(64) prisma_mem_step_kernel(KParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int r = blockIdx.x, lane = threadIdx.x;
    mem_stage(lds, P, r, lane, false);
    __syncthreads();
    LV lv;
    lv.load(P.lay, lane);
    Sim S;
    MemSt R;
    mem_bind(S, R, P, lv, lds, r, lane);
    S.mlp = P.mlp;
    event_loop<MLP>(P, S, R, r);
    mem_stage(lds, P, r, lane, true);
}

// which: 0 step (table / external), 1 reset, 2 step with the DQN-buffer policy
const void* prisma_mem_kernel(int which) {
    if (which == 1) return (const void*)prisma_mem_reset_kernel;
    if (which == 2) return (const void*)prisma_mem_step_kernel<true>;
    return (const void*)prisma_mem_step_kernel<false>;
}

#if PRISMA_TRACE
// diagnostic build only: point the event trace at a device buffer [8][cap][3] (int64)
extern "C" int prisma_debug_trace(void* dev_buf, unsigned int cap) {
    unsigned int z[8] = {0};
    return (hipMemcpyToSymbol(HIP_SYMBOL(g_prisma_trace), &dev_buf, sizeof(void*)) == hipSuccess &&
            hipMemcpyToSymbol(HIP_SYMBOL(g_prisma_trace_cap), &cap, sizeof(cap)) == hipSuccess &&
            hipMemcpyToSymbol(HIP_SYMBOL(g_prisma_trace_n), z, sizeof(z)) == hipSuccess) ? 0 : -1;
}
#endif
