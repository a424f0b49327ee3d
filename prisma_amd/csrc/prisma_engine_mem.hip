// prisma_engine_mem.hip — the memory-resident gfx950 engine.
//
// For topologies beyond the register-resident engine (more than 255 nodes,
// 256 links or 512 flows: the Erdos-Renyi 256-node config, 2 264 links and
// 65 251 flows per replica) the replica state lives in HBM and one 64-lane
// wavefront still owns one replica and runs the same event handlers
// (engine_core.h), over a different store (MemSt):
//   * one 128-byte record per link (FIFO pointers, queued bytes, completion and
//     wire-head keys, ping state of the link's tunnel, the wire slots), read and
//     written as one coalesced wave access (lane j: word j);
//   * the next event of every source under a 64-ary tournament tree (round 5): link
//     leaves {time lo, seq} + kind in LDS, whose 64-leaf blocks report straight to the
//     top level; flow leaves {time lo, time hi, seq, draw} in HBM, under flow blocks (LDS)
//     and flow groups; the top level -- the link blocks in lanes [0, n_lb), the flow groups
//     in lanes [n_lb, n_top) -- sits in four VGPRs (its LDS image carries it from launch to
//     launch).  A source's update re-reduces its block (one LDS read or one coalesced 1 KiB
//     HBM read + a DPP reduction) only when the block minimum can change, and a flow block's
//     group likewise; choosing the next event is one reduction of the top lanes;
//   * FIFO rings, ping windows and ping-back delays in HBM (ring offsets as in
//     the register-resident engine).
// The header, counters and pending observation stay in LDS (staged per launch).
#include "engine_core.h"

// ---------------------------------------------------------------------------
// store
// ---------------------------------------------------------------------------
struct MemSt {
    static constexpr bool kLazy = true;          // empty-queue transmit completions elided (lazy_resolve)
    static constexpr bool kMem = true;
    static constexpr bool kDcache = false;       // (no draw cache: engine_core.h flow_next)
    uint32_t* lrec;              // [L][RW] link records (HBM)
    uint4* fkeys;                // [FG] flow leaf keys {t lo, t hi, seq, draw} (HBM)
    uint2* lkey;                 // LDS [L] link leaf keys {t lo, seq}: t = now + (t lo - lo32(now))
    uint8_t* lkind;              // LDS [L] link event kind (0: none, K_COMPLETE, K_ARRIVE)
    uint4* fblkmin;              // LDS [n_fb] flow block minima {t lo, t hi, seq, code}
    uint4* topimg;               // LDS [64] the top level's image between launches
    uint32_t L, FG, n_lb, n_fb, n_top, RW, WCAP;
    // the 64-leaf block of the flow whose send event runs, loaded (one coalesced 1 KiB
    // load) by flow_draw for its draw index; flow_set re-reduces the block from it instead
    // of storing the new key and loading the block back (one HBM round trip per flow event)
    uint4 fblk;
    uint32_t fblk_b;             // its block index, or ~0u
    // the top level, lane i = entry i {t lo, t hi, seq, code}: link block i (i < n_lb) or flow
    // group i - n_lb (i < n_top); infinite past n_top.  A link event -- most of a hop's events --
    // repairs its block and one top lane, with no LDS round trip at the top and no group level
    // (round 5, A/B on one box: config 5 DQN-buffer 89.1 -> 95.6 Mhops/s, SP table 111 -> 121)
    uint32_t g_tlo, g_thi, g_s, g_c;
};

constexpr int64_t kInf = INT64_MAX;

// uniform (t, seq, code) minimum over the lanes (lowest (t, seq); seqs are unique
// among finite keys, so the winner is unique unless every key is infinite)
struct Key { int64_t t; uint32_t s, c; };
__device__ __forceinline__ Key wave_min_key_exact(int64_t t, uint32_t s, uint32_t c) {
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
// The same minimum when every key is >= now (pending events, infinite keys): reduced as
// 32-bit offsets from the clock, saturated at 2^32-1, with one fused v_min_u32_dpp per step
// (the register-resident engine's select_event) instead of the 64-bit DPP compare/select
// chain; if every key saturates, the exact 64-bit reduction runs.
__device__ __forceinline__ Key wave_min_key(int64_t t, uint32_t s, uint32_t c, int64_t now) {
    const uint32_t o = sat_offset(t, now);
    const uint32_t omin = wave_umin_fast(o);
    if (omin == 0xffffffffu) return wave_min_key_exact(t, s, c);
    Key k;
    k.t = now + (int64_t)omin;
    const bool tie = (o == omin);
    const uint64_t tied = __ballot(tie);
    uint32_t win;
    if ((tied & (tied - 1)) == 0) {
        win = (uint32_t)__builtin_ctzll(tied);
    } else {                                                        // same-ns keys: seq order
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
    *p = make_uint4(lo32(k.t), hi32(k.t), k.s, k.c);     // every lane: same address, same value
}

// ---- the top level (VGPRs) ----
__device__ __forceinline__ Key top_key(const MemSt& R, uint32_t i) {
    Key k;
    k.t = mk64(rdl(R.g_tlo, i), rdl(R.g_thi, i));
    k.s = rdl(R.g_s, i);
    k.c = rdl(R.g_c, i);
    return k;
}
__device__ __forceinline__ void top_put(const Sim& S, MemSt& R, uint32_t i, const Key& k) {
    const bool me = (uint32_t)S.lane == i;
    R.g_tlo = me ? lo32(k.t) : R.g_tlo;
    R.g_thi = me ? hi32(k.t) : R.g_thi;
    R.g_s = me ? k.s : R.g_s;
    R.g_c = me ? k.c : R.g_c;
}
__device__ __forceinline__ void top_load(const Sim& S, MemSt& R) {
    const uint4 k = ((uint32_t)S.lane < R.n_top) ? R.topimg[S.lane] : make_uint4(0xffffffffu, 0x7fffffffu, 0xffffffffu, 0u);
    R.g_tlo = k.x; R.g_thi = k.y; R.g_s = k.z; R.g_c = k.w;
}
__device__ __forceinline__ void top_store(const Sim& S, const MemSt& R) {
    if ((uint32_t)S.lane < R.n_top) R.topimg[S.lane] = make_uint4(R.g_tlo, R.g_thi, R.g_s, R.g_c);
}

// ---- blocks and groups ----
// minimum of link block b (64 link leaves, LDS)
__device__ __forceinline__ Key lblock_min(const Sim& S, const MemSt& R, uint32_t b, int64_t now) {
    const uint32_t l = b * 64u + (uint32_t)S.lane;
    uint32_t s = 0xffffffffu, kind = 0u;
    // link keys are less than 2^31 ns ahead of the clock: the 32-bit offset is exact and needs no
    // 64-bit arithmetic or saturation (no event: 2^32 - 1; round 5, config 5 +1.3 %)
    uint32_t o = 0xffffffffu;
    if (l < R.L) {
        const uint2 k = R.lkey[l];                                  // key and kind read together
        kind = R.lkind[l];
        o = kind ? k.x - lo32(now) : 0xffffffffu;
        s = kind ? k.y : 0xffffffffu;
    }
    const uint32_t c = (kind << 28) | l;
    const uint32_t omin = wave_umin_fast(o);
    Key k;
    if (omin == 0xffffffffu) {                                      // no event in the block
        k.t = kInf; k.s = 0xffffffffu; k.c = rfl(c);
        return k;
    }
    k.t = now + (int64_t)omin;
    const uint64_t tied = __ballot(o == omin);
    uint32_t win;
    if ((tied & (tied - 1)) == 0) {
        win = (uint32_t)__builtin_ctzll(tied);
    } else {                                                        // same-ns keys: seq order
        const uint32_t smin = wave_umin_fast(o == omin ? s : 0xffffffffu);
        win = (uint32_t)__builtin_ctzll(__ballot(o == omin && s == smin));
    }
    k.s = rdl(s, win);
    k.c = rdl(c, win);
    return k;
}
// minimum of flow block fb (64 flow leaves, HBM)
__device__ __forceinline__ Key fblock_min(const Sim& S, const MemSt& R, uint32_t fb, int64_t now) {
    const uint32_t f = fb * 64u + (uint32_t)S.lane;
    int64_t t = kInf;
    uint32_t s = 0xffffffffu;
    if (f < R.FG) {
        const uint4 k = R.fkeys[f];
        t = mk64(k.x, k.y);
        s = k.z;
    }
    return wave_min_key(t, s, (K_FLOW << 28) | f, now);
}
// the cached block of the running flow event (flow_draw), with flow f holding its new key
__device__ __forceinline__ Key fblock_min_cached(const Sim& S, const MemSt& R, uint32_t fb, int64_t now, uint32_t f,
                                                 int64_t nt, uint32_t ns) {
    const uint32_t fi = fb * 64u + (uint32_t)S.lane;
    int64_t t = kInf;
    uint32_t s = 0xffffffffu;
    if (fi == f) {
        t = nt; s = ns;
    } else if (fi < R.FG) {
        t = mk64(R.fblk.x, R.fblk.y);
        s = R.fblk.z;
    }
    return wave_min_key(t, s, (K_FLOW << 28) | fi, now);
}
// minimum of flow group g (64 flow block minima, LDS)
__device__ __forceinline__ Key fgroup_min(const Sim& S, const MemSt& R, uint32_t g, int64_t now) {
    const uint32_t i = g * 64u + (uint32_t)S.lane;
    int64_t t = kInf;
    uint32_t s = 0xffffffffu, c = 0u;
    if (i < R.n_fb) {
        const uint4 k = R.fblkmin[i];
        t = mk64(k.x, k.y);
        s = k.z;
        c = k.w;
    }
    return wave_min_key(t, s, c, now);
}

// Link l's next event changed to (t, seq) of kind `kind` (0: none): store its leaf and repair
// its block's top lane.  The block is re-reduced only if the leaf was its minimum and did not
// become smaller; a new smaller key simply replaces it.
__device__ __forceinline__ void tree_touch_link(const Sim& S, MemSt& R, const Hot& H, uint32_t l, int64_t t,
                                                uint32_t seq, uint32_t code, uint32_t kind) {
    R.lkey[l] = make_uint2(lo32(t), seq);                           // every lane: same address, same value
    R.lkind[l] = (uint8_t)kind;
    const uint32_t b = l >> 6;
    const Key cur = top_key(R, b);
    Key nb;
    if (key_less(t, seq, cur.t, cur.s)) {
        nb.t = t; nb.s = seq; nb.c = code;
    } else if ((cur.c & 0x0fffffffu) == l) {
        nb = lblock_min(S, R, b, H.now);
    } else {
        return;
    }
    top_put(S, R, b, nb);
}
// Flow (slot) f's next event changed to (t, seq) with draw index `draw`: its leaf, its block
// minimum (LDS) and its group's top lane, each repaired only when it can change
__device__ __forceinline__ void tree_touch_flow(const Sim& S, MemSt& R, const Hot& H, uint32_t f, int64_t t,
                                                uint32_t seq, uint32_t draw) {
    st_rep(S, &R.fkeys[f], make_uint4(lo32(t), hi32(t), seq, draw));
    const uint32_t fb = f >> 6;
    const Key cur = lds_key(&R.fblkmin[fb]);
    Key nb;
    if (key_less(t, seq, cur.t, cur.s)) {
        nb.t = t; nb.s = seq; nb.c = (K_FLOW << 28) | f;
    } else if ((cur.c & 0x0fffffffu) == f) {
        nb = (fb == R.fblk_b) ? fblock_min_cached(S, R, fb, H.now, f, t, seq) : fblock_min(S, R, fb, H.now);
    } else {
        return;
    }
    lds_put_key(S, &R.fblkmin[fb], nb);
    const uint32_t g = fb >> 6, i = R.n_lb + g;
    const Key cg = top_key(R, i);
    Key ng;
    if (key_less(nb.t, nb.s, cg.t, cg.s)) {
        ng = nb;
    } else if (((cg.c & 0x0fffffffu) >> 6) == fb) {                // the group's minimum was this block's
        ng = fgroup_min(S, R, g, H.now);
    } else {
        return;
    }
    top_put(S, R, i, ng);
}

// ---- links: the whole record is one coalesced load (lane j: word j) and the fields
// come out with v_readlane; a write-back stores words 0-7 and the wire slots (lane j
// writes word j), so every word is only ever read and written by its own lane ----
__device__ __forceinline__ uint32_t rec_load(const MemSt& R, uint32_t l) {
    const uint32_t j = threadIdx.x;
    return j < R.RW ? R.lrec[l * R.RW + j] : 0u;
}

__device__ __forceinline__ LinkV link_fields(const MemSt& R, uint32_t rec) {
    LinkV k;
    k.rec = rec;
    const uint32_t p0 = rdl(k.rec, LR_P0), p1 = rdl(k.rec, LR_P1), p2 = rdl(k.rec, LR_P2);
    k.head = p0 & 0xffffu; k.txp = p0 >> 16;
    k.tail = p1 & 0xffffu; k.n_wire = p1 >> 16;
    k.n_queue = p2 & 0xffffu; k.busy = p2 >> 16;
    k.qb = rdl(k.rec, LR_QB);
    k.cp_t = rdl(k.rec, LR_CPT);
    k.cp_seq = rdl(k.rec, LR_CPS);
    k.wh_t = rdl(k.rec, LR_WHT);
    k.wh_seq = rdl(k.rec, LR_WHS);
    return k;
}
__device__ __forceinline__ LinkV link_get(const MemSt& R, uint32_t l) { return link_fields(R, rec_load(R, l)); }

template <unsigned MASK = LP_ALL>                 // (the whole record is written back either way)
__device__ __forceinline__ void link_put(const Sim& S, MemSt& R, const Hot& H, uint32_t l, const LinkV& k) {
    const uint32_t j = threadIdx.x;
    uint32_t w = k.rec;
    w = j == LR_P0 ? (k.head | (k.txp << 16)) : w;
    w = j == LR_P1 ? (k.tail | (k.n_wire << 16)) : w;
    w = j == LR_P2 ? (k.n_queue | (k.busy << 16)) : w;
    w = j == LR_QB ? k.qb : w;
    w = j == LR_CPT ? k.cp_t : w;
    w = j == LR_CPS ? k.cp_seq : w;
    w = j == LR_WHT ? k.wh_t : w;
    w = j == LR_WHS ? k.wh_seq : w;
    if (j < LR_PMLO || (j >= LR_WT && j < LR_WT + 3u * R.WCAP)) R.lrec[l * R.RW + j] = w;
    TP1(14);
    // next event of the link (register-resident link_put's rule)
    const uint32_t n0 = lo32(H.now);
    uint32_t t = 0, s = 0xffffffffu, kind = 0;
    if (k.busy && k.n_queue) { t = k.cp_t; s = k.cp_seq; kind = K_COMPLETE; }   // (lazy_resolve)
    if (k.n_wire) {
        const uint32_t rw = k.wh_t - n0, rt = t - n0;
        if (kind == 0 || rw < rt || (rw == rt && k.wh_seq < s)) { t = k.wh_t; s = k.wh_seq; kind = K_ARRIVE; }
    }
    const int64_t at = kind ? H.now + (int64_t)(uint32_t)(t - n0) : kInf;
    tree_touch_link(S, R, H, l, at, s, (kind << 28) | l, kind);
}

// ---- flows ----
__device__ __forceinline__ void flow_min_refresh(const Sim&, MemSt&, const Hot&) {}   // the event tree keeps it
__device__ __forceinline__ uint32_t flow_draw(const Sim& S, MemSt& R, uint32_t f) {
    const uint32_t fb = f >> 6, fi = fb * 64u + (uint32_t)S.lane;
    R.fblk = fi < R.FG ? R.fkeys[fi] : make_uint4(0u, 0u, 0u, 0u);
    R.fblk_b = fb;
    return rdl(R.fblk.w, f & 63u);
}
__device__ __forceinline__ void flow_set(const Sim& S, MemSt& R, const Hot& H, uint32_t f, int64_t t, uint32_t seq,
                                         uint32_t draw) {
    tree_touch_flow(S, R, H, f, t, seq, draw);
    R.fblk_b = ~0u;
}

// ---- ping state of tunnel t (== link t: identity overlays only), words 8-15 ----
__device__ __forceinline__ PingV ping_get(const Sim& S, const MemSt& R, uint32_t t) {
    const uint32_t w = rec_load(R, t);
    PingV p;
    p.lo = rdl(w, LR_PMLO); p.mlo = rdl(w, LR_PMMLO); p.mhi = rdl(w, LR_PMMHI); p.win = rdl(w, LR_PMWIN);
    return p;
}
__device__ __forceinline__ void rec_put2(const MemSt& R, uint32_t t, uint32_t w0, uint32_t a, uint32_t b) {
    const uint32_t j = threadIdx.x;
    if (j == w0 || j == w0 + 1u) R.lrec[t * R.RW + j] = j == w0 ? a : b;
}
__device__ __forceinline__ void ping_set_lo(const Sim& S, MemSt& R, uint32_t t, uint32_t lo, uint64_t od) {
    const uint32_t j = threadIdx.x;
    if (j == LR_PMLO || j == LR_ODLO || j == LR_ODHI)
        R.lrec[t * R.RW + j] = j == LR_PMLO ? lo : (j == LR_ODLO ? (uint32_t)od : (uint32_t)(od >> 32));
}
__device__ __forceinline__ void ping_set_mask(const Sim& S, MemSt& R, uint32_t t, uint64_t mask) {
    rec_put2(R, t, LR_PMMLO, (uint32_t)mask, (uint32_t)(mask >> 32));
}
__device__ __forceinline__ void ping_set_win(const Sim& S, MemSt& R, uint32_t t, uint32_t win, uint64_t avg) {
    const uint32_t j = threadIdx.x;
    if (j == LR_PMWIN || j == LR_PAVLO || j == LR_PAVHI)
        R.lrec[t * R.RW + j] = j == LR_PMWIN ? win : (j == LR_PAVLO ? (uint32_t)avg : (uint32_t)(avg >> 32));
}

// Elided completions (engine_core.h lazy_due): settle every one that precedes the current
// event -- or, at the end of an episode, every one before simTime -- with lane i scanning
// links i, 64 + i, ... (a few dozen dependent loads per launch).  This is the only place
// where a lane other than LR_P2 stores word LR_P2 of a record; the next access to it is
// by the same lane (a later scan of this launch) or in a later launch.
__device__ __forceinline__ void lazy_resolve(const Sim& S, MemSt& R, Hot& H, bool episode_end) {
    const uint32_t n0 = lo32(H.now);
    const int64_t t_end = S.lv.t_end();
    uint32_t n = 0;
    int64_t tmax = H.now;
    for (uint32_t b = 0; b < R.L; b += 64u) {
        const uint32_t l = b + (uint32_t)S.lane;
        bool due = false;
        if (l < R.L) {
            uint32_t* p = R.lrec + l * R.RW;
            const uint32_t p1 = p[LR_P1], p2 = p[LR_P2], cpt = p[LR_CPT], cps = p[LR_CPS];
            const int32_t dt = (int32_t)(cpt - n0);
            const int64_t t = H.now + (int64_t)dt;
            const bool lazy = (p2 >> 16) != 0u && (p2 & 0xffffu) == 0u;
            due = lazy && (episode_end ? ((p1 >> 16) == 0u || t < t_end) : lazy_due(p1 >> 16, cpt, cps, H));
            if (due) p[LR_P2] = p2 & 0xffffu;
            if (due && (p1 >> 16) != 0u && t > tmax) tmax = t;
        }
        n += (uint32_t)__builtin_popcountll(__ballot(due));
    }
    H.ev_launch += n;
    if (episode_end && n) {
        const int64_t m = -wave_min_i64(-tmax);
        if (m > H.now) H.now = m;
    }
}

// observation of node v: lane i (1 <= i <= deg) gathers the words of link ovrow[v] + i - 1
// (written by other lanes of this wave in earlier events)
// (the row pointer and degree arguments of the register-resident engine's version: not taken)
__device__ __forceinline__ uint32_t observe_links(const Sim& S, const MemSt& R, const Hot& H, uint32_t v,
                                                  double now_s, int = -1, int = 0) {
    const int r0 = t_ovrow(S, v), deg = t_ovrow(S, v + 1) - r0;
    const int lane = S.lane;
    if (lane < 1 || lane > deg) return 0u;
    const uint32_t* p = R.lrec + (uint32_t)(r0 + lane - 1) * R.RW;
    if (S.lv.ping_as_obs())
        return ping_value_lane(ld_d(p[LR_PAVLO], p[LR_PAVHI]), p[LR_PMLO], ld_d(p[LR_ODLO], p[LR_ODHI]),
                               H.ping_rounds, now_s);
    return p[LR_QB];
}

// next event: minimum over the top level (VGPRs; infinite past n_top) and the ping timer
__device__ __forceinline__ void select_event(const Sim& S, const MemSt& R, const Hot& H, int lane, int64_t& bt,
                                             uint32_t& bc, uint32_t& bs) {
    int64_t t = mk64(R.g_tlo, R.g_thi);
    uint32_t s = R.g_s, c = R.g_c;
    if (lane == 0 && key_less(H.ping_t, H.ping_seq, t, s)) { t = H.ping_t; s = H.ping_seq; c = K_PING << 28; }
    const Key k = wave_min_key(t, s, c, H.now);
    bt = k.t;
    bc = k.c;
    bs = k.s;
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
    S.table_g = P.table;
    S.tab_lds = false;
    const CAS unsigned char* tb = (const CAS unsigned char*)P.topo;
    S.m_rowptr = (const CAS int32_t*)(tb + LC.t_rowptr);
    S.m_ldst = (const CAS int32_t*)(tb + LC.t_ldst);
    S.m_lrev = (const CAS int32_t*)(tb + LC.t_lrev);
    S.m_acctx = (const CAS int64_t*)(tb + LC.t_acctx);
    S.m_fsrc = (const CAS int32_t*)(tb + LC.t_fsrc);
    S.m_fdst = (const CAS int32_t*)(tb + LC.t_fdst);
    S.m_fmean = (const CAS double*)(tb + LC.t_fmean);
    S.m_esz = (const CAS uint32_t*)(tb + LC.t_esz);
    S.m_etx = (const CAS uint32_t*)(tb + LC.t_etx);
    S.m_abtx = (const CAS uint32_t*)(tb + LC.t_abtx);
    S.m_bpair = (const CAS uint32_t*)(tb + LC.t_bpair);
    S.m_fseq = (const CAS uint32_t*)(tb + LC.t_fseq);
    S.m_bs = (const CAS BigSig*)(tb + LC.t_bsig);
    R.lrec = S.lrec;
    R.fkeys = (uint4*)(img + LC.g_keys);
    R.lkey = (uint2*)(lds + LC.s_lkey);
    R.lkind = (uint8_t*)(lds + LC.s_lkind);
    R.fblkmin = (uint4*)(lds + LC.s_lv1);
    R.topimg = (uint4*)(lds + LC.s_lv2);
    R.L = (uint32_t)LC.L;
    R.FG = LC.n_leaf - R.L;
    R.n_lb = (R.L + 63u) / 64u;                  // (layout_mem: n1 = n_fb flow blocks, n2 = n_top <= 64)
    R.n_fb = LC.n1;
    R.n_top = LC.n2;
    R.RW = LC.lrec_words;
    R.WCAP = (uint32_t)LC.WCAP;
    R.fblk = make_uint4(0u, 0u, 0u, 0u);
    R.fblk_b = ~0u;
    R.g_tlo = 0xffffffffu; R.g_thi = 0x7fffffffu; R.g_s = 0xffffffffu; R.g_c = 0u;
}

// episode start (sim.cc:610-630, data-packet-manager.cc:118-121): LDS header,
// counters and obs zeroed; link records cleared (ping: round 0 pending from its
// send time on); link keys infinite; flow keys at their start offsets; tree built.
__device__ __forceinline__ void init_replica(Sim& S, MemSt& R, Hot& H, uint32_t episode, bool keep_totals,
                                             const uint32_t* rng, uint32_t r) {
    const LV& L = S.lv;
    const int lane = S.lane;
    uint32_t dec = H.dec, hl = H.hops_launch, el = H.ev_launch;
    const uint64_t ht = keep_totals ? (uint64_t)u_ld64((const int64_t*)&S.h->hops_total) : 0u;
    const uint64_t et = keep_totals ? (uint64_t)u_ld64((const int64_t*)&S.h->events_total) : 0u;
    __syncthreads();
    uint4* st4 = (uint4*)S.base;
    for (uint32_t i = (uint32_t)lane; i < L.lds_state_bytes() / 16u; i += kWave) st4[i] = make_uint4(0, 0, 0, 0);
    const uint32_t* rep = rng ? rng + 18u * kMrgPowers + kMrgRepWords * r : nullptr;   // (engine_core.h)
    if (rng) {
        __syncthreads();
        ns3_init_lds(S, rng, rep);
    }
    const uint64_t od = (uint64_t)__double_as_longlong(ping_send_s(L, 0));
    const uint32_t NL = R.L;
    const uint32_t j = (uint32_t)lane;
    if (j < R.RW) {                                   // lane j writes word j of every record
        const uint32_t v = j == LR_ODLO ? (uint32_t)od : (j == LR_ODHI ? (uint32_t)(od >> 32) : 0u);
        for (uint32_t l = 0; l < NL; ++l) R.lrec[l * R.RW + j] = v;
    }
    // flow leaves (link leaves are in LDS, zeroed: no event); lane j writes the leaves
    // 64b + j that its block reductions read back.  Start seqs: the NO ping timers, then the
    // apps in install order (fseq: with big signalling each generator right after its flow);
    // leaf F is the generators' slot (on_bsig), started at AppStartTime (sim.cc:244, 645)
    const uint32_t nbs = S.m_bs->n_gen;
    for (uint32_t f = j; f < R.FG; f += kWave) {
        int64_t t = sec_to_ns(0.0001);
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
            t = sec_to_ns(0.0001 + U);                                // sim.cc:610-630
        }
        R.fkeys[f] = make_uint4(lo32(t), hi32(t), S.m_fseq[f], 0u);
    }
    __syncthreads();
    for (uint32_t b = 0; b < R.n_lb; ++b) top_put(S, R, b, lblock_min(S, R, b, 0));
    for (uint32_t fb = 0; fb < R.n_fb; ++fb) lds_put_key(S, &R.fblkmin[fb], fblock_min(S, R, fb, 0));
    __syncthreads();
    for (uint32_t g = 0; R.n_lb + g < R.n_top; ++g) top_put(S, R, R.n_lb + g, fgroup_min(S, R, g, 0));
    top_store(S, R);
    H.now = 0;
    H.ping_t = L.ping_period();
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
    init_replica(S, R, H, episode, keep, P.rng, (uint32_t)r);
    hot_store(S, R, H);
    __syncthreads();
    publish_counters(S, P, r, lane);
    mem_stage(lds, P, r, lane, true);
}

template <bool MLP, bool CTRL>
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
    S.mlp_rp = P.mlp_rp;
    S.ctrl = CTRL;
#ifndef PRISMA_MLP_B_MEM
#define PRISMA_MLP_B_MEM kMlpAll
#endif
    top_load(S, R);
    event_loop<MLP, PRISMA_MLP_B_MEM>(P, S, R, r, (uint32_t)P.max_hops);
    top_store(S, R);
    __syncthreads();
    mem_stage(lds, P, r, lane, true);
}

// which: 0 step (table / external), 1 reset, 2 step with the DQN-buffer policy; ctrl: the
// --train echo / notify_dest paths compiled in (step_kernel.h)
const void* prisma_mem_kernel(int which, bool ctrl) {
    if (which == 1) return (const void*)prisma_mem_reset_kernel;
    if (which == 2) return ctrl ? (const void*)prisma_mem_step_kernel<true, true>
                                : (const void*)prisma_mem_step_kernel<true, false>;
    return ctrl ? (const void*)prisma_mem_step_kernel<false, true> : (const void*)prisma_mem_step_kernel<false, false>;
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

#if PRISMA_TIMING
// diagnostic build only: read and clear the memory-resident engine's per-phase cycle totals
extern "C" int prisma_debug_timing_mem(unsigned long long* out16) {
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_prisma_timing), kTimingWords * sizeof(unsigned long long)) != hipSuccess) return -1;
    unsigned long long z[kTimingWords] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_prisma_timing), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
