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

#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "../../include/prisma.h"
#include "engine_layout.h"
#include "numerics.h"

#include "engine_core.h"
#include "step_kernel.h"

// memory-resident engine kernels (prisma_engine_mem.hip): 0 step, 1 reset, 2 step + DQN-buffer MLP
const void* prisma_mem_kernel(int which, bool ctrl);


// mode 0: (re)build every replica at episode P.episode.
// mode 3 (auto-reset, launched after each prisma_step / prisma_run when auto_reset is set):
// a replica whose episode ended (and did not fail) starts episode + 1, keeping its
// decision-log position and running totals.  A fused run normally does this inside the step
// kernel from the spare image (engine_core.h spare_restart); this catches the rest.
// With P.spare (auto_reset), both modes also (re)build each replica's spare -- the fresh
// image of the episode after its current one -- unless it is already there.
template <int FS, int LS>
__device__ __forceinline__ void image_store(const unsigned char* lds, CLayout& LC, unsigned char* img, int lane,
                                            Regs<FS, LS>& R) {
    uint4* s4 = (uint4*)img;
    const uint4* d4 = (const uint4*)lds;
    for (uint32_t i = (uint32_t)lane; i < LC.lds_state_bytes / 16u; i += kWave) s4[i] = d4[i];
    regs_io(R, (uint32_t*)(img + LC.s_regs), lane, true);
}

template <int FS, int LS>
__global__ void __launch_bounds__(64) prisma_reset_kernel_t(KParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int r = blockIdx.x, lane = threadIdx.x;
    CLayout& LC = *(CLayout*)P.lay;
    unsigned char* img = P.state + (size_t)r * LC.state_bytes;
    const Hdr* gh = (const Hdr*)(img + kOffHdr);
    LV lv;
    lv.load(P.lay, lane);
    Sim S;
    sim_bind(S, lv, lds, P.topo, P.log + (size_t)r * LC.log_cap * LC.rec_bytes, LC.replica_base + (uint32_t)r, lane);
    Hot H;
    memset(&H, 0, sizeof(H));
    const bool keep = (P.mode == 3);
    uint32_t episode = P.episode;                        // the state's episode after this kernel
    bool build = true;
    if (keep) {
        build = rfl(gh->over) && !rfl(gh->error);       // else: still running (or failed)
        episode = rfl(gh->episode) + (build ? 1u : 0u);
        if (build) {
            H.dec = rfl(gh->dec_count);
            if (lane < (int)(sizeof(Hdr) / 4)) ((uint32_t*)(lds + kOffHdr))[lane] = ((const uint32_t*)gh)[lane];
            __syncthreads();
        }
    }
    if (build) {
        Regs<FS, LS> R;
        init_replica(S, R, H, episode, keep, P.rng, (uint32_t)r);
        hot_store(S, R, H);
        __syncthreads();
        publish_counters(S, P, r, lane);
        image_store(lds, LC, img, lane, R);
    }
    if (P.spare) {
        unsigned char* sp = P.spare + (size_t)r * LC.state_bytes;
        if (!keep || rfl(((const Hdr*)(sp + kOffHdr))->episode) != episode + 1u) {
            __syncthreads();
            Hot H2;
            memset(&H2, 0, sizeof(H2));
            Regs<FS, LS> R2;
            init_replica(S, R2, H2, episode + 1u, false, P.rng, (uint32_t)r);   // log position and totals: patched at restart
            hot_store(S, R2, H2);
            __syncthreads();
            image_store(lds, LC, sp, lane, R2);
        }
    }
}

// step kernels (step_kernel.h): the table-policy instances with the --train / notify_dest
// code paths are compiled here, the in-kernel DQN-buffer ones in prisma_engine_mlp.hip, the
// ones without those paths in prisma_engine_lite.hip / prisma_engine_lite_mlp.hip
const void* prisma_pick_step_lite(int fs, int ls, bool tun);
const void* prisma_pick_step_lite_mlp(int fs, int ls, bool tun);
const void* prisma_pick_step_ctrl_mlp(int fs, int ls, bool tun);
static const void* pick_step_ctrl(int fs, int ls, bool tun) { return pick_step<true, false>(fs, ls, tun); }

template <int FS, int LS> const void* reset_kernel() { return (const void*)prisma_reset_kernel_t<FS, LS>; }
static const void* pick_reset(int fs, int ls) {
#define PK(F_, L_) if (fs == F_ && ls == L_) return reset_kernel<F_, L_>();
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

// Compaction of the pending replicas of a prisma_step (mask 1) into a dense batch for an
// external policy (the Forwarder steps only the nodes that were notified, ns3env.py:417-423):
// one workgroup of 16 waves walks the replicas in chunks of 1 024; each wave ballots its 64
// mask bytes, a lane's rank among the wave's pending lanes is the popcount of the ballot's
// lower bits (v_mbcnt), and the 16 wave totals are scanned in LDS. Ids come out ascending.
constexpr int kCompactThreads = 1024;
__global__ void __launch_bounds__(kCompactThreads) prisma_compact_kernel(
        const uint8_t* __restrict__ mask, const int32_t* __restrict__ obs, const int32_t* __restrict__ node, int32_t R,
        int32_t W, int32_t* __restrict__ ids, int32_t* __restrict__ obs_p, int32_t* __restrict__ node_p,
        int32_t* __restrict__ count) {
    __shared__ uint32_t wsum[kCompactThreads / kWave];
    const uint32_t tid = threadIdx.x, wave = tid / kWave;
    uint32_t base = 0;
    for (int32_t c = 0; c < R; c += kCompactThreads) {
        const int32_t i = c + (int32_t)tid;
        const bool act = i < R && mask[i] != 0;
        const uint64_t bal = __ballot(act);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if ((tid & (kWave - 1)) == 0) wsum[wave] = (uint32_t)__builtin_popcountll(bal);
        __syncthreads();
        uint32_t off = 0, total = 0;
        for (uint32_t w = 0; w < kCompactThreads / kWave; ++w) {
            const uint32_t s = wsum[w];
            off += w < wave ? s : 0u;
            total += s;
        }
        if (act) {
            const uint32_t p = base + off + rank;
            ids[p] = i;
            if (node_p) node_p[p] = node ? node[i] : -1;
            if (obs_p)
                for (int32_t k = 0; k < W; ++k) obs_p[(size_t)p * W + k] = obs[(size_t)i * W + k];
        }
        base += total;
        __syncthreads();                                   // wsum is rewritten by the next chunk
    }
    if (tid == 0) count[0] = (int32_t)base;
}

// The policy's actions for a compacted batch back to one action per replica: fill, then
// actions[ids[i]] = packed[i] for i < count (one workgroup, so the fill is ordered first).
__global__ void __launch_bounds__(kCompactThreads) prisma_expand_kernel(
        const int32_t* __restrict__ ids, const int32_t* __restrict__ count, const int32_t* __restrict__ packed,
        int32_t R, int32_t fill, int32_t* __restrict__ actions) {
    for (int32_t i = (int32_t)threadIdx.x; i < R; i += kCompactThreads) actions[i] = fill;
    __syncthreads();
    const int32_t n = count[0];
    for (int32_t i = (int32_t)threadIdx.x; i < n; i += kCompactThreads) {
        const int32_t r = ids[i];
        if ((uint32_t)r < (uint32_t)R) actions[r] = packed[i];
    }
}

// DQN-buffer weights, row-major [in][out] in the caller's packed buffer (StackedQNet.pack(),
// models.py:258-306), copied into the interleaved per-node blocks mlp_action reads
// (engine_core.h, mlp_rp_*): rp[v] = [Wb chunks, bb, b1][W2 chunks, b2][W3 chunks, b3][W4 chunks, b4].
__global__ void prisma_mlp_repack_kernel(const float* __restrict__ w, float* __restrict__ rp, int N, int D) {
    const int node_f = mlp_rp_node_floats(D);
    const int l1_f = mlp_rp_l1_floats(D), kc = (D + 3) / 4;
    const size_t n = (size_t)N * node_f;
    const float* b1 = w + (size_t)N * N * 32;
    const float* Wb = b1 + (size_t)N * 32;
    const float* bb = Wb + (size_t)N * D * 32;
    const float* W2 = bb + (size_t)N * 32;
    const float* b2 = W2 + (size_t)N * 64 * 64;
    const float* W3 = b2 + (size_t)N * 64;
    const float* b3 = W3 + (size_t)N * 64 * 64;
    const float* W4 = b3 + (size_t)N * 64;
    const float* b4 = W4 + (size_t)N * 64 * D;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int v = (int)(i / node_f);
        int o = (int)(i - (size_t)v * node_f);
        float x = 0.0f;                                   // padding (rows k >= D, alignment)
        if (o < l1_f) {
            if (o < 128 * kc) {
                const int c = o / 128, r = o - c * 128, j = r >> 2, q = r & 3, k = 4 * c + q;
                if (k < D) x = Wb[((size_t)v * D + k) * 32 + j];
            } else if (o < 128 * kc + 32) {
                x = bb[(size_t)v * 32 + (o - 128 * kc)];
            } else {
                x = b1[(size_t)v * 32 + (o - 128 * kc - 32)];
            }
        } else {
            o -= l1_f;
            const float *Wl, *bl;
            int units;
            if (o < mlp_rp_layer_floats(64)) {
                Wl = W2 + (size_t)v * 64 * 64; bl = b2 + (size_t)v * 64; units = 64;
            } else if (o < 2 * mlp_rp_layer_floats(64)) {
                o -= mlp_rp_layer_floats(64);
                Wl = W3 + (size_t)v * 64 * 64; bl = b3 + (size_t)v * 64; units = 64;
            } else {
                o -= 2 * mlp_rp_layer_floats(64);
                Wl = W4 + (size_t)v * 64 * D; bl = b4 + (size_t)v * D; units = D;
            }
            if (o < 64 * units) {
                const int c = o / (4 * units), r = o - c * 4 * units, j = r >> 2, q = r & 3;
                x = Wl[(4 * c + q) * units + j];
            } else if (o < mlp_rp_layer_floats(units)) {
                x = bl[o - 64 * units];
            }
        }
        rp[i] = x;
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
    float* d_mlp_rp = nullptr;           // interleaved DQN-buffer layers 2-4 (prisma_run, mode 4)
    unsigned char* d_spare = nullptr;    // next-episode images (register engine with auto_reset)
    uint32_t* d_rng = nullptr;           // ns-3 stream table (PRISMA_RNG_NS3, engine_layout.h kMrgPowers)
    prisma_kernel_info_t kinfo{};        // the step-kernel instances prisma_create picked
    bool reset_done = false;
};

static thread_local std::string g_err;
static int set_err(int code, const std::string& msg) { g_err = msg; return code; }

extern "C" int prisma_abi_version(void) { return PRISMA_ABI_VERSION; }

// Source hash the library was built from (prisma_amd/buildid.py, passed by the build as
// -DPRISMA_BUILD_ID); the marker lets the loader read it from the file without dlopen.
#ifndef PRISMA_BUILD_ID
#define PRISMA_BUILD_ID "unknown00000"
#endif
static const char k_build_id[] = "PRISMA_BUILD_ID=" PRISMA_BUILD_ID;
extern "C" const char* prisma_build_id(void) { return k_build_id + 16; }

PRISMA_TU_TIMING(prisma_debug_timing)
extern "C" const char* prisma_last_error(void) { return g_err.c_str(); }

static uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }
// largest draw-cache group (build_layout; 2 or 3, engine_core.h flow_next; 1: no cache)
#ifndef PRISMA_DCACHE_KMAX
#define PRISMA_DCACHE_KMAX 3u
#endif
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
    if (OP.T > (int)kMaxTunnels) return set_err(PRISMA_ERR_CONFIG, "more than 4096 tunnels (12-bit tunnel ids)");
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
        // (identity overlays never read it back -- tunnel t is link t -- and their link ids may
        // exceed the 8-bit field: ER-256)
        OP.tinfo[t] = ((uint32_t)l0 & 255u) | ((uint32_t)w << 8) | ((uint32_t)u << 16) | ((uint32_t)len << 24);
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

// Tunnelled overlays: a switch link that no packet can ever cross gets no state.  The
// links packets use are exactly those of the plan's control routes (every tunnel's
// forward path -- data and pings --, every ping-back route, every echo route); with
// their reverses (echoes and ping-backs leave on the reverse of the arrival link) they
// are renumbered 0..E'-1 in ascending original id, so the live links of a node stay
// contiguous and in neighbour order.  Abilene-on-GEANT: 74 -> 40 switch links, so with
// the 23 access links one register slot per lane holds them all (LS = 1: 4 waves per
// SIMD, 16 replicas per CU instead of 8).  Nothing outside the engine sees link ids.
// Access-link tx times depend on the PHYSICAL degree and are computed before this.
static void compact_links(const prisma_topology_t* T, OverlayPlan& OP, prisma_topology_t& TC,
                          std::vector<int32_t>& row, std::vector<int32_t>& dst, std::vector<int32_t>& rev) {
    const int N = T->n_nodes, E = T->n_links;
    std::vector<char> live(E, 0);
    for (const auto* ps : { &OP.cpaths, &OP.epaths })
        for (const auto& p : *ps)
            for (int l : p) { live[l] = 1; live[T->link_rev[l]] = 1; }
    std::vector<int32_t> m(E, -1);
    int E2 = 0;
    for (int l = 0; l < E; ++l)
        if (live[l]) m[l] = E2++;
    row.assign(N + 1, 0);
    dst.resize(E2);
    rev.resize(E2);
    for (int u = 0; u < N; ++u) {
        row[u + 1] = row[u];
        for (int l = T->row_ptr[u]; l < T->row_ptr[u + 1]; ++l)
            if (live[l]) { dst[m[l]] = T->link_dst[l]; rev[m[l]] = m[T->link_rev[l]]; row[u + 1]++; }
    }
    for (auto& ti : OP.tinfo) ti = (ti & ~255u) | (uint32_t)m[ti & 255u];
    for (auto& r : OP.route) {                   // a route over a dead link is never taken
        const uint32_t h = r & 255u;
        if (h != 255u) r = (r & ~255u) | (m[h] >= 0 ? (uint32_t)m[h] : 255u);
    }
    for (auto* ps : { &OP.cpaths, &OP.epaths })
        for (auto& p : *ps)
            for (int& l : p) l = m[l];
    TC = *T;
    TC.n_links = E2;
    TC.row_ptr = row.data();
    TC.link_dst = dst.data();
    TC.link_rev = rev.data();
}

// Signalling tables of the --train instances (build_layout), for either engine's topology image
struct Signal {
    std::vector<uint32_t> esz, etx;              // per switch link: echo size (B), its tx time (ns)
    std::vector<uint32_t> abtx;                  // per node: big segment's access-link tx time (ns)
    std::vector<uint32_t> bpair;                 // per generator (bp_*)
    std::vector<uint32_t> fseq;                  // [F + 1] start seqs of the flow slots
    BigSig bs;
};

// Memory-resident engine (prisma_engine_mem.hip, identity overlays): topology as
// variable-size arrays; state image = LDS part (header, counters, pending obs,
// event-tree levels 1-2, link leaf keys) + HBM part (link records, flow leaf keys,
// rings, ping windows, ping-back delays).  Scenario constants and ring sizing are set
// by build_layout.
static int layout_mem(const prisma_topology_t* T, const prisma_params_t* P, Layout& L,
                      std::vector<unsigned char>& topo, const std::vector<int64_t>& acctx,
                      const std::vector<int32_t>& ldst, uint32_t ring_total, const Signal& SG) {
    const int N = T->n_nodes, E = T->n_links, F = T->n_flows, Lk = E + N;
    if (L.WCAP > (int)kMemMaxWire) return set_err(PRISMA_ERR_CONFIG, "more than 16 packets on a wire (memory-resident engine)");
    L.lrec_words = LR_WT + 3u * (uint32_t)L.WCAP <= 32u ? 32u : 64u;
    // event sources: links, flows, and the big-signalling generators' one slot (on_bsig)
    const uint32_t FG = (uint32_t)F + (SG.bs.n_gen ? 1u : 0u);
    const uint64_t n_leaf = (uint64_t)Lk + (uint64_t)FG;
    if (n_leaf > 64ull * 64ull * 64ull) return set_err(PRISMA_ERR_CONFIG, "more than 262 144 links + flows per replica");
    L.mem = 1;
    L.n_leaf = (uint32_t)n_leaf;
    // event tree (prisma_engine_mem.hip): link blocks report to the top level, flow blocks (n1)
    // to flow groups there; the top level is one VGPR per lane: at most 64 entries
    L.n1 = (FG + 63u) / 64u;
    L.n2 = ((uint32_t)Lk + 63u) / 64u + (L.n1 + 63u) / 64u;
    if (L.n2 > 64u)
        return set_err(PRISMA_ERR_CONFIG, "memory-resident engine: more than 64 link blocks + flow groups "
                                          "(about 3 000 links at 65 000 flows)");
    uint64_t o = 0;
    auto take = [&](uint64_t bytes) { uint64_t r = o; o = (o + bytes + 15u) & ~(uint64_t)15u; return (uint32_t)r; };
    L.t_rowptr = take(4u * (N + 1));
    L.t_ldst = take(4u * (uint64_t)Lk);
    L.t_lrev = take(4u * (uint64_t)E);
    L.t_acctx = take(8u * (uint64_t)N);
    L.t_fsrc = take(4u * (uint64_t)F);
    L.t_fdst = take(4u * (uint64_t)F);
    L.t_fmean = take(8u * (uint64_t)F);
    L.t_esz = take(4u * (uint64_t)E);
    L.t_etx = take(4u * (uint64_t)E);
    L.t_abtx = take(4u * (uint64_t)N);
    L.t_bpair = take(4u * (uint64_t)(SG.bpair.size() ? SG.bpair.size() : 1u));
    L.t_fseq = take(4u * (uint64_t)(F + 1));
    L.t_bsig = take(sizeof(BigSig));
    L.topo_bytes = (uint32_t)o;
    topo.assign(o, 0);
    unsigned char* tb = topo.data();
    memcpy(tb + L.t_rowptr, T->row_ptr, 4u * (N + 1));
    memcpy(tb + L.t_ldst, ldst.data(), 4u * (size_t)Lk);
    memcpy(tb + L.t_lrev, T->link_rev, 4u * (size_t)E);
    memcpy(tb + L.t_acctx, acctx.data(), 8u * (size_t)N);
    memcpy(tb + L.t_fsrc, T->flow_src, 4u * (size_t)F);
    memcpy(tb + L.t_fdst, T->flow_dst, 4u * (size_t)F);
    double* fm = (double*)(tb + L.t_fmean);
    for (int f = 0; f < F; ++f)                      // poisson-application.cc:280-283
        fm[f] = (double)(P->packet_size * 8u) / (double)T->flow_rate_bps[f];
    memcpy(tb + L.t_esz, SG.esz.data(), 4u * (size_t)E);
    memcpy(tb + L.t_etx, SG.etx.data(), 4u * (size_t)E);
    memcpy(tb + L.t_abtx, SG.abtx.data(), 4u * (size_t)N);
    if (!SG.bpair.empty()) memcpy(tb + L.t_bpair, SG.bpair.data(), 4u * SG.bpair.size());
    memcpy(tb + L.t_fseq, SG.fseq.data(), 4u * (size_t)(F + 1));
    memcpy(tb + L.t_bsig, &SG.bs, sizeof(BigSig));
    o = 0;
    L.s_hdr = take(sizeof(Hdr));
    L.s_cnt = take(sizeof(prisma_counters_t));
    L.s_obs = take(4u * L.W);
    if (L.s_hdr != kOffHdr || L.s_cnt != kOffCnt || L.s_obs != kOffObs)
        return set_err(PRISMA_ERR_CONFIG, "internal: LDS header offsets");
    L.s_lv1 = take(16u * L.n1);                      // flow block minima
    L.s_lv2 = take(16u * L.n2);                      // the top level's image between launches
    L.s_lkey = take(8u * (uint64_t)Lk);
    L.s_lkind = take((uint64_t)Lk);
    if (L.rng_mode) take(kRngBytes);                // ns-3 streams: the last kRngBytes (engine_core.h)
    L.lds_state_bytes = (uint32_t)o;
    L.g_lrec = take(4u * L.lrec_words * (uint64_t)Lk);
    L.g_keys = take(16u * (uint64_t)FG);
    L.s_ring = take(4u * (uint64_t)ring_total);
    L.s_win = take(4u * (uint64_t)E * L.MA);
    L.s_pbd = take(4u * (uint64_t)E * L.PBK);
    if (o >= (1ull << 32)) return set_err(PRISMA_ERR_CONFIG, "replica state above 4 GiB");
    L.state_bytes = (uint32_t)o;
    L.s_regs = L.state_bytes;                       // no register part
    L.s_wt = L.s_wseq = 0;                          // wire slots live in the link records
    L.FS = L.LS = 0;
    L.ring_total = ring_total;
    L.lds_bytes = L.lds_state_bytes;                // the action table stays in HBM
    L.table_in_lds = 0;
    L.s_mlp = L.lds_bytes;
    L.lds_mlp_bytes = L.lds_bytes + 256u;
    if (L.lds_bytes + 256u > 160u * 1024u)
        return set_err(PRISMA_ERR_CONFIG, "event tree exceeds the 160 KiB LDS of a gfx950 CU");
    return PRISMA_OK;
}

static int build_layout(const prisma_topology_t* T, const prisma_params_t* P, Layout& L,
                        std::vector<unsigned char>& topo) {
    const int N = T->n_nodes, E0 = T->n_links, F = T->n_flows;
    if (N < 2 || N > 256) return set_err(PRISMA_ERR_CONFIG, "n_nodes must be in [2, 256] (8-bit node ids)");
    if (P->engine > PRISMA_ENGINE_MEMORY) return set_err(PRISMA_ERR_CONFIG, "engine must be PRISMA_ENGINE_AUTO, _REGISTER or _MEMORY");
    if (E0 < 1 || F < 1) return set_err(PRISMA_ERR_CONFIG, "need at least one link and one flow");
    if (!T->row_ptr || !T->link_dst || !T->link_rev || !T->flow_src || !T->flow_dst || !T->flow_rate_bps)
        return set_err(PRISMA_ERR_ARG, "null topology array");
    if (T->row_ptr[0] != 0 || T->row_ptr[N] != E0) return set_err(PRISMA_ERR_CONFIG, "row_ptr must span [0, n_links]");
    int maxdeg = 0;
    for (int u = 0; u < N; ++u) {
        int d = T->row_ptr[u + 1] - T->row_ptr[u];
        if (d < 1) return set_err(PRISMA_ERR_CONFIG, "every node needs at least one link");
        if (d > maxdeg) maxdeg = d;
        for (int l = T->row_ptr[u]; l < T->row_ptr[u + 1]; ++l) {
            int v = T->link_dst[l], rv = T->link_rev[l];
            if (v < 0 || v >= N || v == u) return set_err(PRISMA_ERR_CONFIG, "bad link_dst");
            if (l > T->row_ptr[u] && T->link_dst[l - 1] >= v) return set_err(PRISMA_ERR_CONFIG, "neighbours must be ascending");
            if (rv < 0 || rv >= E0 || T->link_dst[rv] != u || rv < T->row_ptr[v] || rv >= T->row_ptr[v + 1])
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
    // physical degrees (access-link rates, sim.cc:403-404), then a tunnelled overlay's
    // dead links dropped (compact_links); from here on T and E are the live links
    std::vector<int> pdeg(N);
    for (int u = 0; u < N; ++u) pdeg[u] = T->row_ptr[u + 1] - T->row_ptr[u];
    prisma_topology_t TC;
    std::vector<int32_t> c_row, c_dst, c_rev;
    if (OP.tunnels) {
        compact_links(T, OP, TC, c_row, c_dst, c_rev);
        T = &TC;
    }
    const int E = T->n_links;
    const int maxdeg_o = OP.maxdeg;
    if (P->link_bps == 0 || P->link_delay_ns < 0 || P->max_buffer_bytes == 0 || P->packet_size == 0 ||
        P->ma_size == 0 || P->ma_size > 64 || !(P->ping_interval_s > 0.0f))
        return set_err(PRISMA_ERR_CONFIG, "bad link / ping parameters");
    if (!(P->sim_time_s > 0.0) || P->sim_time_s > 4095.0)
        return set_err(PRISMA_ERR_CONFIG, "sim_time_s must be in (0, 4095] (12-bit packet start second)");
    if (P->log_capacity < 1024 || P->log_capacity > (1u << 22) || (P->log_capacity & (P->log_capacity - 1)))
        return set_err(PRISMA_ERR_CONFIG, "log_capacity must be a power of two >= 1024");
    if (P->rng_mode > PRISMA_RNG_NS3) return set_err(PRISMA_ERR_CONFIG, "rng_mode must be PRISMA_RNG_PHILOX or _NS3");
    if (P->rng_mode == PRISMA_RNG_NS3 && (uint64_t)F >= (1ull << kMrgPowers))
        return set_err(PRISMA_ERR_CONFIG, "ns-3 streams: more than 2^18 flows");
    if (P->signaling_type > PRISMA_SIGNALING_TARGET)
        return set_err(PRISMA_ERR_CONFIG, "signaling_type must be PRISMA_SIGNALING_IDEAL, _NN or _TARGET");
    // signalling (sim.cc:373-392): the echo payload of overlay node u by its overlay degree;
    // a tunnelled overlay's echoes cross several links, which the engine sizes per link, so
    // there the payload must be the same for every node
    std::vector<uint32_t> epay(N, 0u);
    for (int u = 0; u < N; ++u) {
        const uint32_t od = (uint32_t)(OP.ovrow[u + 1] - OP.ovrow[u]);
        epay[u] = P->signaling_type == PRISMA_SIGNALING_NN ? 8u + 8u * (od + 1u)
                                                           : (P->signaling_type == PRISMA_SIGNALING_TARGET ? 24u : 0u);
    }
    if (OP.tunnels)
        for (int i = 1; i < OP.NO; ++i)
            if (epay[OP.ovnode[i]] != epay[OP.ovnode[0]])
                return set_err(PRISMA_ERR_CONFIG, "signaling_type NN on a tunnelled overlay needs equal overlay "
                                                  "degrees (echo sizes per node are modelled on identity overlays)");
    // big signalling (sim.cc:634-647): one generator per flow between overlay neighbours, with
    // --train and "NN"; each starts right after its flow (install order: fseq below)
    const bool bsig = P->train && P->big_signaling && P->signaling_type == PRISMA_SIGNALING_NN;
    std::vector<int32_t> gen_of(F, -1);
    std::vector<uint32_t> bpair;
    if (bsig) {
        if (!(P->sync_step_s > 0.0f) || P->big_signaling_bytes == 0)
            return set_err(PRISMA_ERR_CONFIG, "big signalling needs sync_step_s > 0 and big_signaling_bytes > 0");
        for (int f = 0; f < F; ++f) {
            const int u = T->flow_src[f], w = T->flow_dst[f];
            for (int t = OP.ovrow[u]; t < OP.ovrow[u + 1]; ++t) {
                // (tinfo packs 8-bit link ids: on identity overlays tunnel t is switch link t,
                // beyond 255 on the memory-resident engine's ER-256, so read the topology)
                const int tgt = OP.tunnels ? (int)ti_tgt(OP.tinfo[t]) : T->link_dst[t];
                if (tgt == w) {
                    const uint32_t first = OP.tunnels ? ti_link(OP.tinfo[t]) : (uint32_t)t;
                    gen_of[f] = (int32_t)bpair.size();
                    bpair.push_back((uint32_t)u | ((uint32_t)w << 8) | (first << 16));
                    break;
                }
            }
        }
        if (bpair.size() > (1u << kGenBits)) return set_err(PRISMA_ERR_CONFIG, "more than 4096 big-signalling generators");
    }
    const int G = (int)bpair.size();
    // ScheduleNextTx's period in the reference's arithmetic (big-signaling-application.cc:247-250):
    // the uint32 size * 8 over the float syncStep is a float, 4096 over that a double
    const float bs_rate = bsig ? (float)(P->big_signaling_bytes * 8u) / P->sync_step_s : 1.0f;
    const int64_t bs_period = bsig ? sec_to_ns((double)(512u * 8u) / (double)bs_rate) : 0;
    // (the generators share one event slot: a period must outlast an access-link transmission)
    if (bsig && (bs_period < 1000 || bs_period >= ((int64_t)1 << 40)))
        return set_err(PRISMA_ERR_CONFIG, "big-signalling period out of range [1 us, 2^40 ns)");
    // (a segment carries its generator's send index in 17 bits: engine_layout.h g_make)
    if (bsig && sec_to_ns(P->sim_time_s) / bs_period + 2 > (int64_t)kGenSendMask)
        return set_err(PRISMA_ERR_CONFIG, "more than 2^17 big-signalling sends per generator and episode");
    const uint32_t bs_size = 512u + 30u;

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
    L.rng_mode = P->rng_mode;
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
        uint64_t bps = (uint64_t)1000000 * P->link_bps * (uint64_t)pdeg[u];
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
    // (a byte-limited FIFO holds the most packets when they are the smallest non-control ones)
    const uint32_t data_max = P->max_buffer_bytes / (G && bs_size < L.data_size ? bs_size : L.data_size);
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
        // (multiples of kQWin too: the LDS FIFO windows, engine_core.h q_put)
        const uint32_t m = (uint32_t)L.WCAP > kQWin ? (uint32_t)L.WCAP : kQWin;
        for (int l = 0; l < E; ++l) {
            uint32_t qs = data_max + (uint32_t)c[l] + (uint32_t)L.WCAP;
            rcap[l] = (qs + m - 1) / m * m;
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
    if (G) {                                         // all of a node's generators send at the same instants
        std::vector<uint32_t> per(N, 0u);
        uint32_t mx = 0;
        for (uint32_t b : bpair) { const uint32_t c = ++per[b & 255u]; mx = c > mx ? c : mx; }
        const uint32_t want = next_pow2(mx + 8u);
        L.qcap_a = want > L.qcap_a ? want : L.qcap_a;
    }
    tot += (uint32_t)N * L.qcap_a;
    L.ring_total = tot;
    // ping-back delay slots per responder: round k's slot is reused by round
    // k + PBK, whose forward ping arrives after round k's ping-back (at most
    // span after k's send) has been consumed
    L.PBK = next_pow2((uint32_t)(span / ival) + 2u);
    if (L.PBK > (1u << (kRoundBits - 1)))
        return set_err(PRISMA_ERR_CONFIG, "pings in flight span more than 2^13 rounds (14-bit round field)");
    // wire arrival times are kept as their low 32 bits relative to the clock
    int64_t max_acc = 0;
    for (int u = 0; u < N; ++u) max_acc = acctx[u] > max_acc ? acctx[u] : max_acc;
    if ((L.sw_txd > max_acc ? L.sw_txd : max_acc) + L.sw_prop >= ((int64_t)1 << 31))
        return set_err(PRISMA_ERR_CONFIG, "transmission + propagation delay above 2^31 ns");

    // scenario constants
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
    // register-resident engine: every limit of its fixed-size topology image,
    // lane-distributed registers and LDS image
    int fs = 1, ls = 1;
    const int FG = F + (G ? 1 : 0);                  // flow slots: the generators share one (on_bsig)
    while (64 * fs < FG) fs *= 2;
    while (64 * ls < (Lk > OP.T ? Lk : OP.T)) ls *= 2;
    const uint32_t reg_lds = 4u * (uint32_t)Lk * L.WCAP * (OP.tunnels ? 3u : 2u) + (OP.tunnels ? 0u : 4u * tot) +
                             4u * (uint32_t)OP.T * L.MA +
                             4u * (uint32_t)(OP.tunnels ? OP.n_resp : OP.T) * L.PBK + 1024u + 16u * (1u + L.W) +
                             (uint32_t)(N * N);
    const bool reg_fits = N <= 255 && Lk <= 256 && E <= 256 && FG <= 512 && OP.T <= 256 && G <= 256 && fs <= 8 && ls <= 4 &&
                          tot <= 65535u && reg_lds + 256u <= 160u * 1024u;
    uint32_t engine = P->engine == PRISMA_ENGINE_AUTO ? (reg_fits ? PRISMA_ENGINE_REGISTER : PRISMA_ENGINE_MEMORY)
                                                      : P->engine;
    if (engine == PRISMA_ENGINE_REGISTER && !reg_fits)
        return set_err(PRISMA_ERR_CONFIG, "topology exceeds the register-resident engine (255 nodes, 256 links / "
                                          "tunnels / generators, 512 flows, 160 KiB LDS); use PRISMA_ENGINE_MEMORY");
    if (engine == PRISMA_ENGINE_MEMORY && OP.tunnels)
        return set_err(PRISMA_ERR_CONFIG, "the memory-resident engine runs identity overlays only");
    // signalling arrays (both engines): echo size / tx time per switch link (echoes leave node u
    // on its own links), big-segment tx time per access link, start seqs of the flow slots (the
    // ping timers, then the apps in install order: each generator right after its flow; slot F
    // holds generator 0's)
    Signal SG;
    SG.esz.resize(E);
    SG.etx.resize(E);
    for (int u = 0; u < N; ++u)
        for (int l = T->row_ptr[u]; l < T->row_ptr[u + 1]; ++l) {
            SG.esz[l] = (OP.tunnels ? epay[OP.ovnode[0]] : epay[u]) + 30u;
            SG.etx[l] = (uint32_t)sec_to_ns((double)SG.esz[l] * 8 / (double)P->link_bps);
        }
    SG.abtx.resize(N);
    for (int u = 0; u < N; ++u)
        SG.abtx[u] = (uint32_t)sec_to_ns((double)bs_size * 8 / (double)((uint64_t)1000000 * P->link_bps * (uint64_t)pdeg[u]));
    SG.bpair = bpair;
    SG.fseq.assign(F + 1, 0u);
    {
        uint32_t q = (uint32_t)OP.NO;
        for (int f = 0; f < F; ++f) {
            SG.fseq[f] = q++;
            if (gen_of[f] == 0) SG.fseq[F] = q;      // generator 0 opens the group's slot
            if (gen_of[f] >= 0) q++;
        }
        if (!G) SG.fseq[F] = q;
    }
    SG.bs.period = bs_period;
    SG.bs.n_gen = (uint32_t)G;
    SG.bs.nseg = bsig ? P->big_signaling_bytes / 512u : 0u;
    SG.bs.size = bs_size;
    SG.bs.tx_sw = (uint32_t)sec_to_ns((double)bs_size * 8 / (double)P->link_bps);
    uint32_t o = 0;
    auto take = [&](uint32_t bytes) { uint32_t r = o; o = align16(o + bytes); return r; };
    L.table_bytes = (uint32_t)(N * N);
    if (engine == PRISMA_ENGINE_MEMORY)
        return layout_mem(T, P, L, topo, acctx, ldst, tot, SG);
    // topology image
    L.topo_bytes = (uint32_t)sizeof(TopoImage) + (OP.tunnels ? 4u * (uint32_t)(N * N) : 0u);
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
    {                                                // ring of every link (engine_core.h ring_off)
        uint32_t off = 0;
        for (int l = 0; l < Lk; ++l) {
            const uint32_t cap = l < E ? rcap[l] : L.qcap_a;
            TI.rinfo[l] = off | (cap << 16);
            off += cap;
        }
    }
    if (OP.tunnels) memcpy(TI.tresp, OP.tresp.data(), 4u * OP.T);
    for (uint32_t c = 0; c < 8; ++c) {               // entry classes: relay, fresh, ping fwd, ping back, +echo bit
        const bool data = (c & 2u) == 0u, echo = c == 7u, big = c == 6u;
        TI.ctx[c] = (uint32_t)(data ? L.sw_txd : (echo ? L.sw_txe : (big ? sec_to_ns((double)bs_size * 8 / (double)P->link_bps)
                                                                         : L.sw_txp)));
    }
    memcpy(TI.esz, SG.esz.data(), 4u * E);
    memcpy(TI.etx, SG.etx.data(), 4u * E);
    memcpy(TI.abtx, SG.abtx.data(), 4u * N);
    for (int l = 0; l < Lk; ++l)                     // (tx, tx + prop) by link and entry class
        for (uint32_t c = 0; c < 8; ++c) {
            const bool sw = l < E;
            const int64_t tx = sw ? (c == 7u ? (int64_t)SG.etx[l] : (int64_t)TI.ctx[c])
                                  : (c == 6u ? (int64_t)SG.abtx[l - E] : acctx[l - E]);
            const int64_t prop = sw ? L.sw_prop : 0;
            TI.ltx[2 * (l * 8 + (int)c)] = (uint32_t)tx;
            TI.ltx[2 * (l * 8 + (int)c) + 1] = (uint32_t)(tx + prop);
        }
    for (int g = 0; g < G; ++g) TI.bpair[g] = bpair[g];
    for (int f = 0; f < F; ++f) TI.fseq[f] = SG.fseq[f];
    if (G) TI.fseq[F] = SG.fseq[F];
    TI.bs_period = SG.bs.period;
    TI.n_bsig = SG.bs.n_gen;
    TI.bs_nseg = SG.bs.nseg;
    TI.bs_size = SG.bs.size;
    if (OP.tunnels) memcpy(topo.data() + sizeof(TopoImage), OP.route.data(), 4u * (size_t)N * N);

    // state image: LDS part (staged into LDS) then register part (staged into VGPRs)
    L.FS = fs; L.LS = ls;
    o = 0;
    L.s_hdr = take(sizeof(Hdr));
    L.s_cnt = take(sizeof(prisma_counters_t));
    L.s_obs = take(4u * L.W);
    if (L.s_hdr != kOffHdr || L.s_cnt != kOffCnt || L.s_obs != kOffObs)
        return set_err(PRISMA_ERR_CONFIG, "internal: LDS header offsets");
    // Tunnelled overlays keep their FIFOs in HBM (Abilene-on-GEANT: 9.6 KB of rings, sized
    // for the control packets of every route through a link, would hold LDS at 14.8 KB per
    // replica, 10 per CU: two rounds for 4 096 replicas) and the packet entry of each wire
    // slot in LDS after the seqs (Sim::went), so an arrival does not read the ring.
    L.s_wt = take(4u * Lk * L.WCAP);
    // (tunnelled: the wire slots' packet entries, then kQWin FIFO window slots per link, q_put)
    L.s_wseq = take(4u * Lk * (L.WCAP * (OP.tunnels ? 2u : 1u) + (OP.tunnels ? kQWin : 0u)));
    if (!OP.tunnels) L.s_ring = take(4u * tot);
    L.s_win = take(4u * (uint32_t)OP.T * L.MA);
    L.s_pbd = take(4u * (uint32_t)(OP.tunnels ? OP.n_resp : OP.T) * L.PBK);
    if (L.rng_mode) take(kRngBytes);                // ns-3 streams: the last kRngBytes (engine_core.h)
    // Replicas per CU are bounded by LDS (160 KiB / bytes per replica) for the larger
    // topologies, and a launch whose replicas do not all fit at once runs in rounds
    // (GEANT + MLP: 2 048 replicas at 7 per CU took two rounds, the second 1/8 full).
    const uint32_t tb = align16(L.table_bytes);
    // (waves per CU of the step kernel: StepOcc, 4 SIMDs x its waves per SIMD)
    const uint32_t occ = 4u * ((fs <= 2 && ls == 1) ? 4u : (ls <= 2 ? 2u : 1u));
    auto per_cu = [occ](uint32_t b) { const uint32_t n = (160u * 1024u) / (b ? b : 1u); return n < occ ? n : occ; };
    // The flows' draw cache (engine_core.h flow_next: K - 1 next-send delays of 8 B per flow,
    // computed in lanes 1 .. K-1 with the draw before them; K = 3, else 2) where it costs no
    // replica per CU, the action table's LDS placement counted as it would be without it; not
    // with ns-3 streams. Layout::s_dcache = its 16-B aligned offset | K.
    L.s_dcache = 0u;
    if (!L.rng_mode && F > 0 && fs <= 2) {         // (the instances with its code: Regs::kDcache)
        const uint32_t t0 = per_cu(o + tb) == per_cu(o) ? tb : 0u;
        for (uint32_t K = PRISMA_DCACHE_KMAX; K >= 2u; --K) {
            const uint32_t dc = align16(8u * (K - 1u) * (uint32_t)F);
            if (per_cu(o + dc + t0) == per_cu(o + t0)) { L.s_dcache = take(dc) | K; break; }
        }
    }
    L.lds_state_bytes = o;
    if (OP.tunnels) L.s_ring = take(4u * tot);      // HBM part of the image
    L.s_regs = take(4u * (4u * 64u * (uint32_t)fs + 16u * 64u * (uint32_t)ls));
    L.state_bytes = o;
    // The action table goes to LDS only where it costs no replica per CU (else the decision
    // reads it from HBM, L2-resident), and the DQN-buffer activations reuse the table's LDS,
    // dead in MLP launches, when it is there.
    L.table_in_lds = per_cu(L.lds_state_bytes + tb) == per_cu(L.lds_state_bytes) ? 1u : 0u;
    L.lds_bytes = L.lds_state_bytes + (L.table_in_lds ? tb : 0u);
    L.s_mlp = (L.table_in_lds && tb >= 256u) ? L.lds_state_bytes : L.lds_bytes;
    L.lds_mlp_bytes = L.s_mlp + 256u > L.lds_bytes ? L.s_mlp + 256u : L.lds_bytes;
    if (L.lds_mlp_bytes > 160u * 1024u)
        return set_err(PRISMA_ERR_CONFIG, "replica state exceeds the 160 KiB LDS of a gfx950 CU");

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
    if (L.rng_mode == PRISMA_RNG_NS3) {
        // ns-3 streams (mrg32k3a.h): J^(2^b), then per replica the states of stream
        // rng_stream_offset (its first flow's start) and of the run's first stream -- from the
        // package seed simSeed in all six words, advanced by simSeed substreams (SetRun)
        const uint64_t seed0 = params->seed + params->replica_base;
        if (seed0 < 1 || seed0 + (uint64_t)n_replicas > kMrgM2) {
            prisma_destroy(e);
            return set_err(PRISMA_ERR_CONFIG, "ns-3 streams: seed + replica id must lie in [1, 4294944443)");
        }
        std::vector<uint32_t> tab(18u * kMrgPowers + (size_t)kMrgRepWords * n_replicas);
        const MrgMat J = mrg_pow2(127);
        MrgMat Jb = J;
        for (uint32_t b = 0; b < kMrgPowers; ++b) {
            memcpy(&tab[18u * b], Jb.a, sizeof(Jb.a));
            Jb = mrg_mul(Jb, Jb);
        }
        const MrgMat JX = mrg_pow(J, params->rng_stream_offset);
        const MrgMat JXF = mrg_pow(J, (uint64_t)params->rng_stream_offset + (uint64_t)topo->n_flows);
        MrgMat sub[32];                                  // A^(2^(76+i)): AdvanceNthBy(run, 76)
        sub[0] = mrg_pow2(76);
        for (int i = 1; i < 32; ++i) sub[i] = mrg_mul(sub[i - 1], sub[i - 1]);
        for (int32_t r = 0; r < n_replicas; ++r) {
            const uint32_t sd = (uint32_t)(seed0 + (uint64_t)r);
            uint32_t s0[6] = { sd, sd, sd, sd, sd, sd };
            for (int i = 0; i < 32; ++i)
                if ((sd >> i) & 1u) mrg_apply(sub[i].a, s0);
            uint32_t* rep = &tab[18u * kMrgPowers + (size_t)kMrgRepWords * r];
            memcpy(rep, s0, sizeof(s0));
            mrg_apply(JX.a, rep);
            memcpy(rep + 6, s0, sizeof(s0));
            mrg_apply(JXF.a, rep + 6);
        }
        if (!HIP_OK(hipMalloc((void**)&e->d_rng, 4u * tab.size())) ||
            !HIP_OK(hipMemcpy(e->d_rng, tab.data(), 4u * tab.size(), hipMemcpyHostToDevice))) {
            prisma_destroy(e);
            return set_err(PRISMA_ERR_NOMEM, "ns-3 stream table");
        }
    }
    // fused runs with auto_reset continue into the next episode from a prebuilt image
    // (engine_core.h spare_restart): one more state image per replica
    if (L.auto_reset && !L.mem && !HIP_OK(hipMalloc(&e->d_spare, sb))) {
        prisma_destroy(e);
        return set_err(PRISMA_ERR_NOMEM, "hipMalloc of the spare images failed");
    }
    if (!HIP_OK(hipMemcpy(e->d_topo, img.data(), L.topo_bytes, hipMemcpyHostToDevice)) ||
        !HIP_OK(hipMemcpy(e->d_lay, &L, sizeof(Layout), hipMemcpyHostToDevice)) ||
        !HIP_OK(hipMemset(e->d_log, 0, lb)) ||
        !HIP_OK(hipMemset(e->d_cnt, 0, sizeof(prisma_counters_t) * n_replicas))) {
        prisma_destroy(e);
        return set_err(PRISMA_ERR_DEVICE, "device initialisation failed");
    }
    if (L.mem) {
        const bool ctrl = L.train || L.notify_dest || L.rng_mode;   // (ns-3 streams: CTRL instances, flow_next)
        e->k_step = prisma_mem_kernel(0, ctrl);
        e->k_reset = prisma_mem_kernel(1, ctrl);
        e->k_step_mlp = prisma_mem_kernel(2, ctrl);
    } else {
        // the --train echo and notify_dest paths (and the ns-3 streams) are compiled only into the
        // instances that need them; the tunnelled-overlay instances without them carry an 18-bit
        // decision index in relay entries (engine_layout.h rip_make).  Their wrap check (a relay
        // entry older than the log, PRISMA_EBIT_LOGWRAP) needs log ages up to log_cap to stay below
        // 2^18, so a log of 2^18 records or more takes the others (22-bit index)
        const bool ctrl = L.train || L.notify_dest || L.rng_mode || (L.tunnels && L.log_cap >= (1u << kRipDecBits));
        auto pick = ctrl ? pick_step_ctrl : prisma_pick_step_lite;
        auto pick_mlp = ctrl ? prisma_pick_step_ctrl_mlp : prisma_pick_step_lite_mlp;
        e->k_step = pick(L.FS, L.LS, L.tunnels != 0u);
        e->k_reset = pick_reset(L.FS, L.LS);
        e->k_step_mlp = pick_mlp(L.FS, L.LS, L.tunnels != 0u);
        e->kinfo.ctrl = ctrl ? 1u : 0u;
        e->kinfo.relay_ip = (L.tunnels && !ctrl) ? 1u : 0u;
        e->kinfo.relay_dec_bits = L.tunnels ? (ctrl ? 22u : kRipDecBits) : 0u;
    }
    e->kinfo.engine = L.mem ? PRISMA_ENGINE_MEMORY : PRISMA_ENGINE_REGISTER;
    e->kinfo.flow_slots = L.mem ? 0 : L.FS;
    e->kinfo.link_slots = L.mem ? 0 : L.LS;
    e->kinfo.tunnels = L.tunnels ? 1u : 0u;
    if (L.mem) e->kinfo.ctrl = (L.train || L.notify_dest || L.rng_mode) ? 1u : 0u;
    (void)hipFuncSetAttribute(e->k_step_mlp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds_mlp_bytes);
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
    P.spare = e->d_spare;
    P.rng = e->d_rng;
    return P;
}

static int launch(prisma_env_t* e, const void* kern, KParams P, void* stream) {
    (void)hipSetDevice(e->device);
    void* args[] = { &P };
    const size_t lds = kern == e->k_step_mlp ? e->lay.lds_mlp_bytes : e->lay.lds_bytes;
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
        // the weights may change between calls (training): re-interleave them every call,
        // on the caller's stream ahead of the step kernel (~1 us at GEANT size)
        const int N = e->lay.N, D = e->lay.max_deg;
        const size_t n = (size_t)N * mlp_rp_node_floats(D);
        (void)hipSetDevice(e->device);
        if (!e->d_mlp_rp && !HIP_OK(hipMalloc(&e->d_mlp_rp, n * sizeof(float))))
            return set_err(PRISMA_ERR_NOMEM, "hipMalloc of the interleaved DQN-buffer weights failed");
        const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(prisma_mlp_repack_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                           P.mlp, e->d_mlp_rp, N, D);
        if (!HIP_OK(hipGetLastError())) return set_err(PRISMA_ERR_LAUNCH, "repack kernel launch failed");
        P.mlp_rp = e->d_mlp_rp;
    }
    P.max_hops = max_hops;
    int rc = launch(e, P.mode == 4 ? e->k_step_mlp : e->k_step, P, stream);
    // with auto_reset (register engine) the step kernel already continued every replica whose
    // episode ended into the next one; this launch refreshes the spare images it used, and
    // starts the next episode of the replicas it could not continue (memory engine; a second
    // episode end in one launch)
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

extern "C" int prisma_compact_pending(prisma_env_t* e, const uint8_t* mask, const int32_t* obs, const int32_t* node,
                                      int32_t* ids_out, int32_t* obs_packed, int32_t* node_packed, int32_t* count_out,
                                      void* stream) {
    if (!e || !mask || !ids_out || !count_out || (obs_packed && !obs))
        return set_err(PRISMA_ERR_ARG, "null argument (mask, ids_out and count_out are required; obs with obs_packed)");
    (void)hipSetDevice(e->device);
    hipLaunchKernelGGL(prisma_compact_kernel, dim3(1), dim3(kCompactThreads), 0, (hipStream_t)stream, mask, obs, node,
                       e->R, e->lay.W, ids_out, obs_packed, node_packed, count_out);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return set_err(PRISMA_ERR_LAUNCH, std::string("compact launch failed: ") + hipGetErrorString(err));
    return PRISMA_OK;
}

extern "C" int prisma_expand_actions(prisma_env_t* e, const int32_t* ids, const int32_t* count,
                                     const int32_t* packed_actions, int32_t fill, int32_t* actions_out, void* stream) {
    if (!e || !ids || !count || !packed_actions || !actions_out) return set_err(PRISMA_ERR_ARG, "null argument");
    (void)hipSetDevice(e->device);
    hipLaunchKernelGGL(prisma_expand_kernel, dim3(1), dim3(kCompactThreads), 0, (hipStream_t)stream, ids, count,
                       packed_actions, e->R, fill, actions_out);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return set_err(PRISMA_ERR_LAUNCH, std::string("expand launch failed: ") + hipGetErrorString(err));
    return PRISMA_OK;
}

extern "C" int prisma_kernel_info(prisma_env_t* e, prisma_kernel_info_t* out) {
    if (!e || !out) return set_err(PRISMA_ERR_ARG, "null argument");
    *out = e->kinfo;
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
    out->engine = L.mem ? PRISMA_ENGINE_MEMORY : PRISMA_ENGINE_REGISTER;
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
    if (e->d_mlp_rp) (void)hipFree(e->d_mlp_rp);
    if (e->d_spare) (void)hipFree(e->d_spare);
    if (e->d_rng) (void)hipFree(e->d_rng);
    delete e;
}
