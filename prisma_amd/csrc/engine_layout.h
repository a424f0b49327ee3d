// engine_layout.h — per-replica state image shared by host sizing code and
// the gfx950 kernels.  The same byte image lives in HBM between launches
// and in LDS while a wavefront advances its replica.
#pragma once
#include <stdint.h>

namespace prisma {

constexpr int kWave = 64;

// event kinds in the candidate code (kind << 28 | index)
constexpr uint32_t K_PING = 0u, K_FLOW = 1u, K_COMPLETE = 2u, K_ARRIVE = 3u;

// 4-byte packet entry of a link ring; type in bits 0-1:
//   T_RELAY  data packet forwarded by a decision: bits 2-23 = that decision's
//            index mod 2^22, bits 24-31 = the packet's source node (its uid,
//            destination, start second, TTL, decision time and -- through the
//            deciding node and action -- its tunnel are read back from the
//            decision record in the HBM log).  The memory-resident engine's
//            kernels without the --train / notify_dest paths (which never read
//            the source back) carry the destination there instead, so an
//            arrival knows it before the record load returns (r_dst)
//            The register-resident engine's tunnelled-overlay kernels without
//            those paths carry what an IP header would instead (rip_make):
//            bits 2-19 the decision's index mod 2^18, bits 20-23 the live TTL
//            saturated at 15 (tunnels are at most 8 links long, so a saturated
//            TTL cannot expire inside one), bits 24-31 the tunnel's target
//            node: a switch inside the tunnel forwards the packet without the
//            record load (the host picks the other kernels when log_capacity
//            exceeds 2^18)
//   T_FRESH  data packet of a flow app on its access link: bits 2-9 its
//            destination, bit 10 parity of the start second, bits 11-31 uid
//            mod 2^21 (its source is the switch it arrives at)
//   T_PFWD / T_PBACK  ping forward / back (enum-and-constants.h:5-11):
//            bits 2-13 global tunnel id, bits 14-16 responder position on the
//            tunnel (ping-backs: 0 = first node after the origin), bits 17-30
//            round mod 2^14; the one-hop delay a ping-back carries sits in a
//            side table (Layout::s_pbd) keyed by (tunnel, position, round)
//   echo     small-signalling packet (--train): T_PBACK with bit 31 set,
//            bits 2-9 = its destination node (the data packet's last hop),
//            bits 10-30 = the signalled data packet's uid mod 2^21
//   big      big-signalling segment (--signaling, "NN"): T_PFWD with bit 31 set,
//            bits 2-13 = its generator (bpair: up to 4096, one per flow between
//            overlay neighbours -- 2 008 on ER-256), bits 14-30 = the generator's
//            send index (segment and NN index derive from it; < 2^17 per episode,
//            checked on the host)
constexpr uint32_t T_RELAY = 0u, T_FRESH = 1u, T_PFWD = 2u, T_PBACK = 3u;
constexpr uint32_t kEchoBit = 1u << 31;
__host__ __device__ inline uint32_t ent_type(uint32_t x) { return x & 3u; }
__host__ __device__ inline bool ent_is_data(uint32_t x) { return (x & 2u) == 0u; }
__host__ __device__ inline bool ent_is_echo(uint32_t x) { return (x & (kEchoBit | 3u)) == (kEchoBit | T_PBACK); }
__host__ __device__ inline bool ent_is_big(uint32_t x) { return (x & (kEchoBit | 3u)) == (kEchoBit | T_PFWD); }
constexpr uint32_t kGenBits = 12u, kGenSendBits = 17u, kGenSendMask = (1u << kGenSendBits) - 1u;
__host__ __device__ inline uint32_t g_make(uint32_t gen, uint32_t n) {
    return T_PFWD | kEchoBit | (gen << 2) | ((n & kGenSendMask) << (2u + kGenBits));
}
__host__ __device__ inline uint32_t g_gen(uint32_t x) { return (x >> 2) & ((1u << kGenBits) - 1u); }
__host__ __device__ inline uint32_t g_n(uint32_t x) { return (x >> (2u + kGenBits)) & kGenSendMask; }
// big-signalling generator g: source | destination << 8 | first link << 16 (switch link ids
// below 2^16: the memory-resident engine's ER-256 has 2 008)
__host__ __device__ inline uint32_t bp_src(uint32_t bp) { return bp & 255u; }
__host__ __device__ inline uint32_t bp_dst(uint32_t bp) { return (bp >> 8) & 255u; }
__host__ __device__ inline uint32_t bp_link(uint32_t bp) { return bp >> 16; }
__host__ __device__ inline uint32_t r_make(uint32_t dec, uint32_t src) {
    return T_RELAY | ((dec & ((1u << 22) - 1u)) << 2) | (src << 24);
}
__host__ __device__ inline uint32_t r_dec(uint32_t x) { return (x >> 2) & ((1u << 22) - 1u); }
__host__ __device__ inline uint32_t r_src(uint32_t x) { return x >> 24; }
__host__ __device__ inline uint32_t r_dst(uint32_t x) { return x >> 24; }   // (memory-resident, no ctrl)
// FIFO window of the same kernels: the first kQWin packets queued behind a busy transmitter of
// each link sit in LDS (Layout: after the wire-slot entries), the rest in the HBM ring
constexpr uint32_t kQWin = 4u;
constexpr uint32_t kRipDecBits = 18u, kRipMask = (1u << kRipDecBits) - 1u, kRipTtlSat = 15u;
__host__ __device__ inline uint32_t rip_make(uint32_t dec, uint32_t ttl, uint32_t tgt) {
    return T_RELAY | ((dec & kRipMask) << 2) | ((ttl < kRipTtlSat ? ttl : kRipTtlSat) << 20) | (tgt << 24);
}
__host__ __device__ inline uint32_t rip_dec(uint32_t x) { return (x >> 2) & kRipMask; }
__host__ __device__ inline uint32_t rip_ttl(uint32_t x) { return (x >> 20) & 15u; }
__host__ __device__ inline uint32_t rip_tgt(uint32_t x) { return x >> 24; }
__host__ __device__ inline uint32_t f_make(uint32_t dst, uint32_t start_parity, uint32_t uid) {
    return T_FRESH | (dst << 2) | (start_parity << 10) | (uid << 11);
}
__host__ __device__ inline uint32_t f_dst(uint32_t x) { return (x >> 2) & 255u; }
__host__ __device__ inline uint32_t f_parity(uint32_t x) { return (x >> 10) & 1u; }
__host__ __device__ inline uint32_t f_uid(uint32_t x) { return x >> 11; }
constexpr uint32_t kRoundBits = 14u, kRoundMask = (1u << kRoundBits) - 1u;
constexpr uint32_t kMaxTunnels = 4096u;      // 12-bit tunnel ids in ping entries
__host__ __device__ inline uint32_t p_make(uint32_t type, uint32_t tunnel, uint32_t pos, uint32_t round) {
    return type | (tunnel << 2) | (pos << 14) | ((round & kRoundMask) << 17);
}
__host__ __device__ inline uint32_t p_tunnel(uint32_t x) { return (x >> 2) & (kMaxTunnels - 1u); }
__host__ __device__ inline uint32_t p_pos(uint32_t x) { return (x >> 14) & 7u; }
__host__ __device__ inline uint32_t p_round(uint32_t x) { return (x >> 17) & kRoundMask; }
constexpr uint32_t kEchoUidMask = (1u << 21) - 1u;
__host__ __device__ inline uint32_t e_make(uint32_t uid, uint32_t to) {
    return T_PBACK | kEchoBit | (to << 2) | ((uid & kEchoUidMask) << 10);
}
__host__ __device__ inline uint32_t e_uid(uint32_t x) { return (x >> 10) & kEchoUidMask; }
__host__ __device__ inline uint32_t e_to(uint32_t x) { return (x >> 2) & 255u; }
constexpr uint32_t kRelayMask = (1u << 22) - 1u, kUidMask = (1u << 21) - 1u;

// pending-notification flags (Hdr::pend_ent[3])
constexpr uint32_t PEND_DEST = 1u, PEND_ECHO = 2u, PEND_CTRL = 4u;

struct Hdr {                 // 128 bytes at state offset 0
    int64_t  now;
    int64_t  ping_t;
    uint32_t ping_seq;
    uint32_t seq;
    uint32_t uid;
    uint32_t dec_count;
    uint32_t pend;           // 1: a decision waits for an action
    uint32_t pend_link;
    uint32_t pend_node;
    uint32_t pend_dec;
    uint32_t pend_ent[4];    // entry, dst, start second, PEND_* flags
    uint32_t ping_rounds;
    uint32_t episode;
    uint32_t over;
    uint32_t error;
    uint32_t stop;
    uint32_t hops_launch;
    uint64_t hops_total;
    uint64_t events_total;
    uint32_t pend_uid;       // uid of the pending data packet (echo payload)
    uint32_t pend_last;      // its last hop (echo destination)
    uint32_t pad[4];
};
static_assert(sizeof(Hdr) == 128, "Hdr size");
// LDS offsets of the header, the counters (152 B) and the pending observation
constexpr uint32_t kOffHdr = 0u, kOffCnt = 128u, kOffObs = 288u;

// Read-only topology image (HBM, one per engine), fixed-size arrays so every
// field sits at a compile-time offset from one base pointer: N <= 255,
// links incl. access links <= 256, tunnels <= 256, flows <= 512 (checked on
// the host).  Tunnelled overlays append the routing table route[N][N].
struct TopoImage {
    int32_t rowptr[256];         // CSR of directed switch links by source node
    int32_t ldst[256];           // far end of link l (access link E+u: u)
    int32_t lrev[256];           // reverse switch link
    int64_t acctx[256];          // access-link tx time of node u (ns)
    int32_t fsrc[512];
    int32_t fdst[512];
    double  fmean[512];          // mean inter-arrival of flow f (s)
    int32_t ovrow[256];          // CSR of tunnels (actions) by node; identity: == rowptr
    uint32_t tinfo[256];         // tunnel t: first link | target << 8 | origin << 16 | links << 24
    int32_t ovi[256];            // overlay index of node x (obs[0] of a packet for x), -1 if none
    int32_t ovnode[256];         // underlay id of overlay node i (ping timers, overlay order)
    uint32_t rinfo[256];         // ring of link l = entries [off, off + cap): off | cap << 16
    uint32_t tresp[256];         // tunnelled overlays: ping-back delay slot base of tunnel t | responder
                                 // position mask << 16 (overlay nodes on the tunnel, target included)
    uint32_t ctx[8];             // transmission time on a switch link of an entry of class
                                 // (type | echo bit << 2), ns (< 2^31)
    uint32_t ltx[256 * 8 * 2];   // link l, entry class c: (tx, tx + propagation), ns, low 32 bits --
                                 // ctx / acctx / etx / abtx and the switch links' propagation
                                 // delay folded per link (engine_core.h transmit_start)
    // signalling (read only by the --train instances, step_kernel.h CTRL)
    uint32_t esz[256];           // switch link l: size of an echo crossing it (its sender's payload
                                 // + 30 B: one hop on identity overlays, uniform on tunnelled ones)
    uint32_t etx[256];           // ... and its transmission time (ns)
    uint32_t abtx[256];          // access link of node u: transmission time of a big-signalling segment
    uint32_t bpair[256];         // big-signalling generator g: source | destination << 8 | first link << 16 (bp_*)
    uint32_t fseq[512];          // start-event seq of flow slot f (data flows; slot F: generator 0)
    int64_t  bs_period;          // generator send period (ns)
    uint32_t n_bsig;             // generators (all in flow slot F)
    uint32_t bs_nseg;            // segments per NN copy
    uint32_t bs_size;            // segment size on the wire (542 B)
    uint32_t pad_bs;
    // uint32_t route[N][N] follows (tunnelled overlays only): next link x -> y | hops(x, y) << 8
};
__host__ __device__ inline uint32_t ti_link(uint32_t ti) { return ti & 255u; }
__host__ __device__ inline uint32_t ti_tgt(uint32_t ti) { return (ti >> 8) & 255u; }
__host__ __device__ inline uint32_t ti_org(uint32_t ti) { return (ti >> 16) & 255u; }
__host__ __device__ inline uint32_t ti_len(uint32_t ti) { return ti >> 24; }

// Offsets (bytes) of every region; filled on the host, read by the kernels
// from a device copy.
struct Layout {
    int32_t N, E, L, F, W, max_deg, WCAP, MA;
    uint32_t topo_bytes, state_bytes, lds_bytes;
    uint32_t s_dcache;           // register engine: LDS offset of the flows' cached next-send delays
                                 // (engine_core.h flow_next), 0 where LDS has no room for them
    // state image (LDS offset 0) and the action table (LDS offset lds_state_bytes)
    uint32_t s_hdr, s_cnt, s_obs, s_wt, s_wseq, s_ring, s_win, s_pbd, s_mlp;
    int32_t  T, NO;              // tunnels, overlay nodes
    uint32_t tunnels;            // 1: tunnelled overlay (route table present)
    uint32_t PLEN;               // responder positions per tunnel (max tunnel length)
    uint32_t ring_total;         // packet slots over all link FIFOs
    uint32_t lds_state_bytes;    // LDS part of the image (bytes [0, lds_state_bytes))
    uint32_t s_regs;             // register part: 4 x [64*FS] + 16 x [64*LS] u32 arrays
    uint32_t PBK;                // ping-back delay slots per (tunnel, position) (power of two)
    int32_t  FS, LS;             // flow / link register slots per lane
    // link constants (identical on every switch link: sim.cc:414-433)
    int64_t  sw_txd, sw_txp, sw_txe, sw_prop;   // tx of data / ping / echo, propagation
    uint32_t qcap_s, qcap_a, qmax_bytes, acc_qmax_pkts;
    // scenario constants
    int64_t  t_end, ping_period;
    uint32_t data_size, ping_size, echo_size;
    uint32_t ma, ping_as_obs, auto_reset, notify_dest, train;
    uint32_t seed_lo, replica_base;
    uint32_t log_cap, rec_bytes;
    double   loss_penalty;
    float    loss_penalty_f;
    uint32_t rng_mode;           // PRISMA_RNG_*; ns-3 streams keep their state in the last kRngBytes
                                 // of the LDS image (engine_core.h ns3_exp_u01)
    // ---- dwords 64..: not in the LV register (read through the scalar cache) ----
    // memory-resident engine (mem = 1, prisma_engine_mem.hip): the LDS image holds
    // the header, counters, pending obs and the upper levels of the event tree;
    // s_ring / s_win / s_pbd are offsets into the HBM part of the state image.
    uint32_t mem;
    uint32_t n_leaf, n1, n2;     // event tree: sources (links + flow slots), flow blocks, top-level entries
    uint32_t s_lv1, s_lv2;       // LDS offsets of the flow block minima and the top level's image (16-B nodes)
    uint32_t g_lrec, g_keys;     // image offsets of the link records and the flow leaf keys
    uint32_t lrec_words;         // words per link record (32 or 64)
    uint32_t s_lkey, s_lkind;    // LDS offsets of the link leaf keys (time lo, seq) and kinds (bytes)
    // topology image offsets (memory-resident engine; variable-size arrays)
    uint32_t t_rowptr, t_ldst, t_lrev, t_acctx, t_fsrc, t_fdst, t_fmean;
    // ... and its signalling arrays (the --train instances): echo size / tx time per switch
    // link, big-segment tx time per access link, generators, start seqs, BigSig header
    uint32_t t_esz, t_etx, t_abtx, t_bpair, t_fseq, t_bsig;
    // register-resident engine: the [N][N] action table is staged into LDS (after the state
    // image) only where that costs no replica per CU; otherwise it is read from HBM (L2)
    uint32_t table_in_lds;
    uint32_t lds_mlp_bytes;      // LDS of a DQN-buffer launch (its 256 B of activations included)
    uint32_t table_bytes;        // the [N][N] action table
};
constexpr uint32_t kLVWords = 64u;           // Layout dwords held in the LV register

// ns-3 random streams (PRISMA_RNG_NS3, mrg32k3a.h): the replica's LDS image ends with the
// initial state of the next stream to be created (words 0-5) and the one-stream jump J
// (words 8-25); the engine's rng table (KParams::rng) holds J^(2^b), b < kMrgPowers, then
// per replica the state of stream rng_stream_offset (its flows' start streams follow) and of
// the first stream created while the simulation runs
constexpr uint32_t kRngBytes = 112u, kMrgPowers = 18u, kMrgRepWords = 12u;

// memory-resident engine: big-signalling constants (topology image at Layout::t_bsig)
struct BigSig {
    int64_t  period;             // generator send period (ns)
    uint32_t n_gen;              // generators (one event slot: flow slot F)
    uint32_t nseg;               // segments per NN copy
    uint32_t size;               // segment size on the wire (542 B)
    uint32_t tx_sw;              // its transmission time on a switch link (ns)
};

// memory-resident engine: one record of Layout::lrec_words (32 or 64) u32 words per
// link, accessed lane j <-> word j (one coalesced load / masked store per access)
enum : uint32_t {
    LR_P0 = 0, LR_P1, LR_P2, LR_QB, LR_CPT, LR_CPS, LR_WHT, LR_WHS,
    LR_PMLO, LR_PMMLO, LR_PMMHI, LR_PMWIN, LR_PAVLO, LR_PAVHI, LR_ODLO, LR_ODHI,
    LR_WT = 16,                  // wire slots: arrival time [WCAP], seq [WCAP], packet entry [WCAP]
};
constexpr uint32_t kMemMaxWire = 16u;

}  // namespace prisma
