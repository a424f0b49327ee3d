// engine_layout.h — per-replica state image shared by host sizing code and
// the gfx950 kernels.  The same byte image lives in HBM between launches
// and in LDS while a wavefront advances its replica.
#pragma once
#include <stdint.h>

namespace prisma {

constexpr int kWave = 64;

// event kinds in the candidate code (kind << 28 | index)
constexpr uint32_t K_PING = 0u, K_FLOW = 1u, K_COMPLETE = 2u, K_ARRIVE = 3u;

// packet types (enum-and-constants.h:5-11)
constexpr uint32_t T_DATA = 0u, T_PING_FWD = 3u, T_PING_BACK = 4u;

// 8-byte packet entry (uint2) of a link ring:
//   data: x = type(3) | dst(8) << 3 | fresh(1) << 11 | start second(12) << 12
//         y = decision index of the previous hop (fresh packet: its uid)
//   ping: x = type(3) | tunnel(8) << 3 | round(21) << 11
//         y = ping-back one-hop delay (f32 bits)
// The uid and decision time of a forwarded packet are read back from its
// previous decision record in the HBM log when it arrives.
__host__ __device__ inline uint32_t ent_type(uint32_t x) { return x & 7u; }
__host__ __device__ inline uint32_t d_dst(uint32_t x) { return (x >> 3) & 255u; }
__host__ __device__ inline uint32_t d_fresh(uint32_t x) { return (x >> 11) & 1u; }
__host__ __device__ inline uint32_t d_start(uint32_t x) { return x >> 12; }
__host__ __device__ inline uint32_t p_tunnel(uint32_t x) { return (x >> 3) & 255u; }
__host__ __device__ inline uint32_t p_round(uint32_t x) { return x >> 11; }
__host__ __device__ inline uint32_t d_make(uint32_t dst, uint32_t fresh, uint32_t start_s) {
    return T_DATA | (dst << 3) | (fresh << 11) | (start_s << 12);
}
__host__ __device__ inline uint32_t p_make(uint32_t type, uint32_t tunnel, uint32_t round) {
    return type | (tunnel << 3) | (round << 11);
}

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
    uint32_t pend_ent[4];
    uint32_t ping_rounds;
    uint32_t episode;
    uint32_t over;
    uint32_t error;
    uint32_t stop;
    uint32_t hops_launch;
    uint64_t hops_total;
    uint64_t events_total;
    uint32_t pad[6];
};
static_assert(sizeof(Hdr) == 128, "Hdr size");

struct LinkState {           // 32 bytes
    int64_t  complete_t;
    uint32_t complete_seq;
    uint32_t q_bytes;        // bytes waiting in the FIFO (excl. the wire)
    uint16_t head, txp, tail, n_wire;
    uint16_t n_queue, busy, pad0, pad1;
};
static_assert(sizeof(LinkState) == 32, "LinkState size");

struct PingMeta {            // 16 bytes per directed link (= tunnel of its source)
    int32_t  acked_last;     // highest ping index acknowledged, -1 none
    int32_t  first_hole;     // lowest never-acknowledged index below acked_last, -1 none
    uint32_t win_n;
    uint32_t win_head;
};

// Offsets (bytes) of every region; filled on the host, passed by value.
struct Layout {
    int32_t N, E, L, F, W, max_deg, WCAP, MA;
    uint32_t topo_bytes, state_bytes, lds_bytes, table_bytes;
    // topology image (LDS offset 0)
    uint32_t t_rowptr, t_ldst, t_lrev, t_acctx, t_fsrc, t_fdst, t_fmean, t_table;
    // state image (LDS offset topo_bytes)
    uint32_t s_hdr, s_cnt, s_obs, s_wt, s_wseq, s_ring, s_win;
    uint32_t lds_state_bytes;    // LDS part of the image (bytes [0, lds_state_bytes))
    uint32_t s_regs;             // register part: 4 x [64*FS] + 14 x [64*LS] u32 arrays
    int32_t  FS, LS;             // flow / link register slots per lane
    // link constants (identical on every switch link: sim.cc:414-433)
    int64_t  sw_txd, sw_txp, sw_prop;
    uint32_t qcap_s, qcap_a, qmax_bytes, acc_qmax_pkts;
    // scenario constants
    int64_t  t_end, ping_period;
    uint32_t data_size, ping_size;
    uint32_t ma, ping_as_obs, auto_reset;
    uint32_t seed_lo, replica_base;
    uint32_t log_cap, rec_bytes;
    double   loss_penalty;
    float    loss_penalty_f;
    uint32_t pad;
};

}  // namespace prisma
