/*
 * prisma_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's ns-3 packet-hop semantics (identity and
 * tunnelled overlays), used as the
 * parity checker for the HIP engine (tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg only; never linked into the product).
 *
 * The ns-3 C++ path of the reference cannot be built here (ns-3/ns3-gym,
 * waf, libzmq and protobuf are absent), so this is a literal
 * single-replica discrete-event restatement: a binary min-heap of
 * (time_ns, uid) events — ns-3's MapScheduler order — with one handler per
 * ns-3 callback, written independently of the GPU engine (own data
 * structures, own RNG code).  Parity is "GPU == oracle" bit-exact; parity of
 * the oracle with real ns-3 RNG draws is unpinned and is
 * pinned instead by analytic known answers and networkx fixtures.
 */
#ifndef PRISMA_ORACLE_H
#define PRISMA_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_config {
    int32_t n_nodes, n_links, n_flows, max_deg;
    const int32_t*  row_ptr;
    const int32_t*  link_dst;
    const int32_t*  link_rev;
    const int32_t*  flow_src;
    const int32_t*  flow_dst;
    const uint64_t* flow_rate_bps;
    uint64_t link_bps;
    int64_t  link_delay_ns;
    uint32_t max_buffer_bytes;
    uint32_t packet_size;
    double   sim_time_s;
    float    ping_interval_s;
    uint32_t ma_size;
    uint32_t ping_as_obs;
    uint32_t auto_reset;        /* ignored by the oracle (single episode) */
    double   loss_penalty;
    uint64_t seed;
    uint32_t replica;           /* global replica id (Philox key word 1)   */
    uint32_t episode;
    uint32_t notify_dest;       /* or_step also stops at destination and
                                   control (small-signalling) notifications;
                                   their action is ignored                 */
    uint32_t train;             /* --train: small-signalling echo per data
                                   notification at a non-source node       */
    /* overlay (sim.cc:455-476): decisions at overlay nodes over tunnels;
       identity overlays: n_overlay = n_nodes, tunnel t == link t          */
    int32_t n_overlay, n_tunnels;
    const int32_t* overlay_nodes;   /* [n_overlay] underlay id, overlay order */
    const int32_t* overlay_index;   /* [n_nodes] overlay index or -1         */
    const int32_t* ov_row_ptr;      /* [n_nodes + 1] tunnels of node u       */
    const int32_t* tun_dst;         /* [n_tunnels] overlay neighbour         */
    const int32_t* tun_link;        /* [n_tunnels] first physical link       */
    const int32_t* next_link;       /* [n_nodes * n_nodes] link x -> towards y
                                       (ns-3 global routing, -1 if x == y)   */
    /* signalling (sim.cc:142-144, 373-392, 634-647) */
    uint32_t signaling_type;    /* 0 "ideal", 1 "NN", 2 "target": echo payload */
    uint32_t big_signaling;     /* --signaling: NN-weight generators (with NN and train) */
    float    sync_step_s;       /* syncStep                                  */
    uint32_t big_signaling_bytes; /* bigSignalingSize                        */
    /* random streams: 0 Philox (the engine's default), 1 ns-3's RngStream MRG32k3a with one
       stream per RandomVariable object in creation order (simSeed = seed + replica as seed and
       run; streams from rng_stream_offset on: the objects ns-3 itself creates first) */
    uint32_t rng_mode;
    uint32_t rng_stream_offset;
} or_config_t;

typedef struct or_sim or_sim_t;

or_sim_t* or_create(const or_config_t* cfg);
void      or_destroy(or_sim_t* s);

/* Apply `action` to the pending decision (ignored if none is pending), then
 * run until the next decision that needs an action.  Returns 1 if a
 * decision is pending (obs written to obs_out[obs_width]), 0 if the episode
 * is over. */
int or_step(or_sim_t* s, int32_t action, int32_t* obs_out);

/* Like or_run_table, deciding with the DQN_buffer_model restatement over
 * packed fp32 weights (layout: prisma_amd.policies.StackedQNet.pack). */
int64_t or_run_mlp(or_sim_t* s, const float* weights, int64_t max_hops);
int32_t or_mlp_action(or_sim_t* s, const float* weights, int32_t v, const uint32_t* obs);
/* the same decision's fixed-order fp32 Q values into q_out[0..deg-1]; returns the action */
int32_t or_mlp_q(or_sim_t* s, const float* weights, int32_t v, const uint32_t* obs, float* q_out);
void or_mlp_q_batch(or_sim_t* s, const float* weights, int64_t n, const int32_t* nodes, const uint32_t* obs,
                    int32_t obs_stride, float* q_out, int32_t q_stride, int32_t* actions);
double or_det_expm1(double x);
float or_det_expm1f(float x);

/* Node of the pending notification (-1 if none). */
int32_t or_pending_node(const or_sim_t* s);

/* Run with a [N][N] action table until `max_hops` more hops were executed
 * or the episode ended.  Returns hops executed. */
int64_t or_run_table(or_sim_t* s, const uint8_t* table, int64_t max_hops);

/* Records (same byte layout as prisma_record_t; 32 + 4*obs_width bytes). */
int64_t or_record_count(const or_sim_t* s);
int32_t or_obs_width(const or_sim_t* s);
int64_t or_copy_records(const or_sim_t* s, int64_t first, int64_t count, void* out);

/* Counters with the same byte layout as prisma_counters_t. */
void or_counters(const or_sim_t* s, void* out);

/* Test diagnostics: out[0] data packets dropped on a FIFO inside a tunnel (not the deciding
 * node's first link), out[1] the longest switch FIFO now (packets waiting, excluding the one in
 * transmission), out[2] packets waiting in all switch FIFOs, out[3] switch FIFOs with more than
 * 4 waiting (deeper than the engine's LDS FIFO window, so part of them sits in the HBM ring). */
void or_diag(const or_sim_t* s, int64_t out[4]);

/* Optional event trace: (t_ns, seq, kind, id) per executed event. */
void    or_enable_trace(or_sim_t* s, int on);
int64_t or_trace_count(const or_sim_t* s);
int64_t or_copy_trace(const or_sim_t* s, int64_t first, int64_t count, int64_t* out4);

/* The decision "info" string of the reference (packet-manager.cc:119-176 +
 * data-packet-manager.cc:230-248) for the last decision, as the compat shim
 * needs it.  Returns bytes written (excluding NUL). */
int32_t or_last_info(const or_sim_t* s, char* buf, int32_t cap);

/* Exposed building blocks for known-answer tests. */
void     or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* ns-3 RngStream (rng-stream.cc, L'Ecuyer et al. 2002): A1^(2^e) mod m1 and A2^(2^e) mod m2
   (out[0..8], out[9..17], row-major), and the first RandU01 of stream `stream`, substream `run`
   of package seed `seed` */
void     or_mrg_pow2(int e, uint64_t out[18]);
double   or_mrg_first_u01(uint32_t seed, uint64_t stream, uint64_t run);
double   or_det_log(double x);
int64_t  or_seconds_to_ns(double s);
uint64_t or_py_micros(int64_t t_ns);

#ifdef __cplusplus
}
#endif
#endif
