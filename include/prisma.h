/*
 * prisma.h — C-ABI of the MI355X-native PRISMA packet-hop engine.
 *
 * One shared library (libprisma_amd.so, built from prisma_amd/csrc/) holds
 * R independent topology replicas of PRISMA's ns-3 routing scenario as
 * structure-of-arrays state in HBM and advances them with hand-written
 * gfx950 kernels.  Plain C types only: pointers, sizes, status codes.
 * Device pointers are HIP device addresses (e.g. torch.Tensor.data_ptr()).
 *
 * Each entry point replaces one piece of the reference's per-node
 * ns3-gym path (all citations relative to the reference repo root):
 *
 *   prisma_create      sim.cc:274-683 (topology, links, flows, per-node envs)
 *                      + ns3env.py:378-403 (Ns3Env.__init__ / SimInitMsg)
 *   prisma_reset       sim.cc:253-261 (SetSeed/SetRun) + Simulator start,
 *                      ns3env.py:426-445 (Ns3Env.reset)
 *   prisma_step        ns3env.py:420-423 (Ns3Env.step) ==
 *                      packet-routing-gym.cc:197-213 (ExecuteActions) then
 *                      Simulator::Run until the next
 *                      packet-routing-gym.cc:231-267 (NotifyPktRcv -> Notify)
 *                      with the observation of data-packet-manager.cc:171-206
 *   prisma_run         the same loop with the forwarding decision fused
 *                      in-kernel (forwarder.py:149-195 for table policies:
 *                      SP next-hop table, DQ-routing argmin table)
 *   prisma_read_counters  compute-stats-v2.cc:87-266 (ComputeStats) and the
 *                      forwarder.py:308-431 per-episode trackers
 *   prisma_log_view    the per-hop replay transitions of forwarder.py:352-379
 *                      and the loss transitions of forwarder.py:214-244
 *   prisma_destroy     ns3env.py:452-455 (Ns3Env.close) /
 *                      Ns3ZmqBridge.send_close_command
 *
 * Error behaviour: every call returns PRISMA_OK (0) or a negative status;
 * prisma_last_error() returns a static description of the last failure in
 * the calling thread.  The library never calls exit() (the reference
 * NS_FATAL_ERRORs on bad matrices, sim.cc:310-313; here that is
 * PRISMA_ERR_CONFIG).  Per-replica runtime faults (a ring or wire overflow
 * that the host-side sizing should have excluded) set bits in
 * prisma_counters_t.error and stop that replica; they never touch memory
 * outside the replica's own state.
 */
#ifndef PRISMA_AMD_PRISMA_H
#define PRISMA_AMD_PRISMA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRISMA_ABI_VERSION 10

/* status codes */
#define PRISMA_OK              0
#define PRISMA_ERR_CONFIG     -1   /* invalid topology / parameters        */
#define PRISMA_ERR_NOMEM      -2   /* hipMalloc failed                     */
#define PRISMA_ERR_DEVICE     -3   /* no HIP device / wrong architecture   */
#define PRISMA_ERR_LAUNCH     -4   /* kernel launch failed                 */
#define PRISMA_ERR_ARG        -5   /* null handle / bad pointer / bad size */
#define PRISMA_ERR_STATE      -6   /* call not valid in current state      */

/* policy modes for prisma_run (fused decision) */
#define PRISMA_POLICY_TABLE    1   /* action = table[node * n_nodes + dst]
                                      (underlay ids)                       */
#define PRISMA_POLICY_DQN_BUFFER 2 /* in-kernel DQN_buffer_model (models.py:258-306)
                                      over packed fp32 weights, D = max_deg:
                                      W1[N][N][32] b1[N][32] Wb[N][D][32] bb[N][32]
                                      W2[N][64][64] b2[N][64] W3[N][64][64] b3[N][64]
                                      W4[N][64][D] b4[N][D]; x @ W convention;
                                      N = n_nodes, rows by underlay id; the
                                      one-hot input is obs[0] (the overlay
                                      index of the destination)               */

/* engine selection (prisma_params_t.engine) */
#define PRISMA_ENGINE_AUTO     0   /* register-resident when the topology fits it */
#define PRISMA_ENGINE_REGISTER 1   /* replica state in VGPRs + LDS: <= 255 nodes,
                                      256 links / tunnels / big-signalling
                                      generators, 512 flows                      */
#define PRISMA_ENGINE_MEMORY   2   /* replica state in HBM under an event tree:
                                      <= 256 nodes, links + flows <= 262 144,
                                      <= 4 096 generators, identity overlays
                                      (ER-256); every signalling type            */

/* signalling type (prisma_params_t.signaling_type, argument_parser.py:72 /
   sim.cc:142, 373-392): the payload of the --train small-signalling echo a node
   sends, 0 B ("ideal"), 8 + 8 (overlay degree + 1) B ("NN") or 24 B ("target") */
#define PRISMA_SIGNALING_IDEAL  0
#define PRISMA_SIGNALING_NN     1
#define PRISMA_SIGNALING_TARGET 2

/* random streams (prisma_params_t.rng_mode) */
#define PRISMA_RNG_PHILOX 0        /* counter-based Philox4x32-10 per (seed, replica, flow,
                                      draw, episode): replicas and episodes independent [default] */
#define PRISMA_RNG_NS3    1        /* ns-3's RngStream MRG32k3a (rng-stream.cc): one stream per
                                      RandomVariable object in creation order -- a Uniform per flow
                                      for its start offset (sim.cc:610-620), then per packet the
                                      Uniform of SendPacket (poisson-application.cc:311) and the
                                      Exponential of ScheduleNextTx (:281); simSeed = seed +
                                      replica id as seed and run (sim.cc:253-254), the same streams
                                      every episode (run_ns3.py restarts ns-3 with the same seed) */

/* per-decision status (prisma_record_t.status) */
#define PRISMA_ST_PENDING      0   /* waiting for an action (prisma_step)  */
#define PRISMA_ST_ENQUEUED     1   /* forwarded; a later record has prev==d */
#define PRISMA_ST_DROPPED      2   /* output FIFO overflow: loss transition */
#define PRISMA_ST_DESTINATION  3   /* packet reached its destination       */
#define PRISMA_ST_DISCARDED    4   /* action >= degree: silently discarded  */

/* runtime error bits (prisma_counters_t.error) */
#define PRISMA_EBIT_RING       1u  /* link ring overflow                   */
#define PRISMA_EBIT_WIRE       2u  /* more packets on a wire than sized    */
#define PRISMA_EBIT_ACKORDER   4u  /* ping-back acknowledging a round more
                                      than 64 rounds behind a lost one     */
#define PRISMA_EBIT_TIME       8u  /* time beyond the representable range  */
#define PRISMA_EBIT_LOGWRAP   16u  /* a hop outlived log_capacity decisions */
#define PRISMA_EBIT_PINGIDX   32u  /* a ping-back crossing an overlay node
                                      carried a tunnel index beyond that
                                      node's degree (out of range of the
                                      reference's vectors: undefined there) */

/*
 * Topology of one replica.  Directed switch links (the PHYSICAL underlay)
 * are numbered in CSR order: links row_ptr[u] .. row_ptr[u+1]-1 leave node
 * u towards link_dst[] in ascending neighbour id.  link_rev[l] is the
 * opposite direction of l.  Flows are listed in (src, dst) lexicographic
 * order of underlay ids, overlay pairs only, with their load-scaled integer
 * bit rate ceil(trunc_parse(TM[s][d]) * load_factor) (sim.cc:494-514,
 * 599-631, ns-3 DataRate parse).
 *
 * Overlay (sim.cc:455-476): n_overlay = 0 means the identity overlay (every
 * node is an overlay node, overlay adjacency == physical adjacency, the
 * abilene / geant examples).  Otherwise overlay_nodes[i] is the underlay id
 * of overlay node i (the inverse of map_overlay.txt) and overlay_adj the
 * [n_overlay][n_overlay] 0/1 overlay adjacency.  The actions of overlay node
 * u are its overlay neighbours in ascending overlay index; an action is a
 * TUNNEL along the underlay route ns-3 global routing installs (unit
 * metrics: at every hop the lowest-id neighbour on a shortest path, computed
 * by the library).  max_deg is the largest overlay degree.
 */
typedef struct prisma_topology {
    int32_t n_nodes;
    int32_t n_links;            /* directed switch links E                 */
    int32_t n_flows;
    int32_t max_deg;
    const int32_t*  row_ptr;    /* [n_nodes + 1]                           */
    const int32_t*  link_dst;   /* [n_links]                               */
    const int32_t*  link_rev;   /* [n_links]                               */
    const int32_t*  flow_src;   /* [n_flows]                               */
    const int32_t*  flow_dst;   /* [n_flows]                               */
    const uint64_t* flow_rate_bps; /* [n_flows], > 0                       */
    int32_t n_overlay;          /* 0: identity overlay                     */
    const int32_t* overlay_nodes;  /* [n_overlay] underlay ids            */
    const int32_t* overlay_adj;    /* [n_overlay * n_overlay] 0/1         */
} prisma_topology_t;

/* scenario parameters (argument_parser.py:34-94 defaults in brackets) */
typedef struct prisma_params {
    uint64_t link_bps;          /* switch link rate            [500000]    */
    int64_t  link_delay_ns;     /* propagation delay           [1 ms]      */
    uint32_t max_buffer_bytes;  /* DropTail byte limit         [16260]     */
    uint32_t packet_size;       /* UDP payload bytes           [512]       */
    double   sim_time_s;        /* episode length              [60]        */
    float    ping_interval_s;   /* pingPacketIntervalTime      [0.2f]      */
    uint32_t ma_size;           /* movingAverageObsSize        [5]         */
    uint32_t ping_as_obs;       /* pingAsObs                   [1]         */
    uint32_t auto_reset;        /* start next episode when one ends        */
    double   loss_penalty;      /* ((16260+542)*8/cap+0.001)*N             */
    uint64_t seed;              /* simSeed                     [100]       */
    uint32_t replica_base;      /* global id of replica 0 (multi-GPU)      */
    uint32_t log_capacity;      /* records kept per replica (power of 2 in
                                   [1024, 2^22]; must exceed the decisions
                                   made while one packet crosses one link) */
    uint32_t notify_dest;       /* prisma_step also stops at arrivals at the
                                   destination (done=True notifications) and
                                   at control arrivals, obs [1000, a, b, c]:
                                   small-signalling echo: a = signalled uid,
                                   b = its size on the wire, c = 0; big
                                   signalling: a = NN index, b = segment
                                   index, c = 0x10000 | overlay index of the
                                   signalling node; the action given for
                                   them is ignored                          */
    uint32_t train;             /* --train: every data notification at a
                                   non-source node echoes a small-signalling
                                   packet to its last hop
                                   (data-packet-manager.cc:301-347)        */
    uint32_t engine;            /* PRISMA_ENGINE_* (0 = auto)              */
    /* ---- ABI 7 ---- */
    uint32_t signaling_type;    /* PRISMA_SIGNALING_*          ["ideal"]   */
    uint32_t big_signaling;     /* --signaling (signalingSim) with "NN" and
                                   --train: per flow between overlay
                                   neighbours, a BigSignalingGenerator-
                                   Application sending 512-B NN-weight
                                   segments to the neighbour from AppStartTime
                                   on (sim.cc:634-647, big-signaling-
                                   application.cc:224-309)                 */
    float    sync_step_s;       /* syncStep: seconds per NN copy   [1.0]   */
    uint32_t big_signaling_bytes; /* bigSignalingSize: NN bytes; sim.cc's own
                                     default is 35328, the CLI's (argument_parser.py:74)
                                     512 = one segment per NN; prisma_amd's
                                     config.engine_params passes 512 */
    /* ---- ABI 8 ---- */
    uint32_t rng_mode;          /* PRISMA_RNG_*                    [0]     */
    uint32_t rng_stream_offset; /* PRISMA_RNG_NS3: streams ns-3 itself
                                   creates before sim.cc's flow loop (ARP,
                                   ICMPv6, global routing of every node;
                                   version-dependent, so a parameter)      */
} prisma_params_t;

/*
 * One decision record = one data-packet notification of the reference
 * (PacketRoutingEnv::Notify for a valid DATA packet), i.e. one row the
 * reference Forwarder turns into a replay transition.  The transition of
 * decision d is (obs_d, action_d, r, obs_{d'}, done_{d'}) where d' is the
 * record with prev == d and r = reward_{d'}; or, if status_d == DROPPED,
 * (obs_d, action_d, loss_penalty, [dst, 0...], true) (forwarder.py:226-240).
 * reward is the reference's hop_time_real = curr_time - t_decision computed
 * on the microsecond-formatted times (packet-manager.cc:127-128 ->
 * forwarder.py:208,360), bit-identical to the Python float.
 * Record size is 32 + 4 * obs_width bytes (obs_width = 1 + max_deg rounded up
 * to a multiple of 4, so records are whole 16-byte rows).
 */
typedef struct prisma_record {
    int64_t  t_ns;
    uint32_t uid;
    int32_t  prev;
    double   reward;
    uint8_t  node;
    uint8_t  dst;
    uint16_t start_s;           /* whole second the packet was sent (its
                                   start-time tag, packet-manager.cc)       */
    int8_t   action;
    uint8_t  status;
    uint8_t  ttl;               /* IP TTL the packet arrived with (255 from
                                   its app; -1 per intermediate underlay hop
                                   of a tunnel, Ipv4L3Protocol::IpForward)  */
    uint8_t  episode;           /* episode index mod 256                   */
    uint32_t obs[];             /* [obs_width]                             */
} prisma_record_t;

/* Per-replica counters: ComputeStats (compute-stats-v2.cc) + engine stats */
typedef struct prisma_counters {
    uint64_t events;            /* discrete events executed                */
    uint64_t hops;              /* decisions resulting in enqueue or drop  */
    uint64_t decisions;         /* all data notifications (incl. dest)     */
    uint64_t hop_deg_sum;       /* sum of deg(u) over executed hops        */
    int64_t  now_ns;            /* simulation clock                        */
    double   reward_sum;        /* sum of completed hop rewards + penalties*/
    int32_t  ov_injected;       /* compute-stats-v2.cc:131-134             */
    int32_t  ov_arrived;
    int32_t  ov_lost;
    int32_t  un_injected;
    int32_t  un_arrived;
    int32_t  un_lost;
    int32_t  bytes_data;        /* addGlobalBytesData                      */
    int32_t  bytes_signaling;   /* addGlobalBytesSignaling                 */
    float    cost_sum;          /* running float sum of m_globalCost       */
    float    e2e_sum;           /* running float sum of m_globalE2eDelay   */
    int32_t  cost_n;
    int32_t  e2e_n;
    uint32_t episode;
    uint32_t ping_rounds;
    uint32_t seq;               /* events scheduled (ns-3 uid analogue)    */
    uint32_t uid;               /* data packets created                    */
    uint32_t dec_count;         /* records written (monotonic)             */
    uint32_t ctrl_dropped;      /* ping packets lost on full FIFOs         */
    uint32_t error;             /* PRISMA_EBIT_* bits                      */
    uint32_t episode_over;      /* 1 once the current episode ended        */
    uint64_t hops_total;        /* hops over all episodes since reset      */
    uint64_t events_total;      /* events over all episodes since reset    */
    float    un_cost_sum;       /* running float sum of m_globalUnderlayCost
                                   (loss penalties of data packets dropped
                                   at their own destination node, which a
                                   tunnel can cross)                       */
    int32_t  un_cost_n;
} prisma_counters_t;

/* library-owned device buffers (valid until prisma_destroy) */
typedef struct prisma_log_view {
    void*     records;          /* [n_replicas][log_capacity] records      */
    uint32_t  record_bytes;
    uint32_t  log_capacity;
    int32_t   obs_width;
    int32_t   n_replicas;
} prisma_log_view_t;

typedef struct prisma_env prisma_env_t;

int         prisma_abi_version(void);
const char* prisma_last_error(void);
/* 12 hex digits: hash of the sources + compile flags this library was built
 * from (prisma_amd/buildid.py); loaders refuse a library whose id differs
 * from the sources beside it. */
const char* prisma_build_id(void);

/* Size the per-replica state for this topology and allocate it on
 * `device`.  Validates shapes and ids up front. */
int prisma_create(const prisma_topology_t* topo, const prisma_params_t* params,
                  int32_t n_replicas, int32_t device, prisma_env_t** out);

/* Start episode `episode` of every replica (replica r uses Philox key
 * (seed, replica_base + r)).  Asynchronous on `stream` (hipStream_t). */
int prisma_reset(prisma_env_t* env, uint32_t episode, void* stream);

/* Apply one action per replica to its pending decision (actions may be
 * NULL on the first call after reset), then advance every replica to its
 * next pending decision.  obs_out: device int32 [n_replicas][obs_width];
 * mask_out: device uint8 [n_replicas] (1 = a decision is pending, 0 =
 * episode over); node_out: device int32 [n_replicas], the node deciding
 * (-1 if none).  Any output may be NULL.  A launch never crosses an episode
 * boundary: a replica whose episode ends reports mask 0, and with
 * params.auto_reset it starts its next episode before the call returns (on
 * `stream`), so its next step continues there. */
int prisma_step(prisma_env_t* env, const int32_t* actions, int32_t* obs_out,
                uint8_t* mask_out, int32_t* node_out, void* stream);

/* Fused policy: advance every replica by up to max_hops hops, deciding
 * in-kernel: PRISMA_POLICY_TABLE with `policy_data` = device uint8
 * [n_nodes][n_nodes] action table (SP, DQ-routing argmin), or
 * PRISMA_POLICY_DQN_BUFFER with `policy_data` = device packed fp32 weights
 * (row-major, as StackedQNet.pack() lays them out; the library copies them
 * into an interleaved per-node layout on `stream` before each such launch,
 * so weights updated in place between calls take effect on the next call;
 * calls on one env are ordered by their streams: keep one stream per env).
 * A replica stops early at the end of its episode; with params.auto_reset
 * it starts the next episode before the call returns (one launch never
 * crosses an episode boundary). */
int prisma_run(prisma_env_t* env, int32_t policy, const void* policy_data,
               int32_t max_hops, void* stream);

/* Copy per-replica counters (n_replicas entries) to host memory.
 * Synchronises `stream`. */
int prisma_read_counters(prisma_env_t* env, prisma_counters_t* host_out,
                         void* stream);

/* Device pointer to the per-replica counters array (prisma_counters_t
 * [n_replicas]), for device-side reductions / collectives. */
int prisma_counters_device(prisma_env_t* env, void** dev_ptr);

int prisma_log_view(prisma_env_t* env, prisma_log_view_t* out);

/* Device-to-device copy of the whole log ring ([n_replicas][log_capacity]
 * records) into caller memory of at least `bytes` bytes, on `stream`. */
int prisma_copy_log(prisma_env_t* env, void* dst_device, uint64_t bytes, void* stream);

/* Device-to-device copy of the counters (prisma_counters_t [n_replicas]). */
int prisma_copy_counters(prisma_env_t* env, void* dst_device, void* stream);

/* Gather n decision records, record dec[i] of replica replica[i] (both
 * device arrays), into dst_device (n * record_bytes bytes).  The caller
 * keeps dec[i] within the last log_capacity decisions of that replica. */
int prisma_gather_records(prisma_env_t* env, const int32_t* replica, const uint32_t* dec,
                          int32_t n, void* dst_device, void* stream);

/* Active-replica compaction (ABI 9) for a batched external policy, which then
 * evaluates only the replicas with a pending decision -- the reference's
 * Forwarder steps only the nodes that were notified (ns3env.py:417-423,
 * forwarder.py:135-195).  From the outputs of a prisma_step (mask [R], obs
 * [R][obs_width], node [R]; obs / node may be NULL): ids_out[0..count) = the
 * replica ids with mask 1 in ascending order, obs_packed[i] = obs row of
 * ids_out[i], node_packed[i] = its deciding node, count_out[0] = count (all
 * device int32; obs_packed / node_packed may be NULL).  A wavefront ballot and
 * a prefix sum of the wave totals; one launch on `stream`, no host sync. */
int prisma_compact_pending(prisma_env_t* env, const uint8_t* mask, const int32_t* obs,
                           const int32_t* node, int32_t* ids_out, int32_t* obs_packed,
                           int32_t* node_packed, int32_t* count_out, void* stream);

/* The inverse for the actions: actions_out[r] = fill for every replica, then
 * actions_out[ids[i]] = packed_actions[i] for i < count[0] (device arrays);
 * actions_out then feeds prisma_step. */
int prisma_expand_actions(prisma_env_t* env, const int32_t* ids, const int32_t* count,
                          const int32_t* packed_actions, int32_t fill, int32_t* actions_out,
                          void* stream);

/* The step-kernel instances prisma_create picked for this env (ABI 10), as
 * the library decided, for profiles and tests (the demangled kernel name is
 * prisma_step_kernel_t<flow_slots, link_slots, MLP, tunnels, ctrl> on the
 * register engine, prisma_mem_step_kernel<MLP, ctrl> on the memory engine). */
typedef struct prisma_kernel_info {
    uint32_t engine;            /* PRISMA_ENGINE_REGISTER or _MEMORY       */
    int32_t  flow_slots;        /* template slots (register engine; else 0) */
    int32_t  link_slots;
    uint32_t tunnels;           /* tunnelled-overlay instances              */
    uint32_t ctrl;              /* --train / notify_dest / ns-3 stream paths
                                   compiled in (also: tunnelled overlays with
                                   log_capacity >= 2^18)                    */
    uint32_t relay_ip;          /* relay entries carry (decision, TTL, tunnel
                                   target) and FIFO windows sit in LDS       */
    uint32_t relay_dec_bits;    /* decision-index bits of a relay entry (18
                                   with relay_ip, 22 otherwise; 0 without
                                   tunnels): the log-wrap check sees ages up
                                   to 2^bits                               */
} prisma_kernel_info_t;
int prisma_kernel_info(prisma_env_t* env, prisma_kernel_info_t* out);

/* Bytes of per-replica state (the LDS image) and LDS bytes per workgroup. */
int prisma_state_bytes(prisma_env_t* env, uint32_t* state_bytes,
                       uint32_t* lds_bytes);

/* Sizing without a device: validates topo/params exactly as prisma_create
 * does and reports the per-replica footprint (any pointer may be NULL). */
typedef struct prisma_plan {
    uint32_t state_bytes;       /* HBM state image per replica             */
    uint32_t lds_bytes;         /* LDS per workgroup (= per replica)       */
    uint32_t lds_state_bytes;   /* LDS part of the image                   */
    uint32_t ring_entries;      /* packet slots over all link FIFOs        */
    uint32_t record_bytes;      /* decision record size                    */
    int32_t  obs_width;
    int32_t  flow_slots;        /* register slots per lane (64 flows each) */
    int32_t  link_slots;        /* register slots per lane (64 links each) */
    uint32_t engine;            /* PRISMA_ENGINE_REGISTER or _MEMORY       */
} prisma_plan_t;
int prisma_plan(const prisma_topology_t* topo, const prisma_params_t* params, prisma_plan_t* out);

void prisma_destroy(prisma_env_t* env);

#ifdef __cplusplus
}
#endif
#endif /* PRISMA_AMD_PRISMA_H */
