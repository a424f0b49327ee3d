"""HIP engine vs the CPU oracle on the same seeded inputs (bit-exact), through the C-ABI."""
import numpy as np
import pytest
import torch

from prisma_amd.config import engine_params
from prisma_amd.engine import PrismaEngine
from prisma_amd.records import (COUNTERS_DTYPE, ST_DESTINATION, ST_DROPPED, ST_ENQUEUED, ST_PENDING,
                                transitions)
from prisma_amd.topology import Topology, sp_next_hop_table
from parity_util import check_near_ties, compare_steady

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]

CNT_KEYS = [k for k in COUNTERS_DTYPE.names if k not in ("hops_total", "events_total")]


def assert_counters_equal(g, o, r):
    bad = [(k, g[k], o[k]) for k in CNT_KEYS if g[k] != o[k]]
    assert not bad, f"replica {r}: counters differ {bad}"


def run_table_both(oracle_mod, topo, params, R, H, table, launches=1, replicas=None):
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    t = torch.from_numpy(np.ascontiguousarray(table)).cuda()
    for _ in range(launches):
        eng.run(t, H // launches)
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in (range(R) if replicas is None else replicas):
        o = oracle_mod.OracleSim(topo, params, replica=params["replica_base"] + r)
        o.run_table(table, H)
        ref = o.records()
        assert cnt[r]["error"] == 0
        assert int(cnt[r]["dec_count"]) == len(ref)
        n = min(len(ref), eng.log_capacity)
        got = eng.records(r, len(ref) - n, n, log_host=log)
        assert got.tobytes() == ref[len(ref) - n:].tobytes(), f"replica {r} records differ"
        assert_counters_equal(cnt[r], o.counters(), r)
    eng.close()
    return cnt


@pytest.mark.parametrize("name,tm,lf,ping,seed,train", [
    ("abilene", 0, 1.0, 1, 100, 0), ("abilene", 0, 1.0, 0, 100, 0), ("abilene", 2, 2.0, 1, 7, 0),
    ("abilene", 3, 0.5, 0, 12345, 0), ("geant", 0, 1.0, 1, 100, 0), ("geant", 1, 1.5, 0, 3, 0),
    ("abilene", 0, 1.0, 1, 100, 1), ("abilene", 1, 2.0, 0, 9, 1), ("geant", 0, 1.0, 1, 11, 1),
])
def test_table_policy_parity(oracle_mod, name, tm, lf, ping, seed, train):
    topo = Topology.example(name, tm, lf)
    params = engine_params(topo, sim_time_s=15.0, ping_as_obs=ping, seed=seed, replica_base=5, train=train)
    run_table_both(oracle_mod, topo, params, 6, 2500, sp_next_hop_table(topo))


def test_multi_launch_equals_single_launch(oracle_mod):
    """State staged out to HBM and back between launches changes nothing."""
    topo = Topology.example("abilene")
    params = engine_params(topo, sim_time_s=10.0, ping_as_obs=1)
    run_table_both(oracle_mod, topo, params, 4, 1200, sp_next_hop_table(topo), launches=8)


def test_dq_routing_argmin_table_parity(oracle_mod):
    from prisma_amd.policies import StackedQNet
    topo = Topology.example("abilene")
    net = StackedQNet(topo, "routing", seed=11)
    table = net.argmin_table().cpu().numpy()
    # the table is exactly the per-decision argmin of the torch model
    node = torch.arange(11).repeat_interleave(11).cuda()
    obs = torch.zeros(121, 4, dtype=torch.int32).cuda()
    obs[:, 0] = torch.arange(11).repeat(11).int().cuda()
    acts = net.act(obs, node).view(11, 11).cpu().numpy()
    off = ~np.eye(11, dtype=bool)
    assert np.array_equal(acts[off], table[off])
    params = engine_params(topo, sim_time_s=10.0, ping_as_obs=1)
    run_table_both(oracle_mod, topo, params, 4, 1500, table)


def test_external_policy_step_parity(oracle_mod):
    """Gym-style step(): random actions (2% invalid -> discarded) applied to both."""
    topo = Topology.example("abilene")
    params = engine_params(topo, sim_time_s=10.0, ping_as_obs=1)
    R = 12
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    orcs = [oracle_mod.OracleSim(topo, params, replica=r) for r in range(R)]
    ref_obs = [o.step(-1) for o in orcs]
    obs, mask, node = eng.step(None)
    rng = np.random.default_rng(0)
    deg = topo.degrees
    for s in range(400):
        g, m, nd = obs.cpu().numpy(), mask.cpu().numpy(), node.cpu().numpy()
        acts = np.zeros(R, dtype=np.int32)
        for r in range(R):
            assert (ref_obs[r] is None) == (m[r] == 0), (s, r)
            if ref_obs[r] is None:
                continue
            assert np.array_equal(ref_obs[r], g[r]), (s, r, g[r], ref_obs[r])
            assert nd[r] == int(orcs[r].records()[-1]["node"])
            acts[r] = rng.integers(0, deg[nd[r]] + (1 if rng.random() < 0.02 else 0))
        ref_obs = [orcs[r].step(int(acts[r])) for r in range(R)]
        obs, mask, node = eng.step(torch.from_numpy(acts).cuda())
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in range(R):
        ref = orcs[r].records()
        assert eng.records(r, 0, len(ref), log_host=log).tobytes() == ref.tobytes()
        assert_counters_equal(cnt[r], orcs[r].counters(), r)
    eng.close()


def test_external_notify_train_parity(oracle_mod):
    """notify_dest + train: destination and small-signalling notifications reach the caller."""
    topo = Topology.example("abilene", 0, 1.5)
    params = engine_params(topo, sim_time_s=3.0, ping_as_obs=1, notify_dest=1, train=1)
    R = 4
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    orcs = [oracle_mod.OracleSim(topo, params, replica=r) for r in range(R)]
    ref_obs = [o.step(-1) for o in orcs]
    obs, mask, node = eng.step(None)
    rng = np.random.default_rng(5)
    n_ctrl = 0
    for s in range(1500):
        g, m, nd = obs.cpu().numpy(), mask.cpu().numpy(), node.cpu().numpy()
        acts = np.zeros(R, dtype=np.int32)
        for r in range(R):
            assert (ref_obs[r] is None) == (m[r] == 0), (s, r)
            if ref_obs[r] is None:
                continue
            assert np.array_equal(ref_obs[r], g[r]), (s, r, g[r], ref_obs[r])
            assert nd[r] == orcs[r].pending_node()
            n_ctrl += int(g[r][0] == 1000)
            acts[r] = rng.integers(0, topo.degrees[nd[r]])
        ref_obs = [orcs[r].step(int(acts[r])) if ref_obs[r] is not None else None for r in range(R)]
        obs, mask, node = eng.step(torch.from_numpy(acts).cuda())
    torch.cuda.synchronize()
    assert n_ctrl > 0
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in range(R):
        ref = orcs[r].records()
        assert eng.records(r, 0, len(ref), log_host=log).tobytes() == ref.tobytes()
        assert_counters_equal(cnt[r], orcs[r].counters(), r)
    eng.close()


def test_episode_end_and_auto_reset(oracle_mod):
    topo = Topology.example("abilene")
    base = engine_params(topo, sim_time_s=2.0, ping_as_obs=1)
    # without auto-reset the episode ends exactly where the oracle's does
    eng = PrismaEngine(topo, base, 3)
    eng.reset(0)
    eng.run(torch.from_numpy(sp_next_hop_table(topo)).cuda(), 10 ** 6)
    cnt = eng.counters()
    for r in range(3):
        o = oracle_mod.OracleSim(topo, base, replica=r)
        o.run_table(sp_next_hop_table(topo), 10 ** 9)
        assert cnt[r]["episode_over"] == 1
        assert_counters_equal(cnt[r], o.counters(), r)
    eng.close()
    # with auto-reset, a replica whose episode ends inside a launch continues into the next
    # episode in the same launch (from its prebuilt spare image); a second end in the same launch
    # stops it and the reset kernel after the launch starts the one after: every record and the
    # counters after every launch equal an oracle chain of episodes 0, 1, 2, ...
    for hops in (3000, 10000):                  # one episode end per launch / two in a launch
        params = dict(base, auto_reset=1, log_capacity=65536)
        eng = PrismaEngine(topo, params, 2)
        eng.reset(0)
        out = compare_steady(oracle_mod, eng, topo, params, ("table", sp_next_hop_table(topo)), t_target_s=9.0,
                             hops_per_launch=hops, min_episode=3, label=f"abilene 2-s episodes, {hops} hops/launch")
        eng.close()
        assert min(out["episodes"]) >= 3


def test_log_ring_wraps(oracle_mod):
    topo = Topology.example("abilene")
    params = engine_params(topo, sim_time_s=30.0, ping_as_obs=0, log_capacity=1024)
    run_table_both(oracle_mod, topo, params, 3, 6000, sp_next_hop_table(topo))


def test_small_topologies_and_single_replica(oracle_mod):
    adj = np.array([[0, 1], [1, 0]])
    tm = np.array([[0, 900000], [300000, 0]], dtype=object)
    topo = Topology.from_matrices(adj, tm)
    params = engine_params(topo, sim_time_s=5.0, ping_as_obs=1)
    run_table_both(oracle_mod, topo, params, 1, 3000, sp_next_hop_table(topo))
    ring = np.zeros((6, 6), dtype=int)
    for i in range(6):
        ring[i, (i + 1) % 6] = ring[(i + 1) % 6, i] = 1
    tm = np.full((6, 6), 40000, dtype=object)
    np.fill_diagonal(tm, 0)
    topo = Topology.from_matrices(ring, tm)
    run_table_both(oracle_mod, topo, engine_params(topo, sim_time_s=5.0, ping_as_obs=0), 2, 3000,
                   sp_next_hop_table(topo))


def test_full_size_properties(oracle_mod):
    """BASELINE size (4096 Abilene replicas): invariants everywhere, 8 replicas checked exactly."""
    topo = Topology.example("abilene")
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1)
    R, H = 4096, 1500
    rng = np.random.default_rng(3)
    picks = sorted(rng.choice(R, 8, replace=False).tolist())
    cnt = run_table_both(oracle_mod, topo, params, R, H, sp_next_hop_table(topo), replicas=picks)
    assert np.all(cnt["error"] == 0)
    assert np.all(cnt["hops"] == H)
    assert np.all(cnt["ov_injected"] >= cnt["ov_arrived"] + cnt["ov_lost"])
    assert np.all(cnt["cost_n"] == cnt["ov_arrived"] + cnt["ov_lost"])
    assert np.all(cnt["bytes_data"] == 540 * cnt["ov_injected"])
    assert len(np.unique(cnt["now_ns"])) > R // 2          # replicas are independent streams


def test_vec_env_transitions_match_oracle_join(oracle_mod):
    from prisma_amd.env import VecRoutingEnv
    from prisma_amd.policies import SPPolicy
    R = 8
    env = VecRoutingEnv("abilene", n_replicas=R, sim_time_s=10.0, ping_as_obs=1)
    pol = SPPolicy(env.topo)
    obs, info = env.reset()
    got = {k: [] for k in ("obs", "action", "reward", "next_obs", "done", "replica")}
    for _ in range(300):
        a = pol.act(obs, info["node"].clamp_min(0))
        obs, _, _, info = env.step(a)
        tr = info["transitions"]
        for k in got:
            got[k].append(tr[k].cpu().numpy())
    got = {k: np.concatenate(v) for k, v in got.items()}
    log = env.engine.log_tensor().cpu().numpy()
    cnt = env.counters()
    for r in range(R):
        recs = env.engine.records(r, 0, int(cnt[r]["dec_count"]), log_host=log)
        # drop the trailing pending decision, as transitions() does
        if recs["status"][-1] == ST_PENDING:
            recs = recs[:-1]
        ref = transitions(recs, env.loss_penalty)
        sel = got["replica"] == r
        key = lambda o, a, rw, no, d: sorted(zip(map(tuple, o.tolist()), a.tolist(), rw.tolist(),
                                                 map(tuple, no.tolist()), d.tolist()))
        assert key(got["obs"][sel].astype(np.uint32), got["action"][sel], got["reward"][sel],
                   got["next_obs"][sel].astype(np.uint32), got["done"][sel]) == \
            key(ref["obs"], ref["action"], ref["reward"], ref["next_obs"], ref["done"])
    env.close()


@pytest.mark.parametrize("notify", [0, 1])
def test_vec_env_gym_step_matches_oracle(oracle_mod, notify):
    """VecRoutingEnv.step -> (obs, reward, done, info) per replica, as Ns3Env.step hands them to
    a node's agent (ns3env.py:417-420): obs, the hop reward forwarder.py:360 computes for the
    notified packet, done = getGameOver; checked against the oracle stepped with the same actions."""
    from prisma_amd.env import VecRoutingEnv
    R = 4
    env = VecRoutingEnv("abilene", 0, 1.5, n_replicas=R, sim_time_s=3.0, ping_as_obs=1,
                        notify_dest=notify, train=notify)
    orcs = [oracle_mod.OracleSim(env.topo, env.params, replica=r) for r in range(R)]
    ref_obs = [o.step(-1) for o in orcs]
    obs, info = env.reset()
    rng = np.random.default_rng(7)
    n_done = n_rew = n_ctrl = n_tr = 0
    reward = done = None
    for s in range(1200):
        g, m, nd = obs.cpu().numpy(), info["mask"].cpu().numpy(), info["node"].cpu().numpy()
        acts = np.zeros(R, dtype=np.int32)
        for r in range(R):
            assert (ref_obs[r] is None) == (m[r] == 0), (s, r)
            if ref_obs[r] is None:
                continue
            assert np.array_equal(ref_obs[r], g[r]), (s, r)
            if reward is not None:
                if g[r][0] == 1000:
                    n_ctrl += 1
                    assert bool(info["control"][r]) and reward[r] == 0.0 and not done[r]
                else:
                    rec = orcs[r].records()[-1]
                    want_rw = float(rec["reward"]) if int(rec["prev"]) >= 0 else 0.0
                    assert float(reward[r]) == want_rw, (s, r)
                    assert bool(done[r]) == (int(rec["status"]) == ST_DESTINATION), (s, r)
                    assert int(info["uid"][r]) == int(rec["uid"])
                    n_done += int(done[r])
                    n_rew += int(int(rec["prev"]) >= 0)
            acts[r] = rng.integers(0, env.topo.degrees[nd[r]])
        ref_obs = [orcs[r].step(int(acts[r])) if ref_obs[r] is not None else None for r in range(R)]
        obs, reward, done, info = env.step(torch.from_numpy(acts).cuda())
        reward, done = reward.cpu().numpy(), done.cpu().numpy()
        n_tr += int(info["transitions"]["reward"].numel())
    assert n_rew > 500 and n_tr > 500
    assert (n_done > 0 and n_ctrl > 0) if notify else (n_done == 0 and n_ctrl == 0)
    env.close()


@pytest.mark.parametrize("name", ["geant", "er256"])
def test_dqn_buffer_weights_change_between_launches(oracle_mod, name):
    """prisma_run re-interleaves the caller's weights on every DQN-buffer launch (training
    updates them in place): launches with weights A, then B written into the same tensor,
    decide like the oracle run with A then B."""
    from prisma_amd.policies import StackedQNet
    topo = Topology.example(name)
    wa = StackedQNet(topo, "buffer", seed=5).pack()
    wb = StackedQNet(topo, "buffer", seed=6).pack()
    params = engine_params(topo, sim_time_s=10.0, ping_as_obs=1, replica_base=1,
                           log_capacity=65536 if topo.n_links > 256 else 8192)
    R, H = 2, 600
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    w = wa.clone()
    eng.run(w, H)
    w.copy_(wb)                              # same pointer, new contents
    eng.run(w, H)
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in range(R):
        o = oracle_mod.OracleSim(topo, params, replica=1 + r)
        o.run_mlp(wa.cpu().numpy(), H)
        o.run_mlp(wb.cpu().numpy(), H)
        ref = o.records()
        assert cnt[r]["error"] == 0
        assert int(cnt[r]["dec_count"]) == len(ref)
        assert eng.records(r, 0, len(ref), log_host=log).tobytes() == ref.tobytes(), r
    eng.close()


@pytest.mark.parametrize("name,ping,train", [("abilene", 1, 0), ("abilene", 0, 1), ("geant", 1, 0)])
def test_dqn_buffer_in_kernel_parity(oracle_mod, name, ping, train):
    """PRISMA_POLICY_DQN_BUFFER: the in-kernel DQN_buffer_model decides exactly like the
    oracle's fixed-order restatement (and hence like torch up to near-ties)."""
    from prisma_amd.policies import StackedQNet
    topo = Topology.example(name)
    net = StackedQNet(topo, "buffer", seed=21)
    w = net.pack()
    params = engine_params(topo, sim_time_s=10.0, ping_as_obs=ping, train=train, replica_base=3)
    R, H = 4, 2000
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    eng.run(w, H // 2)
    eng.run(w, H // 2)                       # a pending decision carried across launches
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    wh = w.cpu().numpy()
    for r in range(R):
        o = oracle_mod.OracleSim(topo, params, replica=3 + r)
        o.run_mlp(wh, H)
        ref = o.records()
        assert cnt[r]["error"] == 0
        assert int(cnt[r]["dec_count"]) == len(ref)
        assert eng.records(r, 0, len(ref), log_host=log).tobytes() == ref.tobytes(), r
        assert_counters_equal(cnt[r], o.counters(), r)
    # the decisions are torch's fp32 argmin on the logged observations, except at genuine near-ties
    net_cpu = StackedQNet(topo, "buffer", seed=21, device="cpu")
    for r in range(R):
        recs = eng.records(r, 0, int(cnt[r]["dec_count"]), log_host=log)
        n, dis, dq, gap = check_near_ties(net_cpu, wh, o, recs)
        assert n > 500
    eng.close()


# ---- tunnelled overlays ----------------------------------------------
def _random_table(topo, seed):
    rng = np.random.default_rng(seed)
    table = np.zeros((topo.n_nodes, topo.n_nodes), dtype=np.uint8)
    for u in topo.overlay_nodes:
        table[u] = rng.integers(0, topo.degrees[u], topo.n_nodes)
    return table


def _ttl_chain():
    """Underlay path 0-1-2-3-4-5, overlay triangle {0, 3, 5}: tunnel 0<->3 has two
    intermediate hops and 0->5 crosses overlay node 3 (a ping bystander).  With the
    bouncing table below a packet for 5 loops 0 <-> 3 until its TTL (255, -2 per loop
    hop) expires at an intermediate forward."""
    adj = np.zeros((6, 6), dtype=int)
    for i in range(5):
        adj[i, i + 1] = adj[i + 1, i] = 1
    tm = np.zeros((6, 6), dtype=object)
    tm[0, 5] = "40Kbps"
    tm[5, 0] = "20Kbps"
    tm[3, 0] = "10Kbps"
    topo = Topology.from_matrices(adj, tm, map_overlay=[0, -1, -1, 1, -1, 2],
                                  overlay_adjacency=np.ones((3, 3)) - np.eye(3))
    table = np.zeros((6, 6), dtype=np.uint8)
    table[0, 5] = 0          # 0 -> 3
    table[3, 5] = 0          # 3 -> 0
    table[5, 0] = 1          # 5 -> 3
    table[3, 0] = 1          # 3 -> 5
    return topo, table


@pytest.mark.parametrize("name,tm,lf,ping,seed,train,pol", [
    ("overlay_full_mesh_3n_abilene", 0, 1.0, 1, 100, 0, "sp"),
    ("overlay_full_mesh_3n_abilene", 0, 20.0, 0, 7, 0, "rand"),
    ("overlay_full_mesh_3n_abilene", 0, 20.0, 1, 9, 1, "rand"),
    ("abilene_on_geant", 0, 1.0, 1, 100, 0, "sp"),
    ("abilene_on_geant", 1, 3.0, 0, 5, 1, "rand"),
    ("abilene_on_geant", 2, 2.0, 1, 8, 0, "rand"),
])
def test_tunnel_table_parity(oracle_mod, name, tm, lf, ping, seed, train, pol):
    topo = Topology.example(name, tm, lf)
    params = engine_params(topo, sim_time_s=20.0, ping_as_obs=ping, seed=seed, replica_base=2, train=train)
    table = sp_next_hop_table(topo) if pol == "sp" else _random_table(topo, seed)
    cnt = run_table_both(oracle_mod, topo, params, 4, 4000, table)
    if name == "overlay_full_mesh_3n_abilene" and lf > 1:
        assert cnt["ov_lost"].sum() > 0                   # intermediate and first-link drops


def test_tunnel_ttl_expiry_parity(oracle_mod):
    topo, table = _ttl_chain()
    params = engine_params(topo, sim_time_s=30.0, ping_as_obs=1)
    o = oracle_mod.OracleSim(topo, params)
    o.run_table(table, 10 ** 9)
    recs = o.records()
    assert recs["ttl"].min() <= 2                          # packets reach the end of their TTL
    c = o.counters()
    assert c["ov_injected"] > c["ov_arrived"] + c["ov_lost"]   # silently expired (never counted)
    run_table_both(oracle_mod, topo, params, 3, 10 ** 6, table)


@pytest.mark.parametrize("log_bits,relay_ip", [(17, 1), (18, 0), (19, 0)])
def test_tunnel_log_capacity_kernel_pick(log_bits, relay_ip):
    """The library's own report of the instance prisma_create picked (prisma_kernel_info): the
    relay-entry kernels keep 18 bits of the decision index (engine_layout.h rip_make), so their
    log-wrap check holds only for logs below 2^18; a log of 2^18 or more takes the 22-bit kernels."""
    topo = Topology.example("overlay_full_mesh_3n_abilene", 0, 20.0)
    params = engine_params(topo, sim_time_s=10.0, ping_as_obs=0, seed=7, log_capacity=1 << log_bits)
    eng = PrismaEngine(topo, params, 1)
    ki = eng.kernel_info()
    eng.close()
    assert ki["tunnels"] == 1 and ki["relay_ip"] == relay_ip and ki["ctrl"] == 1 - relay_ip
    assert ki["relay_dec_bits"] == (18 if relay_ip else 22)
    assert (1 << log_bits) < (1 << ki["relay_dec_bits"])       # every log age is representable
    assert eng.kernel_name.endswith("true, false>" if relay_ip else "true, true>")


def test_tunnel_big_log_parity(oracle_mod):
    """A log of 2^19 decisions on a tunnelled overlay (the 22-bit relay-entry kernels) run past
    2^18 decisions: 300 000 hops on one replica of the 3-node mesh at load factor 20 in a 150-s
    episode, every record in the log compared, so relay entries carry decision indices above 2^18."""
    topo = Topology.example("overlay_full_mesh_3n_abilene", 0, 20.0)
    params = engine_params(topo, sim_time_s=150.0, ping_as_obs=0, seed=7, log_capacity=1 << 19)
    cnt = run_table_both(oracle_mod, topo, params, 1, 300000, _random_table(topo, 7))
    assert int(cnt["dec_count"][0]) > (1 << 18)
    assert cnt["ov_lost"].sum() > 0


def test_tunnel_external_parity(oracle_mod):
    """External actions on a tunnelled overlay without the --train / notify_dest paths: each
    launch opens with the pending decision (finish_pending), whose relay entry takes the TTL from
    the decision's record."""
    topo = Topology.example("overlay_full_mesh_3n_abilene", 0, 10.0)
    params = engine_params(topo, sim_time_s=4.0, ping_as_obs=1)
    R = 3
    eng = PrismaEngine(topo, params, R)
    assert eng.kernel_name.endswith("true, false>")           # TUN, no CTRL: relay entries with the target
    eng.reset(0)
    orcs = [oracle_mod.OracleSim(topo, params, replica=r) for r in range(R)]
    ref_obs = [o.step(-1) for o in orcs]
    obs, mask, node = eng.step(None)
    rng = np.random.default_rng(3)
    for s in range(800):
        g, m, nd = obs.cpu().numpy(), mask.cpu().numpy(), node.cpu().numpy()
        acts = np.zeros(R, dtype=np.int32)
        for r in range(R):
            assert (ref_obs[r] is None) == (m[r] == 0), (s, r)
            if ref_obs[r] is None:
                continue
            assert np.array_equal(ref_obs[r], g[r]), (s, r, g[r], ref_obs[r])
            acts[r] = rng.integers(0, topo.degrees[nd[r]])
        ref_obs = [orcs[r].step(int(acts[r])) if ref_obs[r] is not None else None for r in range(R)]
        obs, mask, node = eng.step(torch.from_numpy(acts).cuda())
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in range(R):
        ref = orcs[r].records()
        assert eng.records(r, 0, len(ref), log_host=log).tobytes() == ref.tobytes()
        assert_counters_equal(cnt[r], orcs[r].counters(), r)
    eng.close()


def test_tunnel_external_notify_train_parity(oracle_mod):
    topo = Topology.example("overlay_full_mesh_3n_abilene", 0, 10.0)
    params = engine_params(topo, sim_time_s=4.0, ping_as_obs=1, notify_dest=1, train=1)
    R = 3
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    orcs = [oracle_mod.OracleSim(topo, params, replica=r) for r in range(R)]
    ref_obs = [o.step(-1) for o in orcs]
    obs, mask, node = eng.step(None)
    rng = np.random.default_rng(2)
    for s in range(1200):
        g, m, nd = obs.cpu().numpy(), mask.cpu().numpy(), node.cpu().numpy()
        acts = np.zeros(R, dtype=np.int32)
        for r in range(R):
            assert (ref_obs[r] is None) == (m[r] == 0), (s, r)
            if ref_obs[r] is None:
                continue
            assert np.array_equal(ref_obs[r], g[r]), (s, r, g[r], ref_obs[r])
            assert nd[r] == orcs[r].pending_node()
            acts[r] = rng.integers(0, topo.degrees[nd[r]])
        ref_obs = [orcs[r].step(int(acts[r])) if ref_obs[r] is not None else None for r in range(R)]
        obs, mask, node = eng.step(torch.from_numpy(acts).cuda())
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in range(R):
        ref = orcs[r].records()
        assert eng.records(r, 0, len(ref), log_host=log).tobytes() == ref.tobytes()
        assert_counters_equal(cnt[r], orcs[r].counters(), r)
    eng.close()


def test_tunnel_dqn_buffer_parity(oracle_mod):
    from prisma_amd.policies import StackedQNet
    topo = Topology.example("abilene_on_geant", 0, 1.0)
    net = StackedQNet(topo, "buffer", seed=4)
    w = net.pack()
    params = engine_params(topo, sim_time_s=10.0, ping_as_obs=1)
    R, H = 3, 1500
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    eng.run(w, H)
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    wh = w.cpu().numpy()
    for r in range(R):
        o = oracle_mod.OracleSim(topo, params, replica=r)
        o.run_mlp(wh, H)
        ref = o.records()
        assert cnt[r]["error"] == 0
        got = eng.records(r, 0, len(ref), log_host=log)
        assert got.tobytes() == ref.tobytes(), r
        assert_counters_equal(cnt[r], o.counters(), r)
        check_near_ties(StackedQNet(topo, "buffer", seed=4, device="cpu"), wh, o, got)
    eng.close()


def test_tunnel_full_size_properties(oracle_mod):
    """Config 3 size (4096 Abilene-on-GEANT replicas, SP): invariants on every replica,
    4 random replicas compared record by record."""
    topo = Topology.example("abilene_on_geant")
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1)
    R, H = 4096, 600
    rng = np.random.default_rng(4)
    picks = sorted(rng.choice(R, 4, replace=False).tolist())
    cnt = run_table_both(oracle_mod, topo, params, R, H, sp_next_hop_table(topo), replicas=picks)
    assert np.all(cnt["error"] == 0)
    assert np.all(cnt["hops"] == H)
    assert np.all(cnt["ov_injected"] >= cnt["ov_arrived"] + cnt["ov_lost"])
    assert np.all(cnt["bytes_data"] == 540 * cnt["ov_injected"])
    assert len(np.unique(cnt["now_ns"])) > R // 2
