"""Memory-resident engine (PRISMA_ENGINE_MEMORY, prisma_engine_mem.hip) vs the CPU oracle,
bit-exact, through the C-ABI: the same scenarios as the register-resident engine's
parity suite (forced onto the memory engine), the two engines against each other, and
BASELINE config 5 (Erdos-Renyi G(256, 8/255): 2 008 links, 65 251 flows, degree 1-19),
which only the memory engine can hold."""
import numpy as np
import pytest
import torch

from prisma_amd.config import engine_params
from prisma_amd.engine import PRISMA_ENGINE_MEMORY, PRISMA_ENGINE_REGISTER, PrismaEngine
from prisma_amd.records import COUNTERS_DTYPE
from prisma_amd.topology import DATA_DIR, Topology, sp_next_hop_table
from parity_util import check_near_ties

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]

CNT_KEYS = [k for k in COUNTERS_DTYPE.names if k not in ("hops_total", "events_total")]
MEM = PRISMA_ENGINE_MEMORY


def assert_counters_equal(g, o, r):
    bad = [(k, g[k], o[k]) for k in CNT_KEYS if g[k] != o[k]]
    assert not bad, f"replica {r}: counters differ {bad}"


def er256():
    topo = Topology.example("er256")
    table = np.load(f"{DATA_DIR}/er256/sp_next_hop_table.npy")
    return topo, table


def run_both(oracle_mod, topo, params, R, H, policy, launches=1, replicas=None, mlp=False, net_cpu=None):
    eng = PrismaEngine(topo, params, R)
    assert eng.engine_kind == MEM
    eng.reset(0)
    pol = policy if mlp else torch.from_numpy(np.ascontiguousarray(policy)).cuda()
    for _ in range(launches):
        eng.run(pol, H // launches)
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in (range(R) if replicas is None else replicas):
        o = oracle_mod.OracleSim(topo, params, replica=params["replica_base"] + r)
        if mlp:
            o.run_mlp(policy.cpu().numpy(), H)
        else:
            o.run_table(policy, H)
        ref = o.records()
        assert cnt[r]["error"] == 0, (r, int(cnt[r]["error"]))
        assert int(cnt[r]["dec_count"]) == len(ref), (r, int(cnt[r]["dec_count"]), len(ref))
        n = min(len(ref), eng.log_capacity)
        got = eng.records(r, len(ref) - n, n, log_host=log)
        assert got.tobytes() == ref[len(ref) - n:].tobytes(), f"replica {r} records differ"
        assert_counters_equal(cnt[r], o.counters(), r)
        if net_cpu is not None:                  # torch fp32 argmin except at genuine near-ties
            check_near_ties(net_cpu, policy.cpu().numpy(), o, got)
    eng.close()
    return cnt


@pytest.mark.parametrize("name,tm,lf,ping,seed,train", [
    ("abilene", 0, 1.0, 1, 100, 0), ("abilene", 3, 2.0, 0, 12345, 0), ("geant", 0, 1.0, 1, 100, 0),
    ("geant", 1, 1.5, 0, 3, 1), ("abilene", 1, 2.0, 1, 9, 1),
])
def test_mem_table_policy_parity(oracle_mod, name, tm, lf, ping, seed, train):
    topo = Topology.example(name, tm, lf)
    params = engine_params(topo, sim_time_s=15.0, ping_as_obs=ping, seed=seed, replica_base=5, train=train,
                           engine=MEM)
    run_both(oracle_mod, topo, params, 6, 2500, sp_next_hop_table(topo))


def test_mem_multi_launch_and_log_wrap(oracle_mod):
    """State written back to HBM between launches changes nothing; the log ring wraps."""
    topo = Topology.example("abilene")
    params = engine_params(topo, sim_time_s=30.0, ping_as_obs=0, log_capacity=1024, engine=MEM)
    run_both(oracle_mod, topo, params, 3, 6000, sp_next_hop_table(topo), launches=12)


def test_mem_equals_register_engine():
    """Both engines produce byte-identical logs and counters (GEANT, 64 replicas)."""
    topo = Topology.example("geant", 0, 1.25)
    table = torch.from_numpy(sp_next_hop_table(topo)).cuda()
    out = []
    for kind in (PRISMA_ENGINE_REGISTER, MEM):
        eng = PrismaEngine(topo, engine_params(topo, sim_time_s=20.0, ping_as_obs=1, engine=kind), 64)
        assert eng.engine_kind == kind
        eng.reset(0)
        eng.run(table, 3000)
        torch.cuda.synchronize()
        out.append((eng.log_tensor().cpu().numpy(), eng.counters()))
        eng.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert out[0][1].tobytes() == out[1][1].tobytes()


def test_mem_external_step_parity(oracle_mod):
    """Gym-style step() on the memory engine: random actions (2% invalid)."""
    topo = Topology.example("abilene", 0, 1.5)
    params = engine_params(topo, sim_time_s=10.0, ping_as_obs=1, notify_dest=1, train=1, engine=MEM)
    R = 6
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    orcs = [oracle_mod.OracleSim(topo, params, replica=r) for r in range(R)]
    ref_obs = [o.step(-1) for o in orcs]
    obs, mask, node = eng.step(None)
    rng = np.random.default_rng(1)
    deg = topo.degrees
    W = eng.W
    for s in range(300):
        g, m, nd = obs.cpu().numpy(), mask.cpu().numpy(), node.cpu().numpy()
        acts = np.zeros(R, dtype=np.int32)
        for r in range(R):
            assert (ref_obs[r] is None) == (m[r] == 0), (s, r)
            if ref_obs[r] is None:
                continue
            ro = np.zeros(W, dtype=np.int64)
            ro[:len(ref_obs[r])] = ref_obs[r]
            assert np.array_equal(ro, g[r]), (s, r, g[r], ref_obs[r])
            assert nd[r] == orcs[r].pending_node()
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


def test_mem_episode_end_and_auto_reset(oracle_mod):
    topo = Topology.example("abilene")
    base = engine_params(topo, sim_time_s=2.0, ping_as_obs=1, engine=MEM)
    table = sp_next_hop_table(topo)
    params = dict(base, auto_reset=1)
    eng = PrismaEngine(topo, params, 2)
    eng.reset(0)
    t = torch.from_numpy(table).cuda()
    eng.run(t, 10 ** 6)
    cnt = eng.counters()
    assert np.all(cnt["episode"] == 1) and np.all(cnt["episode_over"] == 0) and np.all(cnt["hops"] == 0)
    eng.run(t, 1500)
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in range(2):
        o0 = oracle_mod.OracleSim(topo, base, replica=r, episode=0)
        o0.run_table(table, 10 ** 9)
        n0 = len(o0.records())
        o1 = oracle_mod.OracleSim(topo, base, replica=r, episode=1)
        o1.run_table(table, 1500)
        ref1 = o1.records()
        got = eng.records(r, n0, len(ref1), log_host=log).copy()
        got["prev"] = np.where(got["prev"] >= 0, got["prev"] - n0, got["prev"])
        assert got.tobytes() == ref1.tobytes()
    eng.close()


def test_mem_dqn_buffer_parity(oracle_mod):
    from prisma_amd.policies import StackedQNet
    topo = Topology.example("geant")
    w = StackedQNet(topo, "buffer", seed=21).pack()
    params = engine_params(topo, sim_time_s=10.0, ping_as_obs=0, replica_base=3, engine=MEM)
    run_both(oracle_mod, topo, params, 3, 1500, w, launches=2, mlp=True,
             net_cpu=StackedQNet(topo, "buffer", seed=21, device="cpu"))


# ---- BASELINE config 5: ER-256 ---------------------------------------------------------
def test_er256_sp_table_fixture_matches_networkx_rule():
    """The shipped SP table equals the networkx bidirectional-BFS restatement on a sample."""
    from prisma_amd.topology import _bidirectional_path, _overlay_lists
    topo, table = er256()
    lists = _overlay_lists(topo)
    rng = np.random.default_rng(0)
    for s, d in rng.integers(0, 256, (300, 2)):
        if s != d:
            assert lists[s][table[s, d]] == _bidirectional_path(lists, int(s), int(d))[1]


def test_er256_table_parity(oracle_mod):
    topo, table = er256()
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1, seed=100, replica_base=0)
    run_both(oracle_mod, topo, params, 4, 6000, table, launches=3)


def test_er256_train_buffer_obs_parity(oracle_mod):
    topo, table = er256()
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=0, train=1, seed=7, replica_base=100)
    run_both(oracle_mod, topo, params, 2, 5000, table)


def test_er256_dqn_buffer_parity(oracle_mod):
    """Config 5's agent: the in-kernel DQN-buffer MLP over 256-way one-hot inputs and up to
    19 buffer inputs decides exactly like the oracle's restatement."""
    from prisma_amd.policies import StackedQNet
    topo, _ = er256()
    w = StackedQNet(topo, "buffer", seed=5).pack()
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=0, replica_base=1000)
    run_both(oracle_mod, topo, params, 2, 2000, w, launches=2, mlp=True,
             net_cpu=StackedQNet(topo, "buffer", seed=5, device="cpu"))


def test_er256_full_size_properties(oracle_mod):
    """Config 5's per-GPU share (8192 replicas / 8 GPUs = 1024): invariants on every
    replica, 3 replicas compared record by record."""
    topo, table = er256()
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1)
    R, H = 1024, 1000
    cnt = run_both(oracle_mod, topo, params, R, H, table, replicas=[0, 511, 1023])
    assert np.all(cnt["error"] == 0)
    assert np.all(cnt["hops"] == H)
    assert np.all(cnt["ov_injected"] >= cnt["ov_arrived"] + cnt["ov_lost"])
    assert np.all(cnt["bytes_data"] == 540 * cnt["ov_injected"])
    assert len(np.unique(cnt["now_ns"])) > R // 2


# ---- signalling on the memory engine (sim.cc:373-392, 634-647) ------------------------
def _sig(topo, **kw):
    base = dict(sim_time_s=4.0, ping_as_obs=1, train=1, signaling_type="NN", big_signaling=1, replica_base=3,
                big_signaling_bytes=35328, engine=MEM)
    base.update(kw)
    return engine_params(topo, **base)


@pytest.mark.parametrize("name,tm,lf,kw", [
    ("abilene", 0, 1.0, dict()),
    ("abilene", 1, 2.0, dict(sync_step_s=0.1, seed=7)),                 # 10x the segments, drops
    ("abilene", 0, 1.0, dict(ping_as_obs=0, big_signaling_bytes=4096, sync_step_s=0.05)),
    ("abilene", 2, 1.5, dict(signaling_type="target", big_signaling=0)),
    ("geant", 0, 1.0, dict(sync_step_s=0.5)),                           # per-node echo sizes
])
def test_mem_signaling_table_parity(oracle_mod, name, tm, lf, kw):
    """Echo payloads by signalling type and the big-signalling generators on the memory engine
    (forced), bit-exact against the oracle: the register engine's signalling cases."""
    topo = Topology.example(name, tm, lf)
    cnt = run_both(oracle_mod, topo, _sig(topo, **kw), 4, 2500, sp_next_hop_table(topo))
    assert int(cnt["bytes_signaling"].min()) > 0


def test_mem_signaling_equals_register_engine():
    """Big signalling: both engines produce byte-identical logs and counters (GEANT, 32 replicas)."""
    topo = Topology.example("geant", 0, 1.5)
    table = torch.from_numpy(sp_next_hop_table(topo)).cuda()
    out = []
    for kind in (PRISMA_ENGINE_REGISTER, MEM):
        eng = PrismaEngine(topo, _sig(topo, sim_time_s=10.0, sync_step_s=0.25, engine=kind), 32)
        assert eng.engine_kind == kind
        eng.reset(0)
        eng.run(table, 4000)
        torch.cuda.synchronize()
        out.append((eng.log_tensor().cpu().numpy(), eng.counters()))
        eng.close()
    assert int(out[1][1]["ctrl_dropped"].sum()) >= 0 and int(out[1][1]["bytes_signaling"].min()) > 0
    assert np.array_equal(out[0][0], out[1][0])
    assert out[0][1].tobytes() == out[1][1].tobytes()


def test_mem_signaling_external_notify_parity(oracle_mod):
    """notify_dest + train + big signalling on the memory engine: echo and NN-segment
    notifications reach the caller with the obs fields of include/prisma.h."""
    topo = Topology.example("abilene", 0, 1.5)
    params = _sig(topo, sim_time_s=2.0, notify_dest=1, sync_step_s=0.2)
    R = 3
    eng = PrismaEngine(topo, params, R)
    assert eng.engine_kind == MEM
    eng.reset(0)
    orcs = [oracle_mod.OracleSim(topo, params, replica=params["replica_base"] + r) for r in range(R)]
    ref_obs = [o.step(-1) for o in orcs]
    obs, mask, node = eng.step(None)
    rng = np.random.default_rng(19)
    n_big = n_echo = 0
    for s in range(1500):
        g, m, nd = obs.cpu().numpy(), mask.cpu().numpy(), node.cpu().numpy()
        acts = np.zeros(R, dtype=np.int32)
        for r in range(R):
            assert (ref_obs[r] is None) == (m[r] == 0), (s, r)
            if ref_obs[r] is None:
                continue
            assert np.array_equal(ref_obs[r], g[r]), (s, r, g[r], ref_obs[r])
            assert nd[r] == orcs[r].pending_node()
            if g[r][0] == 1000:
                n_big += int(g[r][3] >> 16)
                n_echo += 1 - int(g[r][3] >> 16)
            acts[r] = rng.integers(0, topo.degrees[nd[r]])
        ref_obs = [orcs[r].step(int(acts[r])) if ref_obs[r] is not None else None for r in range(R)]
        obs, mask, node = eng.step(torch.from_numpy(acts).cuda())
    torch.cuda.synchronize()
    assert n_big > 0 and n_echo > 0
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in range(R):
        ref = orcs[r].records()
        assert eng.records(r, 0, len(ref), log_host=log).tobytes() == ref.tobytes()
        assert_counters_equal(cnt[r], orcs[r].counters(), r)
    eng.close()


def test_er256_big_signaling_parity(oracle_mod):
    """Config 5's graph with --train, "NN" echoes and big signalling: 2 006 generators (one per
    flow between neighbours), beyond the register engine's 256, all in one event slot."""
    topo, table = er256()
    params = _sig(topo, sim_time_s=60.0, sync_step_s=0.5, seed=11, replica_base=77, engine=0)
    cnt = run_both(oracle_mod, topo, params, 2, 6000, table, launches=2)
    assert int(cnt["bytes_signaling"].min()) > 0


def test_er256_big_signaling_dqn_buffer_parity(oracle_mod):
    """... and with the in-kernel DQN-buffer agent deciding (the memory engine's MLP + CTRL
    instance)."""
    from prisma_amd.policies import StackedQNet
    topo, _ = er256()
    w = StackedQNet(topo, "buffer", seed=8).pack()
    params = _sig(topo, sim_time_s=60.0, ping_as_obs=1, sync_step_s=0.25, seed=5, replica_base=9, engine=0)
    run_both(oracle_mod, topo, params, 2, 3000, w, launches=2, mlp=True,
             net_cpu=StackedQNet(topo, "buffer", seed=8, device="cpu"))
