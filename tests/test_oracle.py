"""The CPU oracle (test infrastructure) pinned against published known answers,
analytic results of the reference's link model and the golden fixtures."""
import json
import math
import os

import numpy as np
import pytest

from prisma_amd.config import engine_params
from prisma_amd.records import (ST_DESTINATION, ST_DROPPED, ST_ENQUEUED, transitions)
from prisma_amd.topology import Topology, sp_next_hop_table, sp_paths

GOLD = os.path.join(os.path.dirname(__file__), "golden")
EV_PING, EV_START, EV_SEND, EV_COMPLETE, EV_RECEIVE = range(5)


def test_philox_known_answers(oracle_mod):
    with open(os.path.join(GOLD, "philox_kat.json")) as fh:
        for v in json.load(fh):
            assert oracle_mod.philox(v["ctr"], v["key"]) == v["out"]


def test_det_log_accuracy(oracle_mod):
    L = oracle_mod.lib()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.random(20000), [1.0, 0.5, 2.0 ** -53, 1 - 2 ** -53, 0.7071067811865476]])
    for x in xs:
        if x <= 0:
            continue
        got = L.or_det_log(float(x))
        ref = math.log(x)
        assert abs(got - ref) <= 4e-16 * max(1.0, abs(ref)), (x, got, ref)


def test_time_conversions(oracle_mod):
    L = oracle_mod.lib()
    assert L.or_seconds_to_ns(float(np.float32(0.2))) == 200000003     # Seconds(0.2f), SURVEY A.4
    assert L.or_seconds_to_ns(542 * 8 / 500000) == 8672000               # 542 B at 500 kb/s
    assert L.or_seconds_to_ns(38 * 8 / 500000) == 608000
    for deg, ns in zip(range(1, 7), [9, 4, 3, 2, 2, 1]):                 # access link, SURVEY A.15
        assert L.or_seconds_to_ns(542 * 8 / (1e6 * 500000 * deg)) == ns


def test_python_microsecond_formatting(oracle_mod):
    # the Forwarder reads times back from std::to_string(double) == "%f"
    L = oracle_mod.lib()
    rng = np.random.default_rng(7)
    ts = list(rng.integers(0, 2 * 10 ** 12, 20000)) + [int(x) * 1000 + 500 for x in rng.integers(0, 2 * 10 ** 9, 20000)]
    ts += [500, 1500, 2500, 999999500, 1000000500, 62131136]
    for t in ts:
        t = int(t)
        us = int(("%f" % (t / 1e9)).replace(".", ""))
        assert L.or_py_micros(t) == us, t


def line_topo(rate_bps, n=3):
    adj = np.zeros((n, n), dtype=int)
    for i in range(n - 1):
        adj[i, i + 1] = adj[i + 1, i] = 1
    tm = np.zeros((n, n), dtype=np.int64)
    tm[0, n - 1] = rate_bps
    return Topology.from_matrices(adj, tm.astype(object))


def py_reward(t1, t0):
    return float("%f" % (t1 / 1e9)) - float("%f" % (t0 / 1e9))


def test_unloaded_path_delay(oracle_mod):
    """An idle 3-node line: each hop = 8.672 ms tx + 1 ms propagation."""
    topo = line_topo(2000)
    p = engine_params(topo, sim_time_s=20.0, ping_interval_s=1000.0, ping_as_obs=0)
    s = oracle_mod.OracleSim(topo, p)
    s.enable_trace(True)
    s.run_table(sp_next_hop_table(topo), 10 ** 6)
    recs = s.records()
    tr = s.trace()
    sends = tr[tr[:, 2] == EV_SEND][:, 0]
    first = recs[recs["prev"] == -1]
    assert len(first) == len(sends) or len(first) == len(sends) - 1
    assert np.array_equal(first["t_ns"] - sends[:len(first)], np.full(len(first), 9))   # access link, deg 1
    by_idx = {i: r for i, r in enumerate(recs)}
    for i, r in enumerate(recs):
        if r["prev"] >= 0:
            q = by_idx[int(r["prev"])]
            assert r["t_ns"] - q["t_ns"] == 9672000
            assert r["reward"] == py_reward(int(r["t_ns"]), int(q["t_ns"]))
    dest = recs[recs["status"] == ST_DESTINATION]
    assert len(dest) > 10 and np.all(dest["node"] == 2)
    c = s.counters()
    assert c["ov_lost"] == 0 and c["ov_arrived"] == len(dest)


def test_fifo_byte_limit_and_drops(oracle_mod):
    """Overloaded link: DropTail at 16260 B = 30 data packets."""
    topo = line_topo(2_000_000, n=2)                 # 2 Mb/s offered on a 500 kb/s link
    p = engine_params(topo, sim_time_s=5.0, ping_interval_s=1000.0, ping_as_obs=0)
    s = oracle_mod.OracleSim(topo, p)
    s.run_table(sp_next_hop_table(topo), 10 ** 6)
    recs = s.records()
    at0 = recs[recs["node"] == 0]
    q = at0["obs"][:, 1]
    assert np.all(q % 542 == 0) and q.max() == 16260
    assert np.all(q[at0["status"] == ST_DROPPED] == 16260)
    assert np.all(q[at0["status"] == ST_ENQUEUED] <= 16260 - 542)
    c = s.counters()
    assert c["ov_lost"] == (at0["status"] == ST_DROPPED).sum() > 0
    assert c["cost_n"] == c["ov_lost"] + c["ov_arrived"]


def test_ping_rounds_period(oracle_mod):
    topo = Topology.example("abilene")
    p = engine_params(topo, sim_time_s=1.0, ping_as_obs=1)
    s = oracle_mod.OracleSim(topo, p)
    s.enable_trace(True)
    s.run_table(sp_next_hop_table(topo), 10 ** 6)
    tr = s.trace()
    pings = tr[tr[:, 2] == EV_PING]
    assert np.array_equal(np.unique(pings[:, 0]), np.arange(1, 5) * 200000003)
    for t in np.unique(pings[:, 0]):
        assert list(pings[pings[:, 0] == t][:, 3]) == list(range(11))     # node order
    keys = [(int(a), int(b)) for a, b in tr[:, :2]]
    assert keys == sorted(keys) and len(set(keys)) == len(keys)           # (time, uid) order


@pytest.mark.parametrize("ping_as_obs", [0, 1])
def test_abilene_sp_invariants(oracle_mod, ping_as_obs):
    topo = Topology.example("abilene")
    p = engine_params(topo, sim_time_s=20.0, ping_as_obs=ping_as_obs)
    s = oracle_mod.OracleSim(topo, p, replica=3)
    s.run_table(sp_next_hop_table(topo), 10 ** 9)
    recs = s.records()
    c = s.counters()
    st = recs["status"]
    assert c["decisions"] == len(recs) == c["dec_count"]
    assert c["hops"] == ((st == ST_ENQUEUED) | (st == ST_DROPPED)).sum()
    assert c["ov_lost"] == (st == ST_DROPPED).sum()
    assert c["ov_arrived"] == (st == ST_DESTINATION).sum()
    assert c["ov_injected"] >= c["ov_arrived"] + c["ov_lost"]
    assert c["cost_n"] == c["ov_arrived"] + c["ov_lost"]
    assert c["bytes_data"] == 540 * c["ov_injected"]
    assert c["ov_lost"] > 0                                        # lf=1 overloads SP links
    if ping_as_obs:
        assert recs["obs"][:, 1:].max() <= 2600
    # SP routing follows the networkx paths; e2e = sum of hop rewards (A.5)
    paths = sp_paths(topo)
    idx = {i: r for i, r in enumerate(recs)}
    for i in np.nonzero(st == ST_DESTINATION)[0][:500]:
        chain = [idx[int(i)]]
        while chain[-1]["prev"] >= 0:
            chain.append(idx[int(chain[-1]["prev"])])
        nodes = [int(r["node"]) for r in reversed(chain)]
        assert nodes == paths[(nodes[0], nodes[-1])]
        e2e = sum(float(r["reward"]) for r in chain)
        assert abs(e2e - (chain[0]["t_ns"] - chain[-1]["t_ns"]) * 1e-9) <= 1e-6 * len(chain)
    tr = transitions(recs, p["loss_penalty"])
    assert (tr["reward"] == p["loss_penalty"]).sum() == c["ov_lost"]
    assert len(tr["reward"]) == c["hops"] - ((st == ST_ENQUEUED).sum() - (recs["prev"] >= 0).sum())


def test_external_step_matches_table(oracle_mod):
    topo = Topology.example("abilene")
    p = engine_params(topo, sim_time_s=5.0, ping_as_obs=1)
    table = sp_next_hop_table(topo)
    a = oracle_mod.OracleSim(topo, p, replica=1)
    a.run_table(table, 10 ** 9)
    b = oracle_mod.OracleSim(topo, p, replica=1)
    obs = b.step(-1)
    while obs is not None:
        node = int(b.records()[-1]["node"])
        obs = b.step(int(table[node, obs[0]]))
    assert a.records().tobytes() == b.records().tobytes()


def test_invalid_action_discards(oracle_mod):
    topo = Topology.example("abilene")
    p = engine_params(topo, sim_time_s=3.0, ping_as_obs=0)
    s = oracle_mod.OracleSim(topo, p)
    obs = s.step(-1)
    n = 0
    while obs is not None and n < 200:
        obs = s.step(7)                              # >= degree: sendPacket's silent else-branch
        n += 1
    recs = s.records()
    assert np.all(recs["status"][:-1][recs["prev"][:-1] == -1] == 4)
    c = s.counters()
    assert c["hops"] == 0 and c["ov_lost"] == 0


def test_info_string_contract(oracle_mod):
    """22 comma tokens parsed by forwarder.treat_info."""
    topo = Topology.example("abilene")
    p = engine_params(topo, sim_time_s=5.0, ping_as_obs=1)
    s = oracle_mod.OracleSim(topo, p)
    obs = s.step(-1)
    for _ in range(300):
        node = int(s.records()[-1]["node"])
        obs = s.step(int(sp_next_hop_table(topo)[node, obs[0]]))
    info = s.last_info()
    tokens = info.split(",")
    assert len(tokens) == 22
    vals = [t.split("=")[-1] for t in tokens]
    rec = s.records()[-1]
    assert float(vals[2]) == float("%f" % (rec["t_ns"] / 1e9))
    assert int(vals[3]) == rec["uid"] and int(vals[4]) == 0
    assert int(vals[20]) == rec["dst"] and int(vals[21]) == rec["node"]
    assert int(vals[1]) == 542
    for v in vals[5:18]:
        float(v)


def test_train_echo_known_answer(oracle_mod):
    """--train: a data notification at a non-source node echoes a 30-B
    small-signalling packet to the last hop; it arrives tx(30 B) + 1 ms later as a
    control notification [1000] with a 20-token info string."""
    adj = np.array([[0, 1], [1, 0]])
    tm = np.array([[0, 2000], [0, 0]], dtype=object)         # one slow flow 0 -> 1
    topo = Topology.from_matrices(adj, tm)
    p = engine_params(topo, sim_time_s=3.0, ping_as_obs=0, train=1, notify_dest=1)
    s = oracle_mod.OracleSim(topo, p)
    obs = s.step(-1)
    events = []
    while obs is not None and len(events) < 40:
        info = s.last_info()
        t = float(info.split(",")[2].split("=")[-1])
        events.append((int(obs[0]), t, info))
        obs = s.step(0)
    data0 = [e for e in events if e[0] == 1 and "node=0" in e[2]]           # decisions at the source
    dest1 = [e for e in events if e[0] == 1 and "node=1" in e[2]]           # done at the destination
    ctrl = [e for e in events if e[0] == 1000]
    assert data0 and dest1 and len(ctrl) == len(dest1)
    # echo leaves node 1 at the destination notification and reaches node 0 after 0.48 + 1 ms
    for (_, t1, i1), (_, tc, ic) in zip(dest1, ctrl):
        assert abs((tc - t1) - 0.00148) < 2e-6
        tok = ic.split(",")
        assert len(tok) == 20 and int(tok[4].split("=")[-1]) == 2 and int(tok[1].split("=")[-1]) == 30
        assert tok[18].split("=")[-1] == i1.split(",")[3].split("=")[-1]     # PacketIdSignaled = data uid
        assert tok[19].split("=")[-1] == "1"
    # no echo for the source's own notification, and train=0 sends none
    q = oracle_mod.OracleSim(topo, dict(p, train=0))
    obs, n_ctrl = q.step(-1), 0
    while obs is not None:
        n_ctrl += int(obs[0]) == 1000
        obs = q.step(0)
    assert n_ctrl == 0


def test_train_echo_changes_dynamics_and_counts(oracle_mod):
    topo = Topology.example("abilene")
    table = sp_next_hop_table(topo)
    p0 = engine_params(topo, sim_time_s=5.0, ping_as_obs=1)
    a = oracle_mod.OracleSim(topo, p0)
    a.run_table(table, 10 ** 9)
    b = oracle_mod.OracleSim(topo, dict(p0, train=1))
    b.run_table(table, 10 ** 9)
    ca, cb = a.counters(), b.counters()
    rb = b.records()
    relayed = int((rb["prev"] >= 0).sum())                  # notifications at non-source nodes (SP: no loops)
    # every relayed notification echoes 28 signalling bytes unless the echo was dropped
    extra = int(cb["bytes_signaling"]) - int(ca["bytes_signaling"])
    assert extra > 0 and int(cb["seq"]) > int(ca["seq"])
    assert relayed > 0


def test_det_expm1_accuracy(oracle_mod):
    import math
    xs = [0.0, -1e-300, -1e-12, -1e-6, -0.01, -0.3, -0.35, -0.5, -1.0, -2.0, -7.3, -20.0, -59.0, -80.0]
    xs += list(-np.random.default_rng(0).exponential(2.0, 2000))
    for x in xs:
        got, want = oracle_mod.det_expm1(x), math.expm1(x)
        assert abs(got - want) <= 4e-16 * max(1.0, abs(want)) + 1e-300, (x, got, want)


def test_det_expm1f_accuracy(oracle_mod):
    """The MLP's fp32 ELU: within 2 ulp (fp32) of expm1 on (-inf, 0], exact at the edges."""
    import math
    rng = np.random.default_rng(0)
    xs = [0.0, -0.0, -1e-30, -1e-8, -6e-8, -1e-6, -0.01, -0.3465, -0.3466, -0.5, -1.0, -2.0, -7.3, -16.99,
          -17.0, -17.01, -20.0, -80.0]
    xs += list(-rng.exponential(1.0, 20000)) + list(-rng.uniform(0, 1e-3, 2000))
    worst = 0.0
    for x in xs:
        x = float(np.float32(x))
        got, want = oracle_mod.det_expm1f(x), math.expm1(x)
        ulp = float(np.spacing(np.float32(abs(want)))) if want != 0.0 else 1e-45
        worst = max(worst, abs(got - want) / ulp)
        assert abs(got - want) <= 2.0 * ulp, (x, got, want)
    assert oracle_mod.det_expm1f(-100.0) == -1.0 and oracle_mod.det_expm1f(0.0) == 0.0
    assert worst > 0.0


def test_oracle_mlp_matches_torch_dqn_buffer(oracle_mod):
    """The oracle's fixed-order fp32 DQN_buffer_model picks torch's argmin (models.py:258-306)
    except on near-ties (different summation order)."""
    import torch
    from prisma_amd.policies import StackedQNet
    topo = Topology.example("abilene")
    net = StackedQNet(topo, "buffer", seed=3, device="cpu")
    w = net.pack().numpy()
    p = engine_params(topo, sim_time_s=1.0)
    s = oracle_mod.OracleSim(topo, p)
    rng = np.random.default_rng(1)
    B = 3000
    node = rng.integers(0, topo.n_nodes, B)
    obs = np.zeros((B, 1 + topo.max_deg), dtype=np.int64)
    obs[:, 0] = rng.integers(0, topo.n_nodes, B)
    obs[:, 1:] = rng.integers(0, 16260, (B, topo.max_deg))
    ta = net.act(torch.from_numpy(obs).int(), torch.from_numpy(node)).numpy()
    with torch.no_grad():
        q = net.q_values(torch.from_numpy(obs).int(), torch.from_numpy(node)).numpy()
    mism = 0
    for b in range(B):
        a = s.mlp_action(w, int(node[b]), obs[b].astype(np.uint32))
        if a != ta[b]:
            mism += 1
            assert abs(q[b, a] - q[b, ta[b]]) <= 1e-5 * max(1.0, abs(q[b, a])), (b, a, ta[b], q[b])
    assert mism <= B // 100
