"""Per-node Ns3Env compatibility surface (prisma_amd/ns3env.py).

CPU: the info-string renderer + tracker, driven by the oracle in
notify-destination mode, reproduces the oracle's own DataPacketManager::getInfo
string at every notification (packet-manager.cc:119-176).
GPU: PrismaSession (one engine replica) yields the same notification stream
(node, obs, done, info) as the oracle, and per-node Ns3Env views driven by one
thread per node (forwarder.py:291-332) see exactly that stream.
"""
import threading

import numpy as np
import pytest
import torch

from prisma_amd.config import engine_params
from prisma_amd.ns3env import InfoTracker
from prisma_amd.topology import Topology, sp_next_hop_table


def oracle_stream(oracle_mod, topo, params, policy, n):
    """(node, obs, done, info) of the first n notifications of the oracle."""
    o = oracle_mod.OracleSim(topo, params)
    out = []
    last_done = [False] * topo.n_nodes
    obs = o.step(-1)
    while obs is not None and len(out) < n:
        v = o.pending_node()
        if int(obs[0]) == 1000:                                  # small-signalling (control) notification
            out.append((v, [1000], last_done[v], o.last_info()))
        else:
            rec = o.records()[-1]
            W = 1 + int(topo.degrees[v])
            done = int(rec["status"]) == 3
            last_done[v] = done
            out.append((v, [int(x) for x in obs[:W]], done, o.last_info()))
        obs = o.step(policy(v, obs))
    return o, out


def sp_policy(topo):
    """forwarder.py:149,190-191: action 0 at the destination (obs[0] == own overlay index)
    and for control notifications, else the SP next hop on the overlay graph."""
    table = sp_next_hop_table(topo)
    on, ovi = topo.overlay_nodes, topo.overlay_index
    return lambda v, obs: 0 if obs[0] in (ovi[v], 1000) else int(table[v, on[obs[0]]])


def test_info_renderer_matches_oracle(oracle_mod):
    topo = Topology.example("abilene", 0, 2.0)               # load 2.0: drops fill "Packet Lost="
    params = engine_params(topo, sim_time_s=3.0, ping_as_obs=1, notify_dest=1)
    o = oracle_mod.OracleSim(topo, params)
    tr = InfoTracker(topo.n_nodes, 542)
    table = sp_next_hop_table(topo)
    obs = o.step(-1)
    n, lost_seen, dest_seen = 0, 0, 0
    while obs is not None and n < 4000:
        recs = o.records()
        rec = recs[-1]
        tr.notified(rec)
        info = tr.render(rec, o.counters())
        assert info == o.last_info(), (n, info, o.last_info())
        lost_seen += "Packet Lost=," not in info
        v = int(rec["node"])
        dest_seen += int(rec["status"]) == 3
        d = len(recs) - 1
        obs = o.step(0 if obs[0] == v else int(table[v, obs[0]]))
        tr.applied(o.records(d, 1)[0])
        n += 1
    assert lost_seen > 0 and dest_seen > 0


@pytest.mark.parametrize("sig", [dict(), dict(signaling_type="target"),
                                 dict(signaling_type="NN", big_signaling=1, big_signaling_bytes=35328)])
def test_control_info_renderer_matches_oracle(oracle_mod, sig):
    topo = Topology.example("abilene")
    params = engine_params(topo, sim_time_s=2.0, ping_as_obs=1, notify_dest=1, train=1, **sig)
    o = oracle_mod.OracleSim(topo, params)
    tr = InfoTracker(topo.n_nodes, 542)
    pol = sp_policy(topo)
    obs, n_ctrl, n_big = o.step(-1), 0, 0
    while obs is not None and n_ctrl < 300:
        v = o.pending_node()
        if int(obs[0]) == 1000:
            assert tr.render_control(obs, o.counters()) == o.last_info()
            n_ctrl += 1
            n_big += int(obs[3]) >> 16
        obs = o.step(pol(v, obs))
    assert n_ctrl == 300
    assert (n_big > 0) == bool(sig.get("big_signaling"))


def test_notify_dest_does_not_change_the_trajectory(oracle_mod):
    topo = Topology.example("abilene")
    base = engine_params(topo, sim_time_s=3.0, ping_as_obs=0)
    a = oracle_mod.OracleSim(topo, base)
    a.run_table(sp_next_hop_table(topo), 10 ** 9)
    o, stream = oracle_stream(oracle_mod, topo, dict(base, notify_dest=1), sp_policy(topo), 10 ** 9)
    assert a.records().tobytes() == o.records().tobytes()
    ca, co = a.counters(), o.counters()
    assert ca.tobytes() == co.tobytes()
    assert any(s[2] for s in stream)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")
@pytest.mark.parametrize("name,lf,train,sig", [("abilene", 2.0, 0, 0), ("abilene", 2.0, 1, 0),
                                               ("overlay_full_mesh_3n_abilene", 10.0, 1, 0),
                                               ("abilene", 1.0, 1, 1), ("overlay_full_mesh_3n_abilene", 10.0, 1, 1)])
def test_session_stream_matches_oracle(oracle_mod, name, lf, train, sig):
    from prisma_amd.ns3env import PrismaSession
    topo = Topology.example(name, 0, lf)
    kw = dict(sim_time_s=2.0, ping_as_obs=1, train=train)
    if sig:                                                        # "NN" echoes + big signalling
        kw.update(signaling_type="NN", big_signaling=1, sync_step_s=0.25)
    pol = sp_policy(topo)
    _, ref = oracle_stream(oracle_mod, topo, engine_params(topo, notify_dest=1, **kw), pol, 1500)
    s = PrismaSession(topo=topo, base_port=7000, **kw)
    got = []
    while s.pending() is not None and len(got) < len(ref):
        v, obs, done, info = s.pending()
        got.append((v, obs, done, info))
        s.apply(pol(v, obs))
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g == r, (i, g, r)
    assert len(got) == len(ref)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")
@pytest.mark.parametrize("name,lf", [("abilene", 1.0), ("overlay_full_mesh_3n_abilene", 10.0)])
def test_threaded_per_node_envs(oracle_mod, name, lf):
    """One Forwarder-like thread per overlay node over Ns3Env(port=base+index)."""
    from prisma_amd.ns3env import Ns3Env, PrismaSession
    topo = Topology.example(name, 0, lf)
    kw = dict(sim_time_s=1.5, ping_as_obs=1)
    pol = sp_policy(topo)
    s = PrismaSession(topo=topo, base_port=7100, **kw)
    nodes = [int(x) for x in topo.overlay_nodes]
    seen = {u: [] for u in nodes}
    errors = []

    # the reference builds every node's env in the main thread first (main.py:118-127)
    envs = {u: Ns3Env(port=7100 + i, stepTime=0, startSim=0, simSeed=100) for i, u in enumerate(nodes)}

    def forwarder(u):
        try:
            env = envs[u]
            assert env.node == u
            obs = env.reset()
            assert obs == [-1]
            obs, _, done, info = env.step(0)        # start-up state: the answer is ignored
            while env.connected:
                seen[u].append(list(obs))
                obs, _, done, info = env.step(pol(u, obs))
            env.ns3ZmqBridge.send_close_command()
        except Exception as e:                       # pragma: no cover - surfaced below
            errors.append(e)

    ths = [threading.Thread(target=forwarder, args=(u,)) for u in nodes]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    assert not errors and not any(t.is_alive() for t in ths)
    o, ref = oracle_stream(oracle_mod, topo, engine_params(topo, notify_dest=1, **kw), pol, 10 ** 9)
    for u in nodes:
        assert seen[u] == [obs for (v, obs, _, _) in ref if v == u], u
    got, want = s.counters(), o.counters()
    for k in ("hops", "decisions", "ov_injected", "ov_arrived", "ov_lost", "reward_sum", "cost_sum", "dec_count"):
        assert got[k] == want[k], k
