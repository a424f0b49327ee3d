"""Signalling in the CPU oracle (test infrastructure) and the scenario checks of the C-ABI:
the small-signalling payload by signalling type (sim.cc:373-392) and the big-signalling
NN-weight generators (sim.cc:634-647, big-signaling-application.cc:224-309,
big-signaling-packet-manager.cc:93-123).  Parity of the GPU engine: tests/test_gpu_signaling.py."""
import numpy as np
import pytest

from prisma_amd.config import engine_params, parse_arguments
from prisma_amd.topology import Topology, sp_next_hop_table

EV_START, EV_BSTART, EV_BSEND = 1, 5, 6
APP_START_NS = 100000                      # AppStartTime 0.0001 s (sim.cc:244)
P_NS = 14492754                            # 4096 / (35328 * 8 / 1.0f) s, rounded to ns


def big_params(topo, **kw):
    # sim.cc's NN size (69 segments per NN; engine_params defaults to the Python CLI's 512 B)
    base = dict(sim_time_s=2.0, ping_as_obs=1, train=1, signaling_type="NN", big_signaling=1, big_signaling_bytes=35328)
    base.update(kw)
    return engine_params(topo, **base)


def neighbour_flows(topo):
    """Flows between overlay neighbours, in flow order: the generators' pairs."""
    out = []
    for f in range(topo.n_flows):
        u, w = int(topo.flow_src[f]), int(topo.flow_dst[f])
        t0, t1 = int(topo.ov_row_ptr[u]), int(topo.ov_row_ptr[u + 1])
        if w in [int(x) for x in topo.tun_dst[t0:t1]]:
            out.append(f)
    return out


def test_period_known_answers(oracle_mod):
    L = oracle_mod.lib()
    # dataRate = (uint32 size * 8) / float syncStep is a float; delay = 4096 / dataRate a double
    for size, step, want in [(35328, 1.0, P_NS), (512, 1.0, 1000000000), (35328, 0.5, 7246377),
                             (1024, 0.1, 50000000)]:
        rate = np.float32(np.float32(size * 8) / np.float32(step))
        assert L.or_seconds_to_ns(4096 / float(rate)) == want, (size, step)


def test_generators_follow_their_flows(oracle_mod):
    topo = Topology.example("abilene")
    params = big_params(topo, sim_time_s=1.0)
    o = oracle_mod.OracleSim(topo, params)
    o.enable_trace()
    o.run_table(sp_next_hop_table(topo), 10 ** 9)
    tr = o.trace()
    gens = neighbour_flows(topo)
    assert len(gens) > 0
    starts = tr[tr[:, 2] == EV_BSTART]
    assert sorted(starts[:, 3].tolist()) == list(range(len(gens)))
    assert np.all(starts[:, 0] == APP_START_NS)
    # install order: generator g's start event is scheduled right after its flow's (seq + 1)
    fstart = {int(r[3]): int(r[1]) for r in tr[tr[:, 2] == EV_START]}
    for r in starts:
        assert int(r[1]) == fstart[gens[int(r[3])]] + 1
    # then one segment every period, from one period after the start to the end of the episode
    sends = tr[tr[:, 2] == EV_BSEND]
    n = (int(round(1e9)) - 1 - APP_START_NS) // P_NS
    for g in range(len(gens)):
        t = np.sort(sends[sends[:, 3] == g][:, 0])
        assert np.array_equal(t, APP_START_NS + P_NS * np.arange(1, n + 1)), g


def test_no_generators_unless_train_nn_and_signaling(oracle_mod):
    topo = Topology.example("abilene")
    for kw in (dict(train=0), dict(signaling_type="ideal"), dict(signaling_type="target"), dict(big_signaling=0)):
        o = oracle_mod.OracleSim(topo, big_params(topo, sim_time_s=0.3, **kw))
        o.enable_trace()
        o.run_table(sp_next_hop_table(topo), 10 ** 9)
        assert not np.any(o.trace()[:, 2] >= EV_BSTART), kw


def drive(o, topo, max_steps):
    """SP actions for every data notification; returns the control notifications
    (node, obs, info) in order."""
    table = sp_next_hop_table(topo)
    notes = []
    obs = o.step(-1)
    for _ in range(max_steps):
        if obs is None:
            break
        v = o.pending_node()
        if obs[0] == 1000:
            notes.append((v, obs.copy(), o.last_info()))
            a = 0
        else:
            a = int(table[v, int(topo.overlay_nodes[int(obs[0])])])
        obs = o.step(a)
    return notes


def test_big_signalling_notifications(oracle_mod):
    topo = Topology.example("abilene")
    params = big_params(topo, sim_time_s=0.8, notify_dest=1)
    o = oracle_mod.OracleSim(topo, params)
    notes = drive(o, topo, 200000)
    big = [(v, ob, info) for v, ob, info in notes if ob[3] & 0x10000]
    echo = [(v, ob, info) for v, ob, info in notes if not ob[3] & 0x10000]
    assert big and echo
    nseg = 35328 // 512
    last = {}
    for v, ob, info in big:
        src = int(ob[3]) & 0xffff
        assert src in topo.neighbors(v)
        nn, seg = int(ob[1]), int(ob[2])
        assert 0 <= seg < nseg
        n = nn * nseg + seg
        assert n > last.get((src, v), 0)                  # segments of one generator in order
        last[(src, v)] = n
        tok = info.split(",")
        assert len(tok) == 21
        assert tok[1].strip() == "Packet Size=542" and tok[4].strip() == "packetType =1"
        assert tok[18].strip() == f"NN Index={nn}" and tok[19].strip() == f"segment Index={seg}"
        assert tok[20].strip() == f"NodeId Signaled={src}"
    # every generator between neighbours reached its neighbour
    assert len(last) == len(neighbour_flows(topo))


def test_echo_payload_by_signaling_type(oracle_mod):
    topo = Topology.example("abilene")
    sizes = {"ideal": {30}, "target": {54}, "NN": {30 + 8 + 8 * (int(d) + 1) for d in topo.degrees}}
    for st, want in sizes.items():
        o = oracle_mod.OracleSim(topo, engine_params(topo, sim_time_s=0.3, ping_as_obs=1, train=1, notify_dest=1,
                                                     signaling_type=st))
        got = {int(ob[2]) for v, ob, info in drive(o, topo, 50000)}
        assert got and got <= want, st
        if st == "NN":
            assert len(got) > 1                                # per-node sizes


def test_parse_arguments_signaling_flags():
    p = parse_arguments(["--signaling_type", "NN", "--signalingSim", "1", "--sync_step", "0.5",
                         "--bigSignalingSize", "35328"])
    assert p["signaling_type"] == "NN" and p["signalingSim"] == 1
    assert p["sync_step"] == 0.5 and p["bigSignalingSize"] == 35328
    topo = p["topology"]
    e = engine_params(topo, train=1, signaling_type=p["signaling_type"], big_signaling=p["signalingSim"],
                      sync_step_s=p["sync_step"], big_signaling_bytes=p["bigSignalingSize"])
    assert e["signaling_type"] == 1 and e["big_signaling"] == 1
    with pytest.raises(ValueError):
        engine_params(topo, signaling_type="bogus")


def test_plan_rejects_unsupported_signaling():
    """prisma_plan (no device): both engines plan every signalling type on identity overlays
    (ER-256's 2 006 generators only fit the memory-resident engine); tunnelled overlays with
    per-node echo sizes and send indices beyond the 17-bit segment field refuse instead of
    running a different model."""
    from prisma_amd.engine import PRISMA_ENGINE_MEMORY, PRISMA_ENGINE_REGISTER, PrismaError, plan
    topo = Topology.example("abilene")
    assert plan(topo, big_params(topo))["flow_slots"] >= 1
    assert plan(topo, big_params(topo, engine=PRISMA_ENGINE_MEMORY))["engine"] == PRISMA_ENGINE_MEMORY
    assert plan(topo, engine_params(topo, train=1, signaling_type="target",
                                    engine=PRISMA_ENGINE_MEMORY))["engine"] == PRISMA_ENGINE_MEMORY
    er = Topology.example("er256")
    assert plan(er, big_params(er))["engine"] == PRISMA_ENGINE_MEMORY
    with pytest.raises(PrismaError, match="register-resident"):
        plan(er, big_params(er, engine=PRISMA_ENGINE_REGISTER))
    with pytest.raises(PrismaError, match="2\\^17"):
        plan(topo, big_params(topo, sync_step_s=0.001))
    aog = Topology.example("abilene_on_geant")                    # overlay degrees 2..4
    with pytest.raises(PrismaError, match="equal overlay"):
        plan(aog, big_params(aog))
    assert plan(aog, big_params(aog, signaling_type="target", big_signaling=0))["flow_slots"] >= 1
    mesh = Topology.example("overlay_full_mesh_3n_abilene")        # overlay degree 2 everywhere
    assert plan(mesh, big_params(mesh))["flow_slots"] >= 1
