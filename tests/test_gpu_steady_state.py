"""Steady-state parity: every BASELINE workload compared with the CPU oracle record by record and
counter by counter, after every launch, well past the flow-start transient.

Flows start at 0.0001 + U(0, 1) s (/root/reference/prisma/ns3/sim.cc:610-630), so the first
simulated second is a transient: flows still starting, FIFOs filling. These runs go on until all
flows are active, FIFOs sit at their DropTail limit (point-to-point-net-device.cc:595-666), the
ping windows are full, the uid / FIFO ring / ping round indices have wrapped and the clock is past
2^32 ns; the headline workload runs a whole 60-s episode, its end and the auto-reset into episode 1
(main.py:111-114's episode loop).

Each test prints "compared up to t = ... s" for its workload. The DQN-buffer workloads also check
every in-kernel decision against the fp32 torch model (parity_util.check_near_ties).
"""
import numpy as np
import pytest
import torch

from parity_util import compare_steady
from prisma_amd.config import engine_params
from prisma_amd.engine import PRISMA_ENGINE_MEMORY, PrismaEngine
from prisma_amd.topology import DATA_DIR, Topology, sp_next_hop_table

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]


def _buffer_net(topo, seed):
    from prisma_amd.policies import StackedQNet
    net = StackedQNet(topo, "buffer", seed=seed, device="cpu")
    return net, net.pack().numpy()


def test_config2_headline_full_episode_and_auto_reset(oracle_mod):
    """Config 2 (the headline): Abilene TM0 lf 1.0, DQ-routing greedy table from the bench's
    random-init weights (seed 1234), pingAsObs=1, simTime 60 s, auto-reset: a whole episode, its
    end inside a launch (the replicas continue into episode 1 in the same launch) and 5 s of
    episode 1, on 2 replicas."""
    from prisma_amd.policies import StackedQNet
    topo = Topology.example("abilene", 0, 1.0)
    table = StackedQNet(topo, "routing", seed=1234, device="cpu").argmin_table().numpy()
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1, auto_reset=1, seed=100, replica_base=17,
                           log_capacity=65536)
    eng = PrismaEngine(topo, params, 2)
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("table", table), t_target_s=65.0,
                         hops_per_launch=16384, min_episode=1, label="config 2 abilene dq_routing")
    eng.close()
    assert out["t_compared_s"] >= 65.0 and min(out["episodes"]) >= 1
    # the episode end happened inside a launch and the replicas continued into episode 1 there:
    # every launch executed its whole hop budget (no work lost at the boundary)
    assert out["short_launches"] == 0


def test_config2_headline_at_bench_shape(oracle_mod):
    """The headline at the bench's own launch shape (bench.py PRESETS["config2"] and measure()):
    32 768 hops per replica per launch into a log ring of 8 192 records, auto-reset, seed 100.
    A launch writes ~4x the records the ring holds, so the ring wraps inside every launch: the
    last 8 192 records of each launch and every counter are compared, through the 60-s episode
    end (about every 4 launches at this shape) and the spare-image restart into episode 1, on
    two of the bench's replicas (global ids 4094, 4095)."""
    from prisma_amd.policies import StackedQNet
    topo = Topology.example("abilene", 0, 1.0)
    table = StackedQNet(topo, "routing", seed=1234, device="cpu").argmin_table().numpy()
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1, auto_reset=1, seed=100, replica_base=4094,
                           log_capacity=8192)
    eng = PrismaEngine(topo, params, 2)
    assert eng.log_capacity == 8192
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("table", table), t_target_s=65.0,
                         hops_per_launch=32768, min_episode=1, log_tail=True,
                         label="config 2 abilene dq_routing, bench shape (32768 hops, log 8192)")
    eng.close()
    assert out["t_compared_s"] >= 65.0 and min(out["episodes"]) >= 1
    assert out["short_launches"] == 0
    assert out["tail_launches"] == 2 * out["launches"]         # the ring wrapped inside every launch


@pytest.mark.parametrize("preset,t_target,min_ep", [("config3", 65.0, 1), ("config4", 15.0, 0), ("config5", 3.0, 0)])
def test_dqn_configs_at_bench_shape(oracle_mod, preset, t_target, min_ep):
    """Configs 3-5 at their bench presets' own launch shape (bench.py PRESETS: hops per replica per
    launch; measure(): log capacity 8 192, 65 536 beyond 256 links; auto-reset, seed 100, the
    random-init DQN-buffer weights of seed 1234), with the log tail compared where a launch writes
    more records than the ring holds. Config 3 runs through its 60-s episode end."""
    import bench
    from prisma_amd.policies import StackedQNet
    pr = bench.PRESETS[preset]
    topo = Topology.example(pr["topology"], 0, 1.0)
    net = StackedQNet(topo, "buffer", seed=1234, device="cpu")
    w = net.pack().numpy()
    log_cap = 65536 if topo.n_links > 256 else 8192
    R = 1 if preset == "config5" else 2
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=pr["ping_as_obs"], auto_reset=1, seed=100,
                           replica_base=pr["replicas"] - R, log_capacity=log_cap)
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("mlp", w), t_target_s=t_target, hops_per_launch=pr["hops"],
                         min_episode=min_ep, net_cpu=net, log_tail=True,
                         label=f"{preset} at the bench shape ({pr['hops']} hops, log {log_cap})")
    eng.close()
    assert out["t_compared_s"] >= t_target and min(out["episodes"]) >= min_ep and out["short_launches"] == 0


def test_config3_abilene_on_geant_dqn_buffer_episode_end(oracle_mod):
    """Config 3 through the regime its bench runs in: the tunnelled-overlay kernels (relay entries
    with the tunnel target, LDS FIFO windows, engine_core.h q_put / q_take) from t = 0 past the 60-s
    episode end (Simulator::Stop, /root/reference/prisma/ns3/sim.cc:703-716; main.py:111-115's
    episode loop) and the spare-image restart (engine_core.h spare_restart) into episode 1,
    DQN-buffer with pingAsObs=1, near-ties checked against torch fp32, on 2 replicas."""
    topo = Topology.example("abilene_on_geant", 0, 1.0)
    net, w = _buffer_net(topo, seed=7)
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1, auto_reset=1, seed=100, replica_base=4001,
                           log_capacity=65536)
    eng = PrismaEngine(topo, params, 2)
    assert eng.kernel_info()["relay_ip"] == 1                  # the benchmarked (relay-entry) kernels
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("mlp", w), t_target_s=65.0, hops_per_launch=16384,
                         min_episode=1, net_cpu=net, label="config 3 abilene-on-geant dqn_buffer 60-s episode end")
    eng.close()
    assert out["t_compared_s"] >= 65.0 and min(out["episodes"]) >= 1
    assert out["short_launches"] == 0


def _random_table(topo, seed):
    rng = np.random.default_rng(seed)
    table = np.zeros((topo.n_nodes, topo.n_nodes), dtype=np.uint8)
    for u in topo.overlay_nodes:
        table[u] = rng.integers(0, topo.degrees[u], topo.n_nodes)
    return table


@pytest.mark.parametrize("ping", [0, 1])
def test_tunnel_table_short_episodes_deep_fifos(oracle_mod, ping):
    """Table-policy twin of the config-3 episode-end test on the shipped 3-node tunnelled mesh at
    load factor 20: 4-s episodes, auto-reset, a random action table. FIFOs inside tunnels overflow
    (drops charged to the sender, data-packet-manager.cc:88-106; ipv4-interface.cc:213-229) and
    every episode ends with FIFOs deeper than the LDS window, so packets sit in both the LDS
    windows and the HBM ring when the spare image replaces the state. Compared through 3 episode
    ends."""
    topo = Topology.example("overlay_full_mesh_3n_abilene", 0, 20.0)
    table = _random_table(topo, 11 + ping)
    params = engine_params(topo, sim_time_s=4.0, ping_as_obs=ping, auto_reset=1, seed=23, replica_base=70 + ping,
                           log_capacity=65536)
    eng = PrismaEngine(topo, params, 2)
    assert eng.kernel_info()["relay_ip"] == 1
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("table", table), t_target_s=13.0, hops_per_launch=8192,
                         min_episode=3, label=f"3-node tunnelled mesh lf 20 pingAsObs {ping}, 4-s episodes")
    eng.close()
    assert out["t_compared_s"] >= 13.0 and min(out["episodes"]) >= 3
    assert out["relay_drops"] > 0                              # drops on FIFOs inside tunnels
    ends = out["end_diag"]
    assert len(ends) >= 6 and all(d["deep_fifos"] > 0 for d in ends), ends   # LDS window + HBM ring in use
    print(f"[steady] episode ends: {ends}; drops inside tunnels: {out['relay_drops']}")


@pytest.mark.parametrize("ping", [0, 1])
@pytest.mark.parametrize("lf", [0.5, 1.0, 2.0])
def test_config4_geant_dqn_buffer_steady(oracle_mod, lf, ping):
    """Config 4: GEANT TM0, in-kernel DQN-buffer, 15 s of simulated time on 2 replicas."""
    topo = Topology.example("geant", 0, lf)
    net, w = _buffer_net(topo, seed=41 + int(lf * 4))
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=ping, seed=100, replica_base=2048 + int(lf * 8),
                           log_capacity=65536)
    eng = PrismaEngine(topo, params, 2)
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("mlp", w), t_target_s=15.0, hops_per_launch=16384,
                         net_cpu=net, label=f"config 4 geant lf {lf} pingAsObs {ping}")
    eng.close()
    assert out["t_compared_s"] >= 15.0 and out["mlp_decisions"] > 10000


def test_config4_geant_dqn_buffer_episode_ends(oracle_mod):
    """Config 4's instance (identity overlay, in-kernel DQN-buffer, 8 flow and 2 link slots) through
    two episode ends inside launches: 6-s episodes, auto-reset, so the spare-image restart and the
    second event-loop copy (step_kernel.h) run the MLP, compared through t = 13 s."""
    topo = Topology.example("geant", 0, 1.0)
    net, w = _buffer_net(topo, seed=43)
    params = engine_params(topo, sim_time_s=6.0, ping_as_obs=0, auto_reset=1, seed=100, replica_base=1500,
                           log_capacity=65536)
    eng = PrismaEngine(topo, params, 2)
    ki = eng.kernel_info()
    assert (ki["flow_slots"], ki["link_slots"], ki["tunnels"], ki["ctrl"]) == (8, 2, 0, 0)
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("mlp", w), t_target_s=13.0, hops_per_launch=16384,
                         min_episode=2, net_cpu=net, label="config 4 geant dqn_buffer 6-s episodes")
    eng.close()
    assert out["t_compared_s"] >= 13.0 and min(out["episodes"]) >= 2 and out["short_launches"] == 0


def test_config3_abilene_on_geant_dqn_buffer_steady(oracle_mod):
    """Config 3: the Abilene overlay tunnelled over GEANT, DQN-buffer, pingAsObs=1, 15 s."""
    topo = Topology.example("abilene_on_geant", 0, 1.0)
    net, w = _buffer_net(topo, seed=7)
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1, seed=100, replica_base=4000, log_capacity=65536)
    eng = PrismaEngine(topo, params, 2)
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("mlp", w), t_target_s=15.0, hops_per_launch=16384,
                         net_cpu=net, label="config 3 abilene-on-geant dqn_buffer")
    eng.close()
    assert out["t_compared_s"] >= 15.0 and out["mlp_decisions"] > 5000


def test_config5_er256_dqn_buffer_steady(oracle_mod):
    """Config 5: ER-256 on the memory-resident engine, DQN-buffer, pingAsObs=1, 3 s on 1 replica."""
    topo = Topology.example("er256")
    net, w = _buffer_net(topo, seed=5)
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1, seed=100, replica_base=8191, log_capacity=65536)
    eng = PrismaEngine(topo, params, 1)
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("mlp", w), t_target_s=3.0, hops_per_launch=16384,
                         net_cpu=net, label="config 5 er256 dqn_buffer")
    eng.close()
    assert out["t_compared_s"] >= 3.0


def test_config5_er256_dqn_buffer_episode_end(oracle_mod):
    """Config 5 across an episode end on the memory-resident engine: simTime 6 s, auto-reset, the
    DQN-buffer agent, compared through t = 6.5 s (episode 1 reached). The memory engine keeps
    32-bit link leaf keys (time = now + (lo - lo32(now)), prisma_engine_mem.hip), so this run
    takes them past lo32(now) wrapping at 2^32 ns = 4.295 s, then through Simulator::Stop
    (/root/reference/prisma/ns3/sim.cc:703-716) and the reset into episode 1."""
    topo = Topology.example("er256")
    net, w = _buffer_net(topo, seed=5)
    params = engine_params(topo, sim_time_s=6.0, ping_as_obs=1, auto_reset=1, seed=100, replica_base=8190,
                           log_capacity=65536)
    eng = PrismaEngine(topo, params, 1)
    assert eng.engine_kind == PRISMA_ENGINE_MEMORY
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("mlp", w), t_target_s=6.5, hops_per_launch=16384,
                         min_episode=1, net_cpu=net, label="config 5 er256 dqn_buffer 6-s episodes")
    eng.close()
    assert out["t_compared_s"] >= 6.5 and min(out["episodes"]) >= 1 and out["max_clock_s"] > 4.3


@pytest.mark.parametrize("name,policy", [("abilene", "table"), ("abilene", "mlp"), ("geant", "table"),
                                         ("geant", "mlp")])
def test_mem_engine_forced_long_run(oracle_mod, name, policy):
    """The register engine's workloads forced onto the memory-resident engine for 15 s of
    simulated time (clock past 2^32 ns, FIFOs at their limit, ring and uid wrap)."""
    topo = Topology.example(name, 0, 1.5)
    if policy == "table":
        net, pol = None, ("table", sp_next_hop_table(topo))
    else:
        net, w = _buffer_net(topo, seed=13)
        pol = ("mlp", w)
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1, seed=31, replica_base=600, log_capacity=65536,
                           engine=PRISMA_ENGINE_MEMORY)
    eng = PrismaEngine(topo, params, 2)
    assert eng.engine_kind == PRISMA_ENGINE_MEMORY
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, pol, t_target_s=15.0, hops_per_launch=16384,
                         net_cpu=net, label=f"memory engine {name} {policy}")
    eng.close()
    assert out["t_compared_s"] >= 15.0


def test_config5_er256_big_signaling_long_run(oracle_mod):
    """Config 5's graph with --train, "NN" echoes and big signalling (2 006 generators) on the
    memory-resident engine past 2^32 ns: compared through t = 4.6 s."""
    topo = Topology.example("er256")
    table = np.load(f"{DATA_DIR}/er256/sp_next_hop_table.npy")
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1, train=1, signaling_type="NN", big_signaling=1,
                           big_signaling_bytes=35328, sync_step_s=0.5, seed=11, replica_base=77,
                           log_capacity=65536)
    eng = PrismaEngine(topo, params, 1)
    assert eng.engine_kind == PRISMA_ENGINE_MEMORY
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("table", table), t_target_s=4.6, hops_per_launch=16384,
                         label="config 5 er256 big signalling")
    eng.close()
    assert out["t_compared_s"] >= 4.6


def test_config5_er256_sp_table_steady(oracle_mod):
    """Config 5's graph with the SP table (the memory engine's table path), 3 s on 1 replica."""
    topo = Topology.example("er256")
    table = np.load(f"{DATA_DIR}/er256/sp_next_hop_table.npy")
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=0, seed=100, replica_base=3, log_capacity=65536)
    eng = PrismaEngine(topo, params, 1)
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("table", table), t_target_s=3.0, hops_per_launch=16384,
                         label="config 5 er256 sp")
    eng.close()
    assert out["t_compared_s"] >= 3.0
