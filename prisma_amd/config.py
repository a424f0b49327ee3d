"""Scenario parameters — the reference's argument_parser.py defaults.

``parse_arguments()`` mirrors the flag names, groups and defaults of
prisma/source/argument_parser.py:33-94 for the flags that shape the packet
hop (global simulation, network and the agent type); ``engine_params()``
turns them into the C-ABI ``prisma_params_t`` dictionary the engine and the
oracle both consume.
"""
from __future__ import annotations

import argparse
from typing import Optional

from .topology import Topology, loss_penalty as _loss_penalty

DEFAULTS = dict(
    numEpisodes=1, simTime=60, basePort=6555, seed=100, train=1, max_nb_arrived_pkts=-1,
    movingAverageObsSize=5, activateUnderlayTraffic=0, pingAsObs=1, pingPacketIntervalTime=0.2,
    load_factor=1.0, topology_name="abilene", traffic_matrix_index=0, max_out_buffer_size=16260,
    link_delay=1, packet_size=512, link_cap=500000, agent_type="dqn_buffer", signaling_type="ideal",
    loss_penalty_type="fixed", signalingSim=0, sync_step=1.0, bigSignalingSize=512,
)
SIGNALING_TYPES = {"ideal": 0, "NN": 1, "target": 2}      # include/prisma.h PRISMA_SIGNALING_*
RNG_MODES = {"philox": 0, "ns3": 1}                           # include/prisma.h PRISMA_RNG_*

AGENT_TYPES = ["dqn_buffer", "dqn_routing", "dqn_buffer_fp", "dqn_buffer_lite", "dqn_buffer_lighter",
               "dqn_buffer_lighter_2", "dqn_buffer_lighter_3", "dqn_buffer_ff",
               "dqn_buffer_with_throughputs", "sp", "opt"]


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="prisma_amd", allow_abbrev=False)
    g1 = p.add_argument_group("Global simulation arguments")
    g1.add_argument("--numEpisodes", type=int, default=DEFAULTS["numEpisodes"])
    g1.add_argument("--simTime", type=int, default=DEFAULTS["simTime"])
    g1.add_argument("--basePort", type=int, default=DEFAULTS["basePort"])
    g1.add_argument("--seed", type=int, default=DEFAULTS["seed"])
    g1.add_argument("--train", type=int, default=DEFAULTS["train"])
    g1.add_argument("--max_nb_arrived_pkts", type=int, default=DEFAULTS["max_nb_arrived_pkts"])
    g1.add_argument("--movingAverageObsSize", type=int, default=DEFAULTS["movingAverageObsSize"])
    g1.add_argument("--activateUnderlayTraffic", type=int, default=DEFAULTS["activateUnderlayTraffic"])
    g1.add_argument("--pingAsObs", type=int, default=DEFAULTS["pingAsObs"])
    g1.add_argument("--pingPacketIntervalTime", type=float, default=DEFAULTS["pingPacketIntervalTime"])
    g1.add_argument("--signalingSim", type=int, default=DEFAULTS["signalingSim"])
    g4 = p.add_argument_group("Network parameters")
    g4.add_argument("--load_factor", type=float, default=DEFAULTS["load_factor"])
    g4.add_argument("--topology_name", type=str, choices=["abilene", "geant"], default=DEFAULTS["topology_name"])
    g4.add_argument("--traffic_matrix_index", type=int, default=DEFAULTS["traffic_matrix_index"])
    g4.add_argument("--max_out_buffer_size", type=int, default=DEFAULTS["max_out_buffer_size"])
    g4.add_argument("--link_delay", type=int, default=DEFAULTS["link_delay"])
    g4.add_argument("--packet_size", type=int, default=DEFAULTS["packet_size"])
    g4.add_argument("--link_cap", type=int, default=DEFAULTS["link_cap"])
    g3 = p.add_argument_group("DRL Agent arguments")
    g3.add_argument("--agent_type", choices=AGENT_TYPES, type=str, default=DEFAULTS["agent_type"])
    g3.add_argument("--signaling_type", type=str, choices=["NN", "target", "ideal"], default=DEFAULTS["signaling_type"])
    g3.add_argument("--loss_penalty_type", type=str, choices=["None", "fixed"], default=DEFAULTS["loss_penalty_type"])
    g3.add_argument("--bigSignalingSize", type=int, default=DEFAULTS["bigSignalingSize"])
    g3.add_argument("--sync_step", type=float, default=DEFAULTS["sync_step"])
    return p


def parse_arguments(argv=None) -> dict:
    params = vars(build_parser().parse_args(argv))
    topo = Topology.example(params["topology_name"], params["traffic_matrix_index"], params["load_factor"])
    params["numNodes"] = topo.n_overlay
    params["topology"] = topo
    params["loss_penalty"] = _loss_penalty(params["max_out_buffer_size"], params["packet_size"],
                                           params["link_cap"], topo.n_overlay)
    return params


def engine_params(topo: Topology, *, sim_time_s: float = 60.0, seed: int = 100, ping_as_obs: int = 1,
                  ping_interval_s: float = 0.2, ma_size: int = 5, link_cap: int = 500000,
                  link_delay_ms: float = 1.0, max_buffer: int = 16260, packet_size: int = 512,
                  auto_reset: int = 0, log_capacity: int = 8192, replica_base: int = 0,
                  loss_penalty: Optional[float] = None, train: int = 0, notify_dest: int = 0,
                  engine: int = 0, signaling_type="ideal", big_signaling: int = 0, sync_step_s: float = 1.0,
                  big_signaling_bytes: int = DEFAULTS["bigSignalingSize"], rng: str = "philox",
                  rng_stream_offset: int = 0) -> dict:
    """prisma_params_t as a dict (shared by the engine binding and the oracle).

    train=1 is the reference's --train: every data notification at a non-source
    node sends a small-signalling echo back to its last hop.
    engine: 0 auto (register-resident when the topology fits it), 1 register-resident,
    2 memory-resident (include/prisma.h PRISMA_ENGINE_*).
    signaling_type ("ideal" / "NN" / "target" or 0 / 1 / 2) sets the echo's payload (sim.cc:373-392);
    big_signaling=1 is the simulator's --signaling with "NN" and --train: NN-weight segments of
    big_signaling_bytes every sync_step_s between overlay neighbours (sim.cc:634-647; run_ns3.py
    passes signalingSim, sync_step and bigSignalingSize, whose argument_parser.py:74 default, 512 B = one
    segment per NN, is the default here too; sim.cc's own default is 35328).  The simulator switches --signaling off
    for the sp / opt agents and for "ideal" (sim.cc:374-376): the caller's part, as in run_ns3.py.
    rng: "philox" (counter-based streams per replica, flow, draw and episode) or "ns3" (ns-3's
    MRG32k3a RngStream streams, one per RandomVariable object in the reference's creation order,
    simSeed = seed + replica id; rng_stream_offset = the streams ns-3 creates before sim.cc's flow
    loop, include/prisma.h PRISMA_RNG_NS3)."""
    if log_capacity < 1024 or log_capacity > (1 << 22) or log_capacity & (log_capacity - 1):
        raise ValueError("log_capacity must be a power of two in [1024, 2^22]")
    lp = _loss_penalty(max_buffer, packet_size, link_cap, topo.n_overlay) if loss_penalty is None else loss_penalty
    st = SIGNALING_TYPES.get(signaling_type, -1) if isinstance(signaling_type, str) else int(signaling_type)
    if st not in (0, 1, 2):
        raise ValueError("signaling_type must be 'ideal', 'NN' or 'target'")
    return dict(
        link_bps=int(link_cap), link_delay_ns=int(round(link_delay_ms * 1e6)),
        max_buffer_bytes=int(max_buffer), packet_size=int(packet_size), sim_time_s=float(sim_time_s),
        ping_interval_s=float(ping_interval_s), ma_size=int(ma_size), ping_as_obs=int(ping_as_obs),
        auto_reset=int(auto_reset), loss_penalty=float(lp), seed=int(seed),
        replica_base=int(replica_base), log_capacity=int(log_capacity), notify_dest=int(notify_dest),
        train=int(train), engine=int(engine), signaling_type=st, big_signaling=int(big_signaling),
        sync_step_s=float(sync_step_s), big_signaling_bytes=int(big_signaling_bytes),
        rng_mode=RNG_MODES[rng] if isinstance(rng, str) else int(rng), rng_stream_offset=int(rng_stream_offset),
    )
