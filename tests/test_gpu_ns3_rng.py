"""ns-3 random streams (PRISMA_RNG_NS3) on the HIP engine vs the CPU oracle, bit-exact, through
the C-ABI: the flows' start offsets from the flow loop's UniformRandomVariables (sim.cc:610-620)
and every inter-arrival from a new stream per packet (poisson-application.cc:281, 311), on both
engines, with the table and DQN-buffer policies, and across an auto-reset episode boundary
(ns-3 restarts with the same seed: the same streams).  The oracle's stream assignment itself is
checked in tests/test_mrg32k3a.py."""
import numpy as np
import pytest
import torch

from parity_util import compare_steady
from prisma_amd.config import engine_params
from prisma_amd.engine import PRISMA_ENGINE_MEMORY, PrismaEngine
from prisma_amd.topology import Topology, sp_next_hop_table

from test_gpu_parity import run_table_both
from test_gpu_mem_engine import er256, run_both

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]


@pytest.mark.parametrize("name,tm,lf,kw", [
    ("abilene", 0, 1.0, dict()),
    ("abilene", 2, 2.0, dict(rng_stream_offset=66, seed=7, ping_as_obs=0)),
    ("geant", 0, 1.0, dict(rng_stream_offset=148)),
    ("abilene_on_geant", 0, 1.0, dict(train=1)),
])
def test_ns3_streams_table_parity(oracle_mod, name, tm, lf, kw):
    topo = Topology.example(name, tm, lf)
    params = engine_params(topo, sim_time_s=20.0, rng="ns3", replica_base=3, **kw)
    cnt = run_table_both(oracle_mod, topo, params, 4, 3000, sp_next_hop_table(topo))
    assert int(cnt["ov_injected"].min()) > 0


def test_ns3_streams_memory_engine_parity(oracle_mod):
    topo, table = er256()
    params = engine_params(topo, sim_time_s=60.0, rng="ns3", rng_stream_offset=1536, replica_base=11)
    run_both(oracle_mod, topo, params, 2, 4000, table, launches=2)


def test_ns3_streams_dqn_buffer_parity(oracle_mod):
    from prisma_amd.policies import StackedQNet
    topo = Topology.example("geant")
    net = StackedQNet(topo, "buffer", seed=23, device="cpu")
    w = StackedQNet(topo, "buffer", seed=23).pack()
    params = engine_params(topo, sim_time_s=20.0, ping_as_obs=1, rng="ns3", replica_base=1, engine=PRISMA_ENGINE_MEMORY)
    run_both(oracle_mod, topo, params, 2, 2000, w, launches=2, mlp=True, net_cpu=net)


def test_ns3_streams_auto_reset_repeats_the_episode(oracle_mod):
    """Two 2-s episodes in one fused run: episode 1 continues in the launch (spare image) and
    replays episode 0's streams; every record and counter equal to the oracle's chain."""
    topo = Topology.example("abilene")
    params = engine_params(topo, sim_time_s=2.0, rng="ns3", auto_reset=1, replica_base=9, log_capacity=65536)
    eng = PrismaEngine(topo, params, 2)
    eng.reset(0)
    out = compare_steady(oracle_mod, eng, topo, params, ("table", sp_next_hop_table(topo)), t_target_s=3.0,
                         hops_per_launch=3000, min_episode=1, label="ns-3 streams abilene auto-reset")
    eng.close()
    assert min(out["episodes"]) >= 1
