"""bench.py's host side on CPU: the BASELINE presets resolve to their configurations (explicit flags
win), and the CPU baseline (the oracle on host threads, test infrastructure) runs both kinds of
policy -- the action table and the DQN-buffer MLP -- on a bounded sample, capped at the replica count."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from prisma_amd.config import engine_params  # noqa: E402
from prisma_amd.policies import StackedQNet  # noqa: E402
from prisma_amd.topology import Topology, sp_next_hop_table  # noqa: E402


def test_presets_and_overrides():
    a = bench.parse(["--preset", "config4"])
    assert (a.topology, a.policy, a.replicas, a.ping_as_obs) == ("geant", "dqn_buffer", 2048, 0)
    assert a.lfs == [0.5, 0.75, 1.0, 1.25, 1.5, 1.75, 2.0] and a.hops == 8192
    assert bench.parse(["--preset", "config5"]).hops == 32768 and bench.parse(["--preset", "config2"]).hops == 32768
    a = bench.parse(["--preset", "config4", "--load-factors", "1.0,2.0", "--replicas", "64", "--ping-as-obs", "1"])
    assert a.lfs == [1.0, 2.0] and a.replicas == 64 and a.ping_as_obs == 1
    a = bench.parse(["--preset", "config5"])
    assert (a.topology, a.policy, a.replicas, a.warmup, a.lfs) == ("er256", "dqn_buffer", 1024, 4, [1.0])
    a = bench.parse(["--preset", "config1"])
    assert (a.policy, a.replicas, a.hops) == ("sp", 1, 2048)
    assert bench.parse(["--topology", "er256", "--policy", "dqn_buffer"]).hops == 8192
    a = bench.parse([])                                             # the driver's default: config 2
    assert (a.topology, a.policy, a.replicas, a.lfs, a.warmup, a.hops) == ("abilene", "dq_routing", 4096, [1.0], 2,
                                                                           32768)
    assert a.cpu_hops == 8000000 and bench.parse(["--preset", "config3"]).cpu_hops == 1200000


def test_cpu_baseline_table_and_mlp(oracle_mod):
    topo = Topology.example("abilene")
    params = engine_params(topo, sim_time_s=2.0, ping_as_obs=1, auto_reset=0, seed=100)
    r = bench.cpu_baseline(topo, params, "table", sp_next_hop_table(topo), 30000, 10000, threads=1)
    assert r["cores"] == 1 and r["kind"] == "port" and r["value"] > 0 and r["value_1core"] > 0
    assert "episodes" in r["sample"] and "not runnable" in r["sample"]
    w = StackedQNet(topo, "buffer", seed=1234, device="cpu").pack().numpy().astype(np.float32)
    r = bench.cpu_baseline(topo, params, "mlp", w, 5000, 2000, threads=2, warm_hops=500, workload="abilene mlp")
    assert r["cores"] <= 2 and r["value"] > 0 and "DQN-buffer MLP" in r["sample"] and "500 hops untimed" in r["sample"]
    assert r["workload"] == "abilene mlp"


def test_cpu_baseline_worker_failure_ends_promptly(oracle_mod, monkeypatch):
    """A worker that raises (here: its oracle cannot be built) aborts the threads' barrier, so
    cpu_baseline raises at once instead of waiting for the rank deadline."""
    import time
    topo = Topology.example("abilene")
    params = engine_params(topo, sim_time_s=2.0, ping_as_obs=1, auto_reset=0, seed=100)

    class Broken:
        def __init__(self, *a, **k):
            raise MemoryError("no oracle")

    monkeypatch.setattr(oracle_mod, "OracleSim", Broken)
    t0 = time.perf_counter()
    try:
        bench.cpu_baseline(topo, params, "table", sp_next_hop_table(topo), 1000, 1000, threads=2)
    except RuntimeError as e:
        assert "cpu_baseline worker failed" in str(e)
    else:
        raise AssertionError("cpu_baseline returned with a failing worker")
    assert time.perf_counter() - t0 < 30.0
