"""N>1 path on CPU: world_size-2 gloo ranks shard replicas; the all-gathered per-replica
statistics equal a single-process run of every replica (the oracle stands in for the
per-rank engine: sharding is a pure function of global replica ids)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from prisma_amd.config import engine_params
from prisma_amd.dist import gather_replica_stats, replica_stats, shard
from prisma_amd.topology import Topology, sp_next_hop_table

TOTAL = 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _counters_for(base, n):
    import oracle as O
    topo = Topology.example("abilene")
    params = engine_params(topo, sim_time_s=2.0, ping_as_obs=1)
    out = []
    for r in range(base, base + n):
        s = O.OracleSim(topo, params, replica=r)
        s.run_table(sp_next_hop_table(topo), 10 ** 9)
        out.append(s.counters())
    return np.array(out)


def _worker(rank, world, port, q, total):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    base, n = shard(total, rank, world)
    res = gather_replica_stats(_counters_for(base, n), world, device=torch.device("cpu"))
    if rank == 0:
        q.put(res["stats"])
    dist.barrier()
    dist.destroy_process_group()


def test_shard_covers_all_replicas():
    for total in (4096, 16384, 7):
        for world in (1, 2, 4, 8) if total >= 8 else (1, 2, 7):
            spans = [shard(total, r, world) for r in range(world)]
            ids = [i for b, n in spans for i in range(b, b + n)]
            assert ids == list(range(total))


@pytest.mark.parametrize("total", [TOTAL + 1, TOTAL])      # 3 + 3 (equal) and 3 + 2 (unequal shards)
def test_gloo_world2_gather_equals_single_process(oracle_mod, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, total)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = replica_stats(_counters_for(0, total))
    assert np.array_equal(got, ref)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None, timeout=180):
    import subprocess
    import sys
    import time
    env = dict(os.environ, **(env_extra or {}))
    env.pop("WORLD_SIZE", None)
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT, env=env)
    return p, time.monotonic() - t0


def test_bench_launcher_rendezvous_gloo_world2():
    """bench.py --gpus 2 spawns its own ranks; with --rendezvous-only over gloo they initialise,
    all-gather their replica shards and rank 0 reports world size and the gathered count."""
    import json
    p, _ = _bench(["--gpus", "2", "--rendezvous-only", "--backend", "gloo", "--replicas", "100",
                   "--rank-deadline", "120"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert d["world_size"] == 2 and d["replicas_gathered"] == 200 and d["per_rank_replicas"] == [100, 100]


def test_bench_launcher_deadline_names_stalled_rank():
    """A rank that hangs (here: before its process-group init, so rank 0 waits in the rendezvous)
    makes the launcher terminate every rank at the deadline, name the stalled rank and exit 124."""
    deadline = 25.0
    p, wall = _bench(["--gpus", "2", "--rendezvous-only", "--backend", "gloo", "--rank-deadline", str(deadline)],
                     env_extra={"PRISMA_BENCH_STALL_RANK": "1"})
    assert p.returncode == 124, (p.returncode, p.stderr[-2000:])
    assert wall < deadline + 20.0
    assert "rank 1 (last stage: started)" in p.stderr and "rank 0 (last stage: started)" in p.stderr


@pytest.mark.parametrize("preset", ["config4", "config5"])
def test_bench_presets_rendezvous_gloo_world2(preset):
    """The 8-GPU presets resolve to BASELINE config 4 / 5 per GPU (weak scaling) on every rank:
    two gloo ranks rendezvous, all-gather their replica shards, and rank 0 reports the workload."""
    import json
    p, _ = _bench(["--gpus", "2", "--rendezvous-only", "--backend", "gloo", "--preset", preset,
                   "--rank-deadline", "120"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    w = d["workload"]
    assert d["world_size"] == 2 and w["preset"] == preset and w["policy"] == "dqn_buffer"
    if preset == "config4":
        assert w["topology"] == "geant" and w["ping_as_obs"] == 0 and w["replicas_per_gpu"] == 2048
        assert w["load_factors"] == [0.5, 0.75, 1.0, 1.25, 1.5, 1.75, 2.0]
        assert d["replicas_gathered"] == 4096
    else:
        assert w["topology"] == "er256" and w["ping_as_obs"] == 1 and w["replicas_per_gpu"] == 1024
        assert w["load_factors"] == [1.0] and d["replicas_gathered"] == 2048 and w["warmup"] == 4
