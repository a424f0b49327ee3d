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
