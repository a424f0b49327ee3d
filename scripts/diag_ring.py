"""Diagnostic: error bits of both engines on one scenario (table policy)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from prisma_amd.config import engine_params
from prisma_amd.engine import PrismaEngine
from prisma_amd.topology import Topology, sp_next_hop_table

name, tm, lf, ping, seed, train = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
kinds = [int(k) for k in sys.argv[7].split(",")] if len(sys.argv) > 7 else [1, 2]
topo = Topology.example(name, tm, lf)
table = torch.from_numpy(sp_next_hop_table(topo)).cuda()
for kind in kinds:
    p = engine_params(topo, sim_time_s=15.0, ping_as_obs=ping, seed=seed, replica_base=5, train=train, engine=kind)
    eng = PrismaEngine(topo, p, 6)
    eng.reset(0)
    for step in range(25):
        eng.run(table, 100)
        c = eng.counters()
        print(kind, step, c["error"].tolist(), c["hops"].tolist(), flush=True)
        if c["error"].any():
            break
    print("engine", kind, "after", (step + 1) * 100, "hops: err", c["error"].tolist(), "hops", c["hops"].tolist(),
          "now", c["now_ns"].tolist())
    eng.close()
