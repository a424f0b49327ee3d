"""Diagnostic: memory-resident engine vs oracle, first differing record per replica."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import torch
from prisma_amd.config import engine_params
from prisma_amd.engine import PrismaEngine
from prisma_amd.topology import Topology, sp_next_hop_table
import oracle as O

name, tm, lf, ping, seed, train, H = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), \
    int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7])
kind = int(sys.argv[8]) if len(sys.argv) > 8 else 2
topo = Topology.example(name, tm, lf)
table = sp_next_hop_table(topo)
p = engine_params(topo, sim_time_s=15.0, ping_as_obs=ping, seed=seed, replica_base=5, train=train, engine=kind)
R = 6
eng = PrismaEngine(topo, p, R)
eng.reset(0)
eng.run(torch.from_numpy(table).cuda(), H)
torch.cuda.synchronize()
cnt = eng.counters()
log = eng.log_tensor().cpu().numpy()
for r in range(R):
    o = O.OracleSim(topo, p, replica=5 + r)
    o.enable_trace(True)
    o.run_table(table, H)
    ref = o.records()
    n = min(len(ref), int(cnt[r]["dec_count"]))
    got = eng.records(r, 0, n, log_host=log)
    d = next((i for i in range(n) if got[i].tobytes() != ref[i].tobytes()), None)
    print(f"replica {r}: err {int(cnt[r]['error'])} dec {int(cnt[r]['dec_count'])}/{len(ref)} first diff {d}", flush=True)
    if d is not None:
        print("  got", got[d])
        print("  ref", ref[d])
        print("  prev got", got[d - 1] if d else None)
        oc = o.counters()
        print("  counters got/ref", {k: (cnt[r][k], oc[k]) for k in ("events", "hops", "now_ns", "seq", "uid", "ov_injected", "ctrl_dropped")})
