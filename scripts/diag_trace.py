"""Diagnostic: event trace of the memory-resident engine vs the oracle's (first divergence).

  python scripts/diag_trace.py build          # here: prisma_amd/_ablate/libprisma_amd_trace.so
  python scripts/diag_trace.py run geant 1 1.5 0 3 1 1400   # GPU box (name tm lf ping seed train hops)
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "prisma_amd", "_ablate", "libprisma_amd_trace.so")
CSRC = os.path.join(ROOT, "prisma_amd", "csrc")

if sys.argv[1] == "build":
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    objs = []
    sys.path.insert(0, ROOT)
    from prisma_amd import buildid
    for f in buildid.ENGINE_SOURCES:
        o = os.path.join(os.path.dirname(LIB), f + ".trace.o")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fPIC",
                               "-std=c++17", "-DPRISMA_TRACE=1", "-c", "-o", o, os.path.join(CSRC, f)])
        objs.append(o)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB, *objs])
    sys.exit(0)

os.environ["PRISMA_LIB"] = LIB
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import oracle as O  # noqa: E402
from prisma_amd.config import engine_params  # noqa: E402
from prisma_amd.engine import PrismaEngine, load_library  # noqa: E402
from prisma_amd.topology import Topology, sp_next_hop_table  # noqa: E402

name, tm, lf, ping, seed, train, H = sys.argv[2], int(sys.argv[3]), float(sys.argv[4]), int(sys.argv[5]), \
    int(sys.argv[6]), int(sys.argv[7]), int(sys.argv[8])
topo = Topology.example(name, tm, lf)
table = sp_next_hop_table(topo)
p = engine_params(topo, sim_time_s=15.0, ping_as_obs=ping, seed=seed, replica_base=5, train=train, engine=2)
R, CAP = 6, 200000
lib = load_library()
lib.prisma_debug_trace.argtypes = [C.c_void_p, C.c_uint]
buf = torch.zeros(8 * CAP * 3, dtype=torch.int64, device="cuda")
eng = PrismaEngine(topo, p, R)
assert lib.prisma_debug_trace(buf.data_ptr(), CAP) == 0
eng.reset(0)
eng.run(torch.from_numpy(table).cuda(), H)
torch.cuda.synchronize()
tr = buf.view(8, CAP, 3).cpu().numpy()
cnt = eng.counters()
KMAP = {0: 0, 1: 1, 2: 1, 3: 2, 4: 3}          # oracle EV_* -> engine K_* (ping, flow, complete, arrive)
for r in range(R):
    o = O.OracleSim(topo, p, replica=5 + r)
    o.enable_trace(True)
    o.run_table(table, H)
    ot = o.trace()                               # (t, seq, kind, id)
    ev = []
    for t, s, k, i in ot.tolist():
        k = KMAP[k]
        if k == 0 and ev and ev[-1][1] == 0 and ev[-1][0] == t:
            continue                              # one engine event per ping round
        ev.append((t, k, i if k else 0))
    n = int(cnt[r]["events"])
    got = [tuple(x) for x in tr[r, :n].tolist()]
    got = [(t, k, i if k else 0) for t, k, i in got]
    d = next((j for j in range(min(len(got), len(ev))) if got[j] != ev[j]), None)
    print(f"replica {r}: events got {len(got)} ref {len(ev)} first diff {d}", flush=True)
    if d is not None:
        for j in range(max(0, d - 6), d + 4):
            print("   ", j, "got", got[j] if j < len(got) else None, "ref", ev[j] if j < len(ev) else None)
