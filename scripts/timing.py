"""Diagnostic: per-phase cycle totals of the step kernel (s_memtime build).

  python scripts/timing.py build            # here: builds prisma_amd/_ablate/libprisma_amd_timing.so
  python scripts/timing.py run [--topology abilene]   # GPU box
Results are per executed phase, averaged over waves (cycles of the shader clock).
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "prisma_amd", "_ablate", "libprisma_amd_timing.so")
NAMES = ["select", "arrive", "decision", "complete", "flow", "ping_round", "dec:send", "dec:record"]

if sys.argv[1] == "build":
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fPIC",
                           "-shared", "-std=c++17", "-DPRISMA_TIMING=1", "-o", LIB,
                           os.path.join(ROOT, "prisma_amd", "csrc", "prisma_engine.hip")])
    sys.exit(0)

os.environ["PRISMA_LIB"] = LIB
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from prisma_amd.config import engine_params  # noqa: E402
from prisma_amd.engine import PrismaEngine, load_library  # noqa: E402
from prisma_amd.policies import StackedQNet  # noqa: E402
from prisma_amd.topology import Topology  # noqa: E402

topo_name = sys.argv[sys.argv.index("--topology") + 1] if "--topology" in sys.argv else "abilene"
R = int(sys.argv[sys.argv.index("--replicas") + 1]) if "--replicas" in sys.argv else 4096
topo = Topology.example(topo_name)
eng = PrismaEngine(topo, engine_params(topo, sim_time_s=60.0, ping_as_obs=1, auto_reset=1), R)
lib = load_library()
lib.prisma_debug_timing.argtypes = [C.c_void_p]
table = StackedQNet(topo, "routing", seed=1234).argmin_table()
eng.reset(0)
eng.run(table, 2048)
buf = (C.c_ulonglong * 16)()
lib.prisma_debug_timing(buf)
h0 = int(eng.counters()["hops_total"].sum())
for _ in range(4):
    eng.run(table, 2048)
lib.prisma_debug_timing(buf)
hops = int(eng.counters()["hops_total"].sum()) - h0
tot = sum(buf[i] for i in range(8))
print(f"{topo_name} R={R}: cycles/hop/wave = {tot / max(1, hops):.0f}")
for i in range(8):
    n = buf[8 + i] if i < 6 else buf[8 + 2]
    if n and buf[i]:
        print(f"  {NAMES[i]:11s} n/hop={n / hops:.3f}  cyc/call={buf[i] / n:8.0f}  share={buf[i] / tot:.3f}")
