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
LIB = os.environ.get("PRISMA_TIMING_LIB", os.path.join(ROOT, "prisma_amd", "_ablate", "libprisma_amd_timing.so"))
NAMES = ["select", "arrive", "decision", "complete", "flow", "ping_round", "dec:send", "dec:record"]

if sys.argv[1] == "build":
    # `build mem`: only the memory-resident engine's translation unit with the timing probes,
    # the others from the in-tree objects of the last build_engine (same sources)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    sys.path.insert(0, ROOT)
    from prisma_amd import buildid
    # `build mem` / `build lite_mlp`: that translation unit alone with the probes
    only = {"mem": "prisma_engine_mem.hip", "lite_mlp": "prisma_engine_lite_mlp.hip",
            "lite": "prisma_engine_lite.hip"}.get(sys.argv[2]) if sys.argv[2:] else None
    objs, procs = [], []
    for f in buildid.ENGINE_SOURCES:
        if only and f != only:
            objs.append(os.path.join(ROOT, "prisma_amd", "csrc", os.path.splitext(f)[0] + ".o"))
            continue
        o = os.path.join(os.path.dirname(LIB), f + ".timing.o")
        # PRISMA_TIMING_FLAGS: extra -D flags (the timing build of a variant)
        extra = os.environ.get("PRISMA_TIMING_FLAGS", "").split()
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", *buildid.HIPCC_FLAGS, *extra, "-DPRISMA_TIMING=1", "-c", "-o", o,
                                       os.path.join(ROOT, "prisma_amd", "csrc", f)]))
        objs.append(o)
    if any(p.wait() != 0 for p in procs):
        sys.exit("hipcc failed")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB, *objs])
    for o in objs:
        if o.endswith(".timing.o"):
            os.remove(o)
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
HOPS = int(sys.argv[sys.argv.index("--hops") + 1]) if "--hops" in sys.argv else 2048
POLICY = sys.argv[sys.argv.index("--policy") + 1] if "--policy" in sys.argv else "dq_routing"
PAO = int(sys.argv[sys.argv.index("--ping-as-obs") + 1]) if "--ping-as-obs" in sys.argv else 1
topo = Topology.example(topo_name)
eng = PrismaEngine(topo, engine_params(topo, sim_time_s=60.0, ping_as_obs=PAO, auto_reset=1,
                                      log_capacity=65536 if topo.n_links > 256 else 8192), R)
lib = load_library()
# the kernels without the --train / notify_dest paths live in their own translation unit
# (one translation unit per instance set: step_kernel.h; kernel name <FS, LS, MLP, TUN, CTRL>)
_kname = eng.kernel_name_mlp if POLICY == "dqn_buffer" else eng.kernel_name
_targs = [a.strip() for a in _kname.split("<")[-1].rstrip(">").split(",")]
timing = lib.prisma_debug_timing_mem if eng.engine_kind == 2 else getattr(
    lib, {("false", "true"): "prisma_debug_timing", ("true", "true"): "prisma_debug_timing_mlp",
          ("false", "false"): "prisma_debug_timing_lite",
          ("true", "false"): "prisma_debug_timing_lite_mlp"}[(_targs[2], _targs[4])])
timing.argtypes = [C.c_void_p]
if POLICY == "dqn_buffer":
    table = StackedQNet(topo, "buffer", seed=1234, device="cuda").pack()
else:
    table = StackedQNet(topo, "routing", seed=1234, device="cuda").argmin_table()
eng.reset(0)
WARM = int(sys.argv[sys.argv.index("--warm") + 1]) if "--warm" in sys.argv else 1
for _ in range(WARM):
    eng.run(table, HOPS)
buf = (C.c_ulonglong * 64)()   # engine_core.h kTimingWords
timing(buf)
h0 = int(eng.counters()["hops_total"].sum())
for _ in range(4):
    eng.run(table, HOPS)
timing(buf)
hops = int(eng.counters()["hops_total"].sum()) - h0
tot = sum(buf[i] for i in range(8))
print(f"{topo_name} {POLICY} pao={PAO} R={R}: cycles/hop/wave = {tot / max(1, hops):.0f}")
for i in range(8):
    n = buf[8 + i] if i < 6 else buf[8 + 2]
    if n and buf[i]:
        print(f"  {NAMES[i]:11s} n/hop={n / hops:.3f}  cyc/call={buf[i] / n:8.0f}  share={buf[i] / tot:.3f}")
if buf[16]:
    nd = buf[8 + 2]
    for i, nm in enumerate(["mlp:ln+l1", "mlp:l2", "mlp:l3", "mlp:l4+argmin"]):
        print(f"  {nm:13s} cyc/decision={buf[16 + i] / max(1, nd):8.0f}")
if buf[20]:
    nf = buf[8 + 4]
    for i, nm in enumerate(["flow:record+block", "flow:send", "flow:draw", "flow:tree"]):
        print(f"  {nm:17s} cyc/flow={buf[20 + i] / max(1, nf):8.0f}")
# fine probes TP(i) (engine_core.h): cycles since the previous probe, per execution
PROBES_2 = ["arr:link+entry", "arr:record-issue+obs", "arr:wire-pop", "arr:prev-wait", "arr:data-rest",
            "arr:ctl-pop", "arr:ctl-rest", "dec:rows+src", "dec:send", "dec:record", "dec:counters",
            "cmp:link-get", "cmp:transmit", "cmp:put", "flow:draw+src", "flow:send"]
PROBES = PROBES_2 if os.environ.get("PRISMA_TP_SET") == "2" else (["arr:record", "arr:issue-prev+obs", "arr:wire-pop+tree", "arr:prev-wait", "arr:data-rest",
           "arr:ctl-pop", "arr:ctl-rest", "cmp:record", "cmp:ring", "cmp:transmit", "cmp:put+tree",
           "flowsend:admit", "flowsend:ring", "flowsend:transmit", "put:store", "put:tree"] if os.environ.get("PRISMA_TP_SET") == "1" else
          ["mlp:wait-arrival", "mlp:sum", "mlp:w3-issue", "mlp:var", "mlp:w4-issue", "mlp:den+xn",
          "mlp:l1-chunks", "mlp:l1-elu+store", "mlp:l2", "mlp:l3", "mlp:l4", "mlp:argmin",
          "dec:send", "dec:record+cnt", "probe14", "probe15"])
for i, nm in enumerate(PROBES):
    n = buf[40 + i]
    if n:
        print(f"  probe {nm:17s} n/hop={n / hops:.3f}  cyc/call={buf[24 + i] / n:8.0f}  share={buf[24 + i] / tot:.3f}")
