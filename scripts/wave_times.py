"""Diagnostic: how evenly the headline's waves finish (a -DPRISMA_WAVE_TIMES=1 build of the lite
translation unit: s_memrealtime at each wave's start and end, and its HW_ID / XCC_ID).

  ONLY=prisma_engine_lite.hip bash scripts/build_variant.sh wt -DPRISMA_WAVE_TIMES=1   # here
  python scripts/wave_times.py                                                        # GPU box
Prints the spread of wave end times over the last launch and how much of the kernel's SIMD time
the waves were resident."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PRISMA_LIB"] = os.path.join(ROOT, "prisma_amd", "_ablate", "libprisma_amd_wt.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from prisma_amd.config import engine_params  # noqa: E402
from prisma_amd.engine import PrismaEngine, load_library  # noqa: E402
from prisma_amd.policies import StackedQNet  # noqa: E402
from prisma_amd.topology import Topology  # noqa: E402

R = 4096
HOPS = int(sys.argv[sys.argv.index("--hops") + 1]) if "--hops" in sys.argv else 32768
topo = Topology.example("abilene")
eng = PrismaEngine(topo, engine_params(topo, sim_time_s=60.0, ping_as_obs=1, auto_reset=1, log_capacity=8192), R)
lib = load_library()
fn = lib.prisma_debug_wave_times_lite
fn.argtypes = [C.c_void_p, C.c_int]
table = StackedQNet(topo, "routing", seed=1234, device="cuda").argmin_table()
eng.reset(0)
buf = (C.c_ulonglong * (4 * R))()
for it in range(6):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    eng.run(table, HOPS)
    ev1.record()
    torch.cuda.synchronize()
    assert fn(buf, R) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(R, 4).astype(np.int64)
    t0, t1 = a[:, 0], a[:, 1]
    base = t0.min()
    s, e = (t0 - base) * 10e-3, (t1 - base) * 10e-3       # us (100 MHz)
    life = e - s
    span = e.max()
    hw = a[:, 2]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    xcc = a[:, 3] & 15
    key = ((xcc * 8 + se) * 16 + cu) * 4 + simd
    n_simd = len(np.unique(key))
    per = np.bincount(np.unique(key, return_inverse=True)[1])
    print(f"launch {it}: event {ev0.elapsed_time(ev1):.2f} ms, wave span {span / 1e3:.2f} ms; start max {s.max():.1f} us; "
          f"end min/p10/p50/p90/max {np.percentile(e, [0, 10, 50, 90, 100]).round(0).tolist()} us; "
          f"mean life / span {life.mean() / span:.3f}; SIMDs {n_simd}, waves per SIMD {np.bincount(per).nonzero()[0].tolist()}",
          flush=True)
# per-SIMD: the last wave's end against the SIMD's mean wave end (how long a SIMD runs short-handed)
order = np.argsort(key)
ks, ee = key[order], e[order]
bounds = np.flatnonzero(np.diff(ks)) + 1
groups = np.split(ee, bounds)
tail = np.array([g.max() - np.sort(g)[-2] if len(g) > 1 else 0.0 for g in groups])
print(f"per SIMD, last wave end - second-last: mean {tail.mean():.0f} us, p90 {np.percentile(tail, 90):.0f} us; "
      f"SIMD end spread (max over SIMDs of last end) - (min) {max(g.max() for g in groups) - min(g.max() for g in groups):.0f} us")
