"""The C-ABI library loads without a GPU and exports exactly what include/prisma.h declares;
the ctypes mirrors of the ABI structs match the C layout."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from prisma_amd import engine
from prisma_amd.records import COUNTERS_DTYPE, record_dtype

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "prisma.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(prisma_\w+)\s*\(", txt, re.M)))


def test_header_declares_engine_exports():
    assert declared_functions() == sorted(engine.EXPORTS)


def test_library_loads_and_exports_every_symbol():
    if not os.path.exists(engine.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build_engine()
    lib = engine.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.prisma_abi_version() == engine.ABI_VERSION == 10
    out = subprocess.run(["nm", "-D", "--defined-only", engine.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (prisma_\w+)", out))
    assert set(declared_functions()) <= exported


def test_integration_recipe_matches_engine_sources():
    """INTEGRATION.md §1's hand-build recipe compiles exactly buildid.ENGINE_SOURCES with
    buildid.HIPCC_FLAGS, and the library those translation units link to leaves no prisma_*
    symbol undefined (one defined in a unit the recipe forgot would fail at dlopen)."""
    from prisma_amd import buildid
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    tu = re.search(r'^TU="([^"]+)"', txt, re.M)
    assert tu, "INTEGRATION.md lists no TU=... translation units"
    assert [f + ".hip" for f in tu.group(1).split()] == buildid.ENGINE_SOURCES
    flags = re.search(r'^F="([^"]+)"', txt, re.M).group(1).split()
    assert flags == buildid.HIPCC_FLAGS
    if not os.path.exists(engine.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build_engine()
    out = subprocess.run(["nm", "-D", "--undefined-only", engine.LIB_PATH], capture_output=True, text=True).stdout
    undefined = re.findall(r"\bU (\S*prisma\S*)", out)
    assert not undefined, undefined


def test_errors_are_status_codes_not_exits():
    lib = engine.load_library()
    h = C.c_void_p()
    assert lib.prisma_create(None, None, 1, 0, C.byref(h)) == -5          # PRISMA_ERR_ARG
    assert b"null" in lib.prisma_last_error()
    assert lib.prisma_reset(None, 0, None) == -5
    assert lib.prisma_step(None, None, None, None, None, None) == -5


C_PROBE = r'''
#include <stdio.h>
#include <stddef.h>
#include "prisma.h"
int main(void) {
  printf("%zu %zu %zu %zu\n", sizeof(prisma_topology_t), sizeof(prisma_params_t), sizeof(prisma_counters_t),
         sizeof(prisma_log_view_t));
  printf("%zu %zu %zu %zu %zu\n", offsetof(prisma_record_t, obs), offsetof(prisma_params_t, loss_penalty),
         offsetof(prisma_params_t, log_capacity), offsetof(prisma_counters_t, cost_sum),
         offsetof(prisma_counters_t, hops_total));
  printf("%zu %zu %zu\n", offsetof(prisma_params_t, engine), sizeof(prisma_plan_t), offsetof(prisma_plan_t, engine));
  printf("%zu %zu %zu %zu\n", offsetof(prisma_params_t, signaling_type), offsetof(prisma_params_t, big_signaling),
         offsetof(prisma_params_t, sync_step_s), offsetof(prisma_params_t, big_signaling_bytes));
  printf("%zu %zu\n", offsetof(prisma_params_t, rng_mode), offsetof(prisma_params_t, rng_stream_offset));
  printf("%zu %zu %zu\n", sizeof(prisma_kernel_info_t), offsetof(prisma_kernel_info_t, relay_ip),
         offsetof(prisma_kernel_info_t, relay_dec_bits));
  return 0;
}
'''


def test_ctypes_layouts_match_header():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "probe.c")
        exe = os.path.join(d, "probe")
        open(src, "w").write(C_PROBE)
        subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), src, "-o", exe])
        lines = subprocess.check_output([exe], text=True).split("\n")
    sizes = list(map(int, lines[0].split()))
    offs = list(map(int, lines[1].split()))
    assert sizes == [C.sizeof(engine._Topo), C.sizeof(engine._Params), COUNTERS_DTYPE.itemsize, C.sizeof(engine._LogView)]
    assert offs[0] == 32 == record_dtype(4).fields["obs"][1]
    assert offs[1] == engine._Params.loss_penalty.offset
    assert offs[2] == engine._Params.log_capacity.offset
    assert offs[3] == COUNTERS_DTYPE.fields["cost_sum"][1]
    assert offs[4] == COUNTERS_DTYPE.fields["hops_total"][1]
    eng = list(map(int, lines[2].split()))
    assert eng == [engine._Params.engine.offset, C.sizeof(engine._Plan), engine._Plan.engine.offset]
    sig = list(map(int, lines[3].split()))
    assert sig == [getattr(engine._Params, k).offset for k in
                   ("signaling_type", "big_signaling", "sync_step_s", "big_signaling_bytes")]
    rng = list(map(int, lines[4].split()))
    assert rng == [engine._Params.rng_mode.offset, engine._Params.rng_stream_offset.offset]
    ki = list(map(int, lines[5].split()))
    assert ki == [C.sizeof(engine._KernelInfo), engine._KernelInfo.relay_ip.offset,
                  engine._KernelInfo.relay_dec_bits.offset]


def test_engine_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from prisma_amd.config import engine_params
    from prisma_amd.topology import Topology
    t = Topology.example("abilene")
    with pytest.raises(engine.PrismaError):
        engine.PrismaEngine(t, engine_params(t), 4)


def test_plan_sizes_and_limits_without_a_device():
    """prisma_plan validates like prisma_create and reports the footprint."""
    from prisma_amd.config import engine_params
    from prisma_amd.topology import Topology
    ab = Topology.example("abilene")
    p = engine.plan(ab, engine_params(ab))
    assert p["obs_width"] == 4 and p["record_bytes"] == 48
    assert (p["flow_slots"], p["link_slots"]) == (2, 1)
    assert p["lds_bytes"] <= 10 * 1024                 # 16 replicas per CU (160 KiB LDS)
    assert p["ring_entries"] == 28 * 44 + 11 * 8
    ge = Topology.example("geant")
    g = engine.plan(ge, engine_params(ge))
    assert (g["flow_slots"], g["link_slots"]) == (8, 2) and g["obs_width"] == 8
    assert g["lds_bytes"] <= 20 * 1024                 # 8 replicas per CU
    # Abilene on GEANT: only the 40 GEANT links on some tunnel, ping-back or echo route get
    # state (compact_links), so 40 + 23 access links take one register slot per lane (4 waves
    # per SIMD), and with the FIFOs in HBM a replica's LDS fits 16 per CU (one round of 4 096)
    ag = Topology.example("abilene_on_geant")
    for train in (0, 1):
        a = engine.plan(ag, engine_params(ag, train=train))
        assert (a["flow_slots"], a["link_slots"]) == (2, 1)
        assert a["lds_bytes"] + 256 <= 10 * 1024
    # errors are status codes with a message, never exits
    with pytest.raises(engine.PrismaError, match="log_capacity"):
        engine.plan(ab, dict(engine_params(ab), log_capacity=1000))
    with pytest.raises(engine.PrismaError, match="sim_time_s"):
        engine.plan(ab, dict(engine_params(ab), sim_time_s=5000.0))
    ring = np.zeros((300, 300), dtype=int)
    for i in range(300):
        ring[i, (i + 1) % 300] = ring[(i + 1) % 300, i] = 1
    tm = np.zeros((300, 300), dtype=object)
    tm[0, 1] = 1000
    big = Topology.from_matrices(ring, tm)
    with pytest.raises(engine.PrismaError, match="n_nodes"):
        engine.plan(big, engine_params(big))


def test_plan_engine_selection():
    """Auto picks the register-resident engine when the topology fits it, the
    memory-resident one beyond (256 nodes, > 256 links); either can be forced
    where it applies."""
    from prisma_amd.config import engine_params
    from prisma_amd.topology import Topology
    ab = Topology.example("abilene")
    assert engine.plan(ab, engine_params(ab))["engine"] == engine.PRISMA_ENGINE_REGISTER
    m = engine.plan(ab, engine_params(ab, engine=engine.PRISMA_ENGINE_MEMORY))
    assert m["engine"] == engine.PRISMA_ENGINE_MEMORY and m["flow_slots"] == 0
    assert m["obs_width"] == 4 and m["record_bytes"] == 48
    # 28 + 11 links and 110 flows: 2 flow blocks (LDS minima), a top level of 1 link block + 1
    # flow group (its LDS image), and the 39 link leaf keys (8 B) and kinds (1 B), each region
    # 16-B aligned
    assert m["lds_state_bytes"] == 128 + 160 + 16 + 2 * 16 + 2 * 16 + 320 + 48
    n = 256
    ring = np.zeros((n, n), dtype=int)
    for i in range(n):
        for d in (1, 2):
            ring[i, (i + d) % n] = ring[(i + d) % n, i] = 1
    tm = np.full((n, n), 1000, dtype=object)
    big = Topology.from_matrices(ring, tm)
    p = engine.plan(big, engine_params(big))
    assert p["engine"] == engine.PRISMA_ENGINE_MEMORY
    with pytest.raises(engine.PrismaError, match="register-resident"):
        engine.plan(big, engine_params(big, engine=engine.PRISMA_ENGINE_REGISTER))
    # the memory-resident event tree's top level is one VGPR per lane: link blocks + flow groups
    # <= 64 (3 584 + 256 links = 60 link blocks: fits with one flow group, not with 16)
    dense = np.zeros((n, n), dtype=int)
    for i in range(n):
        for d in range(1, 8):
            dense[i, (i + d) % n] = dense[(i + d) % n, i] = 1
    one = np.zeros((n, n), dtype=object)
    one[0, 1] = 1000
    assert engine.plan(Topology.from_matrices(dense, one), engine_params(Topology.from_matrices(dense, one)))[
        "engine"] == engine.PRISMA_ENGINE_MEMORY
    full = Topology.from_matrices(dense, tm)
    with pytest.raises(engine.PrismaError, match="64 link blocks"):
        engine.plan(full, engine_params(full))
    ov = Topology.example("overlay_full_mesh_3n_abilene")
    with pytest.raises(engine.PrismaError, match="identity overlays"):
        engine.plan(ov, engine_params(ov, engine=engine.PRISMA_ENGINE_MEMORY))


def test_plan_tunnelled_overlay():
    """overlay_full_mesh_3n_abilene: 12 tunnels over 16 physical links, responder positions
    up to 2 (two-link tunnels), obs width 1 + 3 -> 4; a non-overlay flow is refused."""
    from prisma_amd.config import engine_params
    from prisma_amd.topology import Topology
    t = Topology.example("overlay_full_mesh_3n_abilene")
    p = engine.plan(t, engine_params(t))
    assert p["obs_width"] == 4 and p["record_bytes"] == 48 and p["link_slots"] == 1
    bad = Topology.example("overlay_full_mesh_3n_abilene")
    bad.flow_src = bad.flow_src.copy()
    bad.flow_src[0] = 1                                  # underlay-only node 1
    with pytest.raises(engine.PrismaError, match="overlay"):
        engine.plan(bad, engine_params(bad))


def test_plan_draw_cache_keeps_replicas_per_cu():
    """The flows' draw cache (engine_core.h flow_next: K - 1 cached 8-B send delays per flow) is laid
    out only where it costs no replica per CU (prisma_engine.hip build_layout): K = 3 on Abilene
    (110 flows: 1 760 B, 16 replicas of 9 728 B per 160-KiB CU as without it) and Abilene-on-GEANT,
    none on GEANT (506 flows at 8 replicas per CU), none with ns-3 streams (their state ends the
    image) and none on the memory-resident engine."""
    from prisma_amd.config import engine_params
    from prisma_amd.topology import Topology
    per_cu = lambda b: min(16, (160 * 1024) // b)
    ab = Topology.example("abilene")
    p = engine.plan(ab, engine_params(ab))
    assert p["lds_bytes"] == 7968 + 2 * 8 * 110 and per_cu(p["lds_bytes"]) == per_cu(7968) == 16
    q = engine.plan(ab, engine_params(ab, rng="ns3"))
    assert q["lds_state_bytes"] == 7840 + 112                      # no cache; the ns-3 stream state instead
    m = engine.plan(ab, engine_params(ab, engine=engine.PRISMA_ENGINE_MEMORY))
    assert m["lds_state_bytes"] == 128 + 160 + 16 + 2 * 16 + 2 * 16 + 320 + 48
    ge = Topology.example("geant")
    assert engine.plan(ge, engine_params(ge))["lds_bytes"] == 20400
    aog = Topology.example("abilene_on_geant")
    assert engine.plan(aog, engine_params(aog))["lds_bytes"] == 7232 + 2 * 8 * 110
