"""ns-3 random streams (PRISMA_RNG_NS3): the oracle's RngStream restatement (MRG32k3a,
L'Ecuyer, Simard, Chen, Kelton 2002, as ns-3's rng-stream.cc uses it) against the jump matrices
the paper publishes, against an independent integer restatement here, and the stream assignment
of sim.cc / poisson-application.cc replayed over the oracle's event trace.  The engine's HIP path
is compared with the oracle in tests/test_gpu_ns3_rng.py.

Parity with ns-3 itself stays unpinned (ns-3 is absent): the number of RandomVariable objects
ns-3 creates before sim.cc's flow loop is version-dependent, hence the rng_stream_offset
parameter."""
import ctypes as C

import numpy as np
import pytest

from prisma_amd.config import engine_params
from prisma_amd.topology import Topology, sp_next_hop_table

EV_START, EV_SEND = 1, 2
M1, M2 = 4294967087, 4294944443

# RngStream.c / ns-3 rng-stream.cc: A1p127, A2p127, A1p76, A2p76 (L'Ecuyer et al. 2002)
A1P127 = [2427906178, 3580155704, 949770784, 226153695, 1230515664, 3580155704, 1988835001, 986791581, 1230515664]
A2P127 = [1464411153, 277697599, 1610723613, 32183930, 1464411153, 1022607788, 2824425944, 32183930, 2093834863]
A1P76 = [82758667, 1871391091, 4127413238, 3672831523, 69195019, 1871391091, 3672091415, 3528743235, 69195019]
A2P76 = [1511326704, 3759209742, 1610795712, 4292754251, 1511326704, 3889917532, 3859662829, 4292754251, 3708466080]


def _pow2(L, e):
    out = (C.c_uint64 * 18)()
    L.or_mrg_pow2(e, out)
    return list(out)


def test_jump_matrices_match_published(oracle_mod):
    L = oracle_mod.lib()
    assert _pow2(L, 127) == A1P127 + A2P127
    assert _pow2(L, 76) == A1P76 + A2P76


# ---- independent restatement: Python integers, matrix powers with arbitrary exponents
A1 = [[0, 1, 0], [0, 0, 1], [M1 - 810728, 1403580, 0]]
A2 = [[0, 1, 0], [0, 0, 1], [M2 - 1370589, 0, 527612]]


def _mm(X, Y, m):
    return [[sum(X[i][k] * Y[k][j] for k in range(3)) % m for j in range(3)] for i in range(3)]


def _mpow(A, n, m):
    R = [[int(i == j) for j in range(3)] for i in range(3)]
    while n:
        if n & 1:
            R = _mm(R, A, m)
        A = _mm(A, A, m)
        n >>= 1
    return R


def _mv(A, v, m):
    return [sum(A[i][k] * v[k] for k in range(3)) % m for i in range(3)]


def py_first_u01(seed, stream, run):
    """RngStream(seed, stream, run).RandU01(): state = A^(stream 2^127 + run 2^76) (seed x 6)."""
    n = stream * 2 ** 127 + run * 2 ** 76
    s1 = _mv(_mpow(A1, n, M1), [seed] * 3, M1)
    s2 = _mv(_mpow(A2, n, M2), [seed] * 3, M2)
    p1 = (1403580 * s1[1] - 810728 * s1[0]) % M1
    p2 = (527612 * s2[2] - 1370589 * s2[0]) % M2
    return ((p1 - p2) if p1 > p2 else (p1 - p2 + M1)) * 2.328306549295727688e-10


@pytest.mark.parametrize("seed,stream,run", [(12345, 0, 0), (1, 0, 1), (100, 3, 100), (100, 65280, 100),
                                             (4294944442, 123456789, 7), (7, 2 ** 40 + 5, 2 ** 31 + 3)])
def test_first_values_match_integer_restatement(oracle_mod, seed, stream, run):
    assert oracle_mod.lib().or_mrg_first_u01(seed, stream, run) == py_first_u01(seed, stream, run)


def test_package_first_output():
    """The package's first RandU01 from seed 12345 in all six words (stream 0, no substream)."""
    assert py_first_u01(12345, 0, 0) == pytest.approx(0.12701112204657714, abs=1e-16)


def _ns3_params(topo, **kw):
    base = dict(sim_time_s=3.0, ping_as_obs=0, rng="ns3", seed=100)
    base.update(kw)
    return engine_params(topo, **base)


@pytest.mark.parametrize("offset,replica", [(0, 0), (37, 5)])
def test_oracle_stream_assignment_replayed(oracle_mod, offset, replica):
    """sim.cc:610-620 creates one UniformRandomVariable per flow, in flow order, for its start
    offset; then every StartSending creates the packet's ExponentialRandomVariable
    (poisson-application.cc:281) and every SendPacket a UniformRandomVariable (:311) before
    it.  Replaying that order over the oracle's event trace gives every start and send time."""
    topo = Topology.example("abilene")
    p = _ns3_params(topo, rng_stream_offset=offset)
    s = oracle_mod.OracleSim(topo, p, replica=replica)
    s.enable_trace(True)
    s.run_table(sp_next_hop_table(topo), 10 ** 9)
    tr = s.trace()
    L = oracle_mod.lib()
    seed = p["seed"] + replica
    F = topo.n_flows
    starts = {int(r[3]): int(r[0]) for r in tr if r[2] == EV_START}
    assert len(starts) == F
    for f in range(F):
        u = py_first_u01(seed, offset + f, seed) if f < 3 else L.or_mrg_first_u01(seed, offset + f, seed)
        assert starts[f] == L.or_seconds_to_ns(0.0001 + u)
    nxt = offset + F
    mean = (p["packet_size"] * 8) / np.asarray(topo.flow_rate_bps, dtype=np.float64)
    due = {}
    for t, _, kind, f in tr:
        if kind not in (EV_START, EV_SEND):
            continue
        f = int(f)
        if f in due:
            assert t == due.pop(f)
        if kind == EV_SEND:
            nxt += 1                                  # SendPacket's UniformRandomVariable
        u = L.or_mrg_first_u01(seed, nxt, seed)       # ScheduleNextTx's ExponentialRandomVariable
        nxt += 1
        due[f] = int(t) + L.or_seconds_to_ns(-mean[f] * L.or_det_log(u))
    assert len(due) == F


def test_ns3_streams_repeat_every_episode(oracle_mod):
    """run_ns3.py restarts ns-3 with the same --simSeed every episode: the same traffic."""
    topo = Topology.example("abilene")
    table = sp_next_hop_table(topo)
    recs = {}
    for rng in ("ns3", "philox"):
        for ep in (0, 1):
            s = oracle_mod.OracleSim(topo, _ns3_params(topo, rng=rng), replica=2, episode=ep)
            s.run_table(table, 3000)
            r = s.records().copy()
            r["episode"] = 0                          # (the record's episode field)
            recs[rng, ep] = r
    assert recs["ns3", 0].tobytes() == recs["ns3", 1].tobytes()
    assert recs["philox", 0].tobytes() != recs["philox", 1].tobytes()
    assert recs["ns3", 0].tobytes() != recs["philox", 0].tobytes()


def test_plan_accepts_ns3_streams():
    from prisma_amd.engine import PrismaError, plan
    topo = Topology.example("abilene")
    assert plan(topo, _ns3_params(topo))["engine"] >= 1
    with pytest.raises(PrismaError, match="rng_mode"):
        plan(topo, dict(_ns3_params(topo), rng_mode=2))
