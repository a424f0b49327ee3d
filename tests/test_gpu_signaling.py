"""Signalling on the HIP engine vs the CPU oracle (bit-exact), through the C-ABI: echo payloads
by signalling type (sim.cc:373-392) and the big-signalling NN-weight generators
(sim.cc:634-647, big-signaling-application.cc:224-309, big-signaling-packet-manager.cc:93-123).
The engine runs all generators in one event slot (engine_core.h on_bsig); the oracle keeps
one event per generator, as ns-3 does."""
import numpy as np
import pytest
import torch

from prisma_amd.config import engine_params
from prisma_amd.engine import PrismaEngine
from prisma_amd.topology import Topology, sp_next_hop_table

from test_gpu_parity import assert_counters_equal, run_table_both

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]


def sig_params(topo, **kw):
    # sim.cc's default NN size (69 segments per NN); engine_params defaults to the Python CLI's 512
    base = dict(sim_time_s=4.0, ping_as_obs=1, train=1, signaling_type="NN", big_signaling=1, replica_base=3,
                big_signaling_bytes=35328)
    base.update(kw)
    return engine_params(topo, **base)


@pytest.mark.parametrize("name,tm,lf,kw", [
    ("abilene", 0, 1.0, dict()),
    ("abilene", 1, 2.0, dict(sync_step_s=0.1, seed=7)),                 # 10x the segments, drops
    ("abilene", 0, 1.0, dict(ping_as_obs=0, big_signaling_bytes=4096, sync_step_s=0.05)),
    ("abilene", 2, 1.5, dict(signaling_type="target", big_signaling=0)),
    ("geant", 0, 1.0, dict(sync_step_s=0.5)),                           # per-node echo sizes, 8 flow slots
    ("overlay_full_mesh_3n_abilene", 0, 10.0, dict(sync_step_s=0.25)),  # tunnels
])
def test_signaling_table_parity(oracle_mod, name, tm, lf, kw):
    topo = Topology.example(name, tm, lf)
    params = sig_params(topo, **kw)
    cnt = run_table_both(oracle_mod, topo, params, 5, 2500, sp_next_hop_table(topo))
    assert int(cnt["bytes_signaling"].min()) > 0


def test_signaling_external_notify_parity(oracle_mod):
    """notify_dest + train + big signalling: echo and NN-segment notifications reach the caller
    with the obs fields of include/prisma.h."""
    topo = Topology.example("abilene", 0, 1.5)
    params = sig_params(topo, sim_time_s=2.0, notify_dest=1, sync_step_s=0.2)
    R = 4
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    orcs = [oracle_mod.OracleSim(topo, params, replica=params["replica_base"] + r) for r in range(R)]
    ref_obs = [o.step(-1) for o in orcs]
    obs, mask, node = eng.step(None)
    rng = np.random.default_rng(9)
    n_big = n_echo = 0
    for s in range(2500):
        g, m, nd = obs.cpu().numpy(), mask.cpu().numpy(), node.cpu().numpy()
        acts = np.zeros(R, dtype=np.int32)
        for r in range(R):
            assert (ref_obs[r] is None) == (m[r] == 0), (s, r)
            if ref_obs[r] is None:
                continue
            assert np.array_equal(ref_obs[r], g[r]), (s, r, g[r], ref_obs[r])
            assert nd[r] == orcs[r].pending_node()
            if g[r][0] == 1000:
                n_big += int(g[r][3] >> 16)
                n_echo += 1 - int(g[r][3] >> 16)
            acts[r] = rng.integers(0, topo.degrees[nd[r]])
        ref_obs = [orcs[r].step(int(acts[r])) if ref_obs[r] is not None else None for r in range(R)]
        obs, mask, node = eng.step(torch.from_numpy(acts).cuda())
    torch.cuda.synchronize()
    assert n_big > 0 and n_echo > 0
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in range(R):
        ref = orcs[r].records()
        assert eng.records(r, 0, len(ref), log_host=log).tobytes() == ref.tobytes()
        assert_counters_equal(cnt[r], orcs[r].counters(), r)
    eng.close()


def test_signaling_full_episode_properties():
    """A 60-s training episode of 512 Abilene replicas with big signalling: no engine fault, and
    the NN-segment traffic is what the generator schedule implies.  At the reference's defaults
    (35 328-B NN every second) a neighbour pair carries 299 kb/s of segments on 500 kb/s links,
    so control drops are the norm: every segment sent either arrives (540 B of signalling), is
    dropped (ctrl_dropped, with the pings and echoes dropped) or is in flight at the end."""
    from test_signaling import neighbour_flows
    topo = Topology.example("abilene")
    params = sig_params(topo, sim_time_s=60.0)
    R = 512
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    eng.run(torch.from_numpy(sp_next_hop_table(topo)).cuda(), 10 ** 8)
    torch.cuda.synchronize()
    cnt = eng.counters()
    assert int(cnt["error"].max()) == 0 and int(cnt["episode_over"].min()) == 1
    G = len(neighbour_flows(topo))
    sent = G * ((60 * 10 ** 9 - 1 - 100000) // 14492754)
    in_flight = G * 64
    sig = cnt["bytes_signaling"].astype(np.int64)
    assert np.all(sig + 540 * in_flight >= 540 * (sent - cnt["ctrl_dropped"].astype(np.int64)))
    assert np.all(cnt["ctrl_dropped"] > 0)
    eng.close()
