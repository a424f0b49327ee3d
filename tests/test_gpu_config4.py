"""BASELINE config 4 (GEANT 23 nodes, in-kernel DQN-buffer policy, load-factor sweep 0.5-2.0,
16 384 replicas over 8 GPUs = 2 048 per GPU) and the replica sharding of SURVEY 8(e), on the GPU,
bit-exact against the CPU oracle through the C-ABI.

Refs: load-scaled flow rates ceil(rate * lf) (/root/reference/prisma/ns3/sim.cc:623),
DQN_buffer_model (/root/reference/prisma/source/models.py:258-306), the per-port runs of
/root/reference/prisma/scripts/run_multiples_itc.py:40-46 (independent simulations = shards).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from prisma_amd.config import engine_params
from prisma_amd.engine import PrismaEngine
from prisma_amd.records import COUNTERS_DTYPE
from prisma_amd.topology import Topology
from parity_util import check_near_ties

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CNT_KEYS = [k for k in COUNTERS_DTYPE.names if k not in ("hops_total", "events_total")]
LOAD_FACTORS = [0.5, 0.75, 1.0, 1.25, 1.5, 1.75, 2.0]


def _weights(topo, seed):
    from prisma_amd.policies import StackedQNet
    return StackedQNet(topo, "buffer", seed=seed).pack()


def _check_mlp_replicas(oracle_mod, eng, topo, params, w, H, picks, launches=1, seed=None):
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    wh = w.cpu().numpy()
    net_cpu = None
    if seed is not None:
        from prisma_amd.policies import StackedQNet
        net_cpu = StackedQNet(topo, "buffer", seed=seed, device="cpu")
    for r in picks:
        o = oracle_mod.OracleSim(topo, params, replica=params["replica_base"] + r)
        o.run_mlp(wh, H)
        ref = o.records()
        assert cnt[r]["error"] == 0, (r, cnt[r]["error"])
        assert int(cnt[r]["dec_count"]) == len(ref)
        n = min(len(ref), eng.log_capacity)
        got = eng.records(r, len(ref) - n, n, log_host=log)
        assert got.tobytes() == ref[len(ref) - n:].tobytes(), f"replica {r}: records differ"
        oc = o.counters()
        bad = [(k, cnt[r][k], oc[k]) for k in CNT_KEYS if cnt[r][k] != oc[k]]
        assert not bad, f"replica {r}: counters differ {bad}"
        if net_cpu is not None:                  # torch fp32 argmin except at genuine near-ties
            check_near_ties(net_cpu, wh, o, got)
    return cnt


@pytest.mark.parametrize("ping", [0, 1])
@pytest.mark.parametrize("lf", LOAD_FACTORS)
def test_geant_dqn_buffer_load_factor_sweep(oracle_mod, lf, ping):
    """Config 4 at every load factor of the sweep, pingAsObs 0 and 1: records and counters
    bit-identical to the oracle over 2 launches (a pending decision carried across)."""
    topo = Topology.example("geant", 0, lf)
    seed = 31 + int(lf * 4)
    w = _weights(topo, seed=seed)
    params = engine_params(topo, sim_time_s=20.0, ping_as_obs=ping, seed=100 + int(lf * 100), replica_base=7)
    R, H = 3, 2400
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    eng.run(w, H // 2)
    eng.run(w, H // 2)
    cnt = _check_mlp_replicas(oracle_mod, eng, topo, params, w, H, range(R), seed=seed)
    if lf >= 1.5:
        assert cnt["ov_lost"].sum() > 0                    # heavy-load regime: FIFO drops happen
    eng.close()


@pytest.mark.parametrize("lf", [0.5, 2.0])
def test_geant_dqn_buffer_full_share(oracle_mod, lf):
    """The per-GPU share of config 4 (2 048 GEANT replicas, DQN-buffer, pingAsObs 0): invariants on
    every replica, 4 random replicas compared record by record with the oracle."""
    topo = Topology.example("geant", 0, lf)
    w = _weights(topo, seed=77)
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=0, replica_base=2048)
    R, H = 2048, 700
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    eng.run(w, H)
    rng = np.random.default_rng(int(lf * 10))
    picks = sorted(rng.choice(R, 4, replace=False).tolist())
    cnt = _check_mlp_replicas(oracle_mod, eng, topo, params, w, H, picks, seed=77)
    assert np.all(cnt["error"] == 0)
    assert np.all(cnt["hops"] == H)
    assert np.all(cnt["ov_injected"] >= cnt["ov_arrived"] + cnt["ov_lost"])
    assert np.all(cnt["cost_n"] == cnt["ov_arrived"] + cnt["ov_lost"])
    assert np.all(cnt["bytes_data"] == 540 * cnt["ov_injected"])
    assert len(np.unique(cnt["now_ns"])) > R // 2
    eng.close()


@pytest.mark.parametrize("name,policy", [("abilene", "dq_routing"), ("geant", "dqn_buffer"),
                                         ("er256", "sp")])
def test_sharded_engines_equal_unsharded(name, policy):
    """Replica sharding: one engine with 2R replicas and two engines with replica_base
    0 and R (what ranks 0 and 1 run) produce byte-identical decision logs and counters."""
    from prisma_amd.policies import StackedQNet
    from prisma_amd.topology import sp_next_hop_table
    topo = Topology.example(name)
    if policy == "dq_routing":
        pol = StackedQNet(topo, "routing", seed=3).argmin_table()
    elif policy == "dqn_buffer":
        pol = StackedQNet(topo, "buffer", seed=3).pack()
    else:
        pol = torch.from_numpy(sp_next_hop_table(topo)).cuda()
    R = 8 if name != "er256" else 4
    H = 1500 if name != "er256" else 800
    cap = 65536 if topo.n_links > 256 else 8192

    def run(base, n):
        params = engine_params(topo, sim_time_s=60.0, ping_as_obs=1, replica_base=base, seed=100,
                               auto_reset=1, log_capacity=cap)
        eng = PrismaEngine(topo, params, n)
        eng.reset(0)
        eng.run(pol, H)
        eng.run(pol, H)
        torch.cuda.synchronize()
        out = eng.counters(), eng.log_tensor().cpu().numpy()
        eng.close()
        return out

    c_all, l_all = run(0, 2 * R)
    c0, l0 = run(0, R)
    c1, l1 = run(R, R)
    assert c_all.tobytes() == np.concatenate([c0, c1]).tobytes()
    assert l_all.tobytes() == np.concatenate([l0, l1]).tobytes()
    assert np.all(c_all["error"] == 0) and np.all(c_all["hops_total"] == 2 * H)


def test_bench_two_ranks_same_device():
    """bench.py --gpus 2 starts its own two ranks (no outside launcher); --same-device puts both on
    cuda:0 over gloo, so the spawn / all-gather / max-over-ranks / JSON path runs on a 1-GPU box."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same-device", "--steps", "2",
           "--warmup", "1", "--replicas", "128", "--hops", "256", "--cpu-baseline", "0"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout                     # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["replicas_total"] == 256 and len(d["per_rank_hops_s"]) == 2
    assert d["errors"] == 0 and d["n_gpus"] == 1
    assert abs(d["value"] - sum(d["per_rank_hops_s"])) <= 1e-6 * d["value"]
    assert d["roofline"]["build_id"]


@pytest.mark.parametrize("mode", ["rendezvous", "bench"])
def test_bench_rccl_one_rank_group(mode):
    """The RCCL path on a one-GPU box: a one-rank nccl process group initialises (device-bound,
    as bench.py's ranks do) and runs the bench's collectives -- the barriers, the max-over-ranks
    all-reduce and the replica-statistics all-gather of prisma_amd/dist.py (--force-dist)."""
    if mode == "rendezvous":
        args = ["--rendezvous-only", "--backend", "nccl", "--replicas", "64"]
    else:
        args = ["--force-dist", "--backend", "nccl", "--steps", "2", "--warmup", "1", "--replicas", "128",
                "--hops", "256", "--cpu-baseline", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    if mode == "rendezvous":
        assert d["backend"] == "nccl" and d["world_size"] == 1 and d["replicas_gathered"] == 64
    else:
        assert d["dist"] == {"world_size": 1, "backend": "nccl", "replicas_gathered": 128}
        assert d["errors"] == 0 and d["replicas_total"] == 128


@pytest.mark.parametrize("preset,lfs", [("config4", "0.5,2.0"), ("config5", None)])
def test_bench_presets_two_ranks_same_device(preset, lfs):
    """The 8-GPU presets as one command each (bench.py --preset config4 / config5), rehearsed with
    two ranks on cuda:0 at a small replica count: config 4 prints one line per load factor of its
    sweep, config 5 runs the ER-256 DQN-buffer workload on the memory-resident engine."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same-device", "--preset", preset,
           "--steps", "2", "--warmup", "1", "--replicas", "16", "--hops", "256", "--cpu-baseline", "0"]
    if lfs:
        cmd += ["--load-factors", lfs]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    want = [float(x) for x in lfs.split(",")] if lfs else [1.0]
    assert [d["config"]["load_factor"] for d in lines] == want
    for d in lines:
        assert d["config"]["preset"] == preset and d["replicas_total"] == 32 and d["errors"] == 0
        assert d["config"]["policy"] == "dqn_buffer" and d["config"]["replicas_per_gpu"] == 16
        assert d["config"]["topology"] == ("geant" if preset == "config4" else "er256")
        assert "mem_step" in d["roofline"]["kernel"] if preset == "config5" else "step_kernel_t<8" in d["roofline"]["kernel"]
