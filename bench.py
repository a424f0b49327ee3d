"""Headline benchmark: packet-hop transitions/s at 4096 Abilene replicas per MI355X.

Workload (BASELINE.json configs[1]): Abilene TM0, load_factor 1.0, DQ-Routing
agent (per-node DQN_routing_model restated in torch, random-init weights from
a fixed seed, greedy argmin -> exact [N, N] action table), pingAsObs=1,
train=0, simTime 60 s with auto-reset, 4096 replicas per GPU.
One step = refresh the policy table from the torch model (the agent's
forward pass over every (node, dst)) + one engine launch in which every
replica executes `--hops` forwarding decisions (enqueue or drop), logging
one decision record per data notification to HBM.

Run: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL); replicas are sharded
(weak scaling: replica ids rank*R .. rank*R+R-1), no data-path collective;
the per-replica episode statistics are all-gathered over RCCL at the end.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "packet-hop transitions/sec at 4096 Abilene replicas; achieved HBM GB/s"   # BASELINE.json
KERNEL_SOURCES = ["prisma_amd/csrc/prisma_engine.hip", "prisma_amd/csrc/prisma_engine_mem.hip",
                  "prisma_amd/csrc/engine_core.h", "prisma_amd/csrc/engine_layout.h", "prisma_amd/csrc/numerics.h"]
HBM_PEAK_GBS = 8000.0                    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=None,
                   help="untimed steps (default 2; er256: past the first simulated second, whose 65 251 "
                        "flow-start events are a transient of the episode)")
    p.add_argument("--replicas", type=int, default=None, help="replicas per GPU (default 4096; er256: 1024 = "
                                                             "BASELINE config 5's 8192 over 8 GPUs)")
    p.add_argument("--hops", type=int, default=8192, help="hops per replica per step (default 8192: one launch "
                   "of ~60 ms at the headline, so the per-step policy refresh and launch costs stay ~1 %%)")
    p.add_argument("--topology", default="abilene")
    p.add_argument("--tm", type=int, default=0)
    p.add_argument("--load-factor", type=float, default=1.0)
    p.add_argument("--ping-as-obs", type=int, default=1)
    p.add_argument("--policy", default="dq_routing", choices=["dq_routing", "dqn_buffer", "sp"],
                   help="in-kernel policy: DQ-routing argmin table (BASELINE configs[1]), DQN-buffer MLP, SP table")
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--cpu-hops", type=int, default=8000000, help="oracle hops per host thread (cpu_baseline)")
    a = p.parse_args()
    big = a.topology == "er256"
    if a.replicas is None:
        a.replicas = 1024 if big else 4096
    if a.warmup is None:
        a.warmup = 13 if big else 2          # er256: 13 x 8192 hops ~ 1.3 simulated seconds
    return a


def algorithmic_bytes(hops: int, deg_sum: int) -> int:
    """B_hop(u) = 85 + 12*deg(u) bytes, summed over executed hops."""
    return 85 * hops + 12 * deg_sum


def cpu_baseline(topo, params, table, hops_per_thread: int):
    """The C oracle (oracle/, kind 'port') on host threads: each thread runs one
    replica's episodes back to back (as auto-reset does) until it executed
    `hops_per_thread` hops, on the same scenario and DQ-routing table."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    cores = max(1, min(16, os.cpu_count() or 1))
    done = [0] * cores
    episodes = [0] * cores

    def work(i):
        ep = 0
        while done[i] < hops_per_thread:
            sim = O.OracleSim(topo, params, replica=100000 + i, episode=ep)
            done[i] += sim.run_table(table, hops_per_thread - done[i])   # ctypes releases the GIL
            sim.close()
            ep += 1
        episodes[i] = ep

    ths = [threading.Thread(target=work, args=(i,)) for i in range(cores)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    hops = int(sum(done))
    return {"value": hops / dt, "unit": "hops/s", "cores": cores, "kind": "port",
            "sample": f"{cores} host threads x {hops_per_thread} hops ({sum(episodes)} Abilene episodes of "
                      f"{params['sim_time_s']:g} s, same params and DQ-routing table), {hops} hops in {dt:.1f} s wall; "
                      f"the ns-3 reference path is not runnable here (SURVEY 8c)"}


def kernel_source_hash() -> str:
    import hashlib
    h = hashlib.sha1()
    for f in KERNEL_SOURCES:
        with open(os.path.join(ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]


def pmc_traffic(topology: str, replicas: int, hops: int):
    """HBM bytes per launch from the committed rocprofv3 --pmc passes (profiles/pmc_traffic.json),
    used only when they were collected on this workload with this exact kernel source."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        for e in d.get("entries", [d]):
            if (e.get("topology") == topology and int(e.get("replicas", -1)) == replicas
                    and int(e.get("hops", -1)) == hops and e.get("kernel_source") == kernel_source_hash()):
                return float(e["bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        pass
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from prisma_amd.config import engine_params
    from prisma_amd.dist import gather_replica_stats, shard
    from prisma_amd.engine import PrismaEngine
    from prisma_amd.policies import StackedQNet
    from prisma_amd.topology import Topology, sp_next_hop_table

    topo = Topology.example(args.topology, args.tm, args.load_factor)
    base, R = shard(args.replicas * world, rank, world)
    # the decision log must outlive one link crossing (queueing included): ER-256 makes
    # ~80 k decisions per simulated second against up to ~0.27 s per crossing
    log_cap = 65536 if topo.n_links > 256 else 8192
    params = engine_params(topo, sim_time_s=60.0, ping_as_obs=args.ping_as_obs, auto_reset=1,
                           replica_base=base, seed=100, log_capacity=log_cap)
    eng = PrismaEngine(topo, params, R, device=local)
    if args.policy == "dqn_buffer":
        agent = StackedQNet(topo, "buffer", seed=1234, device=dev)
        policy = agent.pack                       # packed weights, decided in-kernel per hop
    elif args.policy == "sp":
        sp = torch.from_numpy(sp_next_hop_table(topo)).to(dev)
        policy = lambda: sp
    else:
        agent = StackedQNet(topo, "routing", seed=1234, device=dev)
        policy = agent.argmin_table               # policy forward for every (node, dst)

    def step():
        eng.run(policy(), args.hops)

    eng.reset(0)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    c0 = eng.counters()
    stream = torch.cuda.current_stream()
    evs = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pol = policy()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.run(pol, args.hops)
        e1.record(stream)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    c1 = eng.counters()
    hops_local = int((c1["hops_total"] - c0["hops_total"]).sum())
    deg_avg = float(c1["hop_deg_sum"].sum()) / max(1, int(c1["hops"].sum()))   # mean deg(u) over hops
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    errors = int(c1["error"].max())
    stats = gather_replica_stats(c1, world)                    # RCCL all-gather (outside the timed region)
    hops_total = hops_local
    if world > 1:
        ht = torch.tensor([hops_local], dtype=torch.int64, device=dev)
        dist.all_reduce(ht)
        hops_total = int(ht.item())

    if rank == 0:
        # per-launch algorithmic bytes: the hops one launch executes on this rank x B_hop at their mean degree
        hops_per_launch = hops_local / args.steps
        alg_bytes = algorithmic_bytes(int(round(hops_per_launch)), int(round(hops_per_launch * deg_avg)))
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        traffic = pmc_traffic(args.topology, args.replicas, args.hops)
        metric = METRIC if (args.topology, args.replicas) == ("abilene", 4096) else \
            f"packet-hop transitions/sec at {args.replicas} {topo.name} replicas; achieved HBM GB/s"
        result = {
            "metric": metric,
            "value": hops_total / elapsed,
            "unit": "hops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": f"synthetic (Poisson traffic from the shipped {topo.name} TM{args.tm} x load_factor "
                    f"{args.load_factor}; {'random-init ' + args.policy + ' weights' if args.policy != 'sp' else 'SP table'})",
            "config": {
                "workload": f"{args.topology} tm{args.tm} lf{args.load_factor} {args.policy} greedy, "
                            f"{args.replicas} replicas/GPU x {args.hops} hops/step, pingAsObs={args.ping_as_obs}, "
                            f"simTime 60 s auto-reset",
                "topology": args.topology, "replicas_per_gpu": args.replicas, "hops_per_step": args.hops,
                "policy": args.policy, "parallelism": f"replica-sharded x{world}",
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": eng.kernel_name_mlp if args.policy == "dqn_buffer" else eng.kernel_name, "kernel_ms": kern_ms, "kernel_source": kernel_source_hash(),
                "alg_bytes_per_launch": alg_bytes, "hops_per_launch": hops_per_launch,
            },
            "errors": errors,
            "episodes_completed": stats["episodes_completed"],
        }
        if args.cpu_baseline and world == 1 and args.policy != "dqn_buffer":
            result["cpu_baseline"] = cpu_baseline(topo, dict(params, auto_reset=0),
                                                  policy().cpu().numpy(), args.cpu_hops)
        print(json.dumps(result), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
