"""Headline benchmark: packet-hop transitions/s at 4096 Abilene replicas per MI355X.

Workload (BASELINE.json configs[1]): Abilene TM0, load_factor 1.0, DQ-Routing
agent (per-node DQN_routing_model restated in torch, random-init weights from
a fixed seed, greedy argmin -> exact [N, N] action table), pingAsObs=1,
train=0, simTime 60 s with auto-reset, 4096 replicas per GPU.
One step = refresh the policy table from the torch model (the agent's
forward pass over every (node, dst)) + one engine launch in which every
replica executes `--hops` forwarding decisions (enqueue or drop), logging
one decision record per data notification to HBM.

Run: python bench.py [--gpus N --steps K --warmup W] [--preset configK].  N > 1: one process per
GPU over RCCL, either under torch.distributed.run (RANK/WORLD_SIZE set) or
launched by this script itself (it starts N child ranks before anything
touches the GPU, then waits for them).  Replicas are sharded (weak scaling:
replica ids rank*R .. rank*R+R-1), no data-path collective; the per-replica
episode statistics are all-gathered over RCCL at the end.  --same-device runs
the N ranks on cuda:0 over gloo (a rehearsal of the spawn/gather/JSON path on
a one-GPU box; its value is not a scaling figure).

--preset config1 ... config5 selects one BASELINE.json configuration per GPU (replicas per GPU
fixed, weak scaling: config 4's 16 384 GEANT replicas and config 5's 8 192 ER-256 replicas are
2 048 and 1 024 per GPU at N = 8), config4 with its load-factor sweep: one JSON line per load
factor (--load-factors overrides the sweep).  Explicit flags override a preset's values.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "packet-hop transitions/sec at 4096 Abilene replicas; achieved HBM GB/s"   # BASELINE.json
HBM_PEAK_GBS = 8000.0                    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


# BASELINE.json configs, per GPU (weak scaling): explicit flags override these values
PRESETS = {
    "config1": dict(topology="abilene", policy="sp", replicas=1, ping_as_obs=1, hops=2048),
    "config2": dict(topology="abilene", policy="dq_routing", replicas=4096, ping_as_obs=1, hops=32768),
    "config3": dict(topology="abilene_on_geant", policy="dqn_buffer", replicas=4096, ping_as_obs=1, hops=8192),
    "config4": dict(topology="geant", policy="dqn_buffer", replicas=2048, ping_as_obs=0, hops=8192,
                    load_factors="0.5,0.75,1.0,1.25,1.5,1.75,2.0"),
    # (4 warm-up steps x 32 768 hops: past the first simulated second's 65 251 flow starts)
    "config5": dict(topology="er256", policy="dqn_buffer", replicas=1024, ping_as_obs=1, hops=32768, warmup=4),
}
# hops per replica per step in the BASELINE presets, each the better of 8 192 and 32 768 measured on
# build efc0e356bcf3: 32 768 for config2 (also a run with no workload flags: +0.9 %, and a default run
# keeps the GPU busy for seconds, not the ~1 s of round 4 against ~17 s of CPU baseline) and config5
# (+3.8 %: the launch's tail -- the last replica to finish its hops ends it, at one wave per SIMD --
# amortised); 8 192 for config3 and config4 (-2.5 % / -1 % at 32 768) and ad-hoc workloads
DEFAULTS = dict(topology="abilene", policy="dq_routing", ping_as_obs=1, hops=8192, load_factor=1.0)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--preset", choices=sorted(PRESETS), default=None,
                   help="a BASELINE.json configuration (per GPU); explicit flags override its values")
    p.add_argument("--load-factors", default=None,
                   help="comma-separated load factors: one measurement and JSON line each (config 4's sweep)")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=None,
                   help="untimed steps (default 2; er256: past the first simulated second, whose 65 251 "
                        "flow-start events are a transient of the episode: 13 x 8192 hops, the config5 preset "
                        "4 x 32768)")
    p.add_argument("--replicas", type=int, default=None, help="replicas per GPU (default 4096; er256: 1024 = "
                                                             "BASELINE config 5's 8192 over 8 GPUs)")
    p.add_argument("--hops", type=int, default=None, help="hops per replica per step (default 32768 at the "
                   "headline: one launch of ~0.16 s, so the per-step policy refresh and launch costs stay well "
                   "under 1 %%; 8192 in the config3-5 presets)")
    p.add_argument("--topology", default=None)
    p.add_argument("--tm", type=int, default=0)
    p.add_argument("--load-factor", type=float, default=None)
    p.add_argument("--ping-as-obs", type=int, default=None)
    p.add_argument("--policy", default=None, choices=["dq_routing", "dqn_buffer", "sp"],
                   help="in-kernel policy: DQ-routing argmin table (BASELINE configs[1]), DQN-buffer MLP, SP table")
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--cpu-hops", type=int, default=None,
                   help="oracle hops per host thread (cpu_baseline; default 8e6 with a table policy, 1.2e6 with "
                        "the DQN-buffer MLP: ~10-20 s of host work either way)")
    p.add_argument("--cpu-hops-1core", type=int, default=None, help="oracle hops of the single-thread pass "
                   "(default: half of --cpu-hops)")
    p.add_argument("--same-device", action="store_true",
                   help="N ranks share cuda:0 over gloo (rehearsal of the N-rank path on one GPU)")
    p.add_argument("--rank-deadline", type=float, default=None,
                   help="seconds the N-rank launcher waits for every rank to finish before it terminates them "
                        "all and names the ranks that had not reported (default: init allowance + a per-step "
                        "bound x (warmup + steps) + the CPU-baseline allowance)")
    p.add_argument("--rendezvous-only", action="store_true",
                   help="ranks only initialise torch.distributed and all-gather their replica counts (no GPU "
                        "work unless the backend is nccl): a check of the N-rank plumbing")
    p.add_argument("--force-dist", action="store_true",
                   help="initialise torch.distributed and run the collectives even with one rank (exercises "
                        "RCCL init and the all-gather on a one-GPU box)")
    p.add_argument("--backend", default=None, choices=["nccl", "gloo"],
                   help="process-group backend (default: nccl = RCCL; gloo with --same-device)")
    a = p.parse_args(argv)
    if a.preset is None and a.topology is None and a.policy is None and a.replicas is None:
        a.preset = "config2"                     # the driver's default run: the headline
    for k, v in (PRESETS[a.preset] if a.preset else {}).items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    for k, v in DEFAULTS.items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    big = a.topology == "er256"
    if a.replicas is None:
        a.replicas = 1024 if big else 4096
    if a.warmup is None:
        a.warmup = 13 if big else 2          # er256: 13 x 8192 hops ~ 1.3 simulated seconds
    a.lfs = ([float(x) for x in a.load_factors.split(",") if x.strip()] if a.load_factors
             else [float(a.load_factor)])
    mlp = a.policy == "dqn_buffer"
    if a.cpu_hops is None:
        a.cpu_hops = 1200000 if mlp else 8000000
    if a.cpu_hops_1core is None:
        a.cpu_hops_1core = a.cpu_hops // 2
    return a


def algorithmic_bytes(hops: int, deg_sum: int) -> int:
    """B_hop(u) = 85 + 12*deg(u) bytes, summed over executed hops."""
    return 85 * hops + 12 * deg_sum


def host_cpus():
    """(threads to use, description): the CPUs this process may actually run on — its affinity
    set, capped by a cgroup CPU quota (on the GPU box `nproc` shows the whole machine, while the
    job's quota is its share) — plus nproc and the CPU model name."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    use = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return use, {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "model": model}


def cpu_baseline(topo, params, kind: str, policy, hops_per_thread: int, hops_1core: int, threads: int = None,
                 warm_hops: int = 0, workload: str = ""):
    """The C oracle (oracle/, kind 'port') on the host: one replica per thread over every CPU this
    job may use (at most `threads`: config 1 has one replica), each running back-to-back episodes,
    as auto-reset does, until it executed `hops_per_thread` hops, and a single-thread pass for the
    per-core figure.  kind "table": the [N, N] action table (SP / DQ-routing); "mlp": the packed
    DQN-buffer weights, decided by the oracle's fixed-order fp32 restatement of the in-kernel MLP
    (models.py:258-306).  warm_hops: executed untimed first on every thread (the GPU line's warm-up
    past ER-256's flow-start transient)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    avail, host = host_cpus()
    cores = avail if threads is None else max(1, min(avail, int(threads)))
    pol = np.ascontiguousarray(policy)

    def timed(n_threads, hops_each):
        done = [0] * n_threads
        episodes = [0] * n_threads
        sims = [None] * n_threads
        bar = threading.Barrier(n_threads + 1)

        def run(sim, n):
            return sim.run_table(pol, n) if kind == "table" else sim.run_mlp(pol, n)

        errs = []

        def work(i):
            try:
                body(i)
            except BaseException as exc:            # a failed worker releases the others
                errs.append(exc)
                bar.abort()

        def body(i):
            ep = 0
            sims[i] = O.OracleSim(topo, params, replica=100000 + i, episode=ep)
            w = 0
            while w < warm_hops:                    # untimed (ends inside the first episode here)
                got = run(sims[i], warm_hops - w)
                w += got
                if w < warm_hops:
                    ep += 1
                    sims[i].close()
                    sims[i] = O.OracleSim(topo, params, replica=100000 + i, episode=ep)
            bar.wait()
            while done[i] < hops_each:
                done[i] += run(sims[i], hops_each - done[i])   # ctypes releases the GIL
                if done[i] < hops_each:
                    sims[i].close()
                    ep += 1
                    sims[i] = O.OracleSim(topo, params, replica=100000 + i, episode=ep)
            sims[i].close()
            episodes[i] = ep + 1
            bar.wait()

        ths = [threading.Thread(target=work, args=(i,)) for i in range(n_threads)]
        for t in ths:
            t.start()
        try:
            bar.wait()                              # every thread built (and warmed) its replica
            t0 = time.perf_counter()
            bar.wait()
            dt = time.perf_counter() - t0
        except threading.BrokenBarrierError:
            dt = None
        for t in ths:
            t.join()
        if errs or dt is None:
            raise RuntimeError(f"cpu_baseline worker failed: {errs[0] if errs else 'barrier broken'}")
        return int(sum(done)), int(sum(episodes)), dt

    h1, e1, d1 = timed(1, hops_1core)
    hn, en, dn = timed(cores, hops_per_thread)
    what = "DQN-buffer MLP (the oracle's fixed-order fp32 restatement)" if kind == "mlp" else "action table"
    warm = f", each thread first {warm_hops} hops untimed" if warm_hops else ""
    return {"value": hn / dn, "unit": "hops/s", "cores": cores, "kind": "port",
            "value_1core": h1 / d1, "host": host, "workload": workload,
            "sample": f"{cores} host threads x {hops_per_thread} hops ({en} {topo.name} episodes of "
                      f"{params['sim_time_s']:g} s, same params and {what}{warm}), {hn} hops in {dn:.1f} s wall; "
                      f"1 thread x {hops_1core} hops in {d1:.1f} s; {cores} = the CPUs this job may use "
                      f"(affinity {host['affinity']}, cgroup quota {host['cgroup_quota_cpus']}, nproc {host['nproc']})"
                      f"{', capped at the replica count' if cores < avail else ''}; "
                      f"the ns-3 reference path is not runnable here (SURVEY 8c)"}


def _profile_entry(name: str, topology: str, replicas: int, hops: int, build: str):
    """The entry of a committed profile table (profiles/<name>.json) for this workload, used only
    when it was collected with this exact library build (prisma_build_id())."""
    try:
        with open(os.path.join(ROOT, "profiles", name)) as fh:
            d = json.load(fh)
        for e in d.get("entries", []):
            if (e.get("topology") == topology and int(e.get("replicas", -1)) == replicas
                    and int(e.get("hops", -1)) == hops and e.get("build_id") == build):
                return e
    except (OSError, ValueError, KeyError):
        pass
    return None


def pmc_traffic(topology: str, replicas: int, hops: int, build: str):
    """HBM bytes per launch from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes."""
    e = _profile_entry("pmc_traffic.json", topology, replicas, hops, build)
    return None if e is None else float(e["bytes_per_launch"])


def issue_roofline(topology: str, replicas: int, hops: int, build: str):
    """Instruction-issue utilisation of the step kernel from the committed SQ counter passes
    (profiles/pmc_sq.json, scripts/pmc_to_json.py): scalar-ALU instructions per CU-cycle (one
    scalar unit per CU issues at most one per cycle) and wave64 VALU instructions per SIMD-cycle
    (a SIMD-32 issues one every 2 cycles: peak 0.5), with the per-hop instruction counts."""
    e = _profile_entry("pmc_sq.json", topology, replicas, hops, build)
    if e is None:
        return None
    keys = ("salu_busy", "valu_busy", "salu_per_hop", "valu_per_hop", "branch_per_hop", "vmem_rd_per_hop",
            "wait_mem_frac", "wait_dep_frac", "tag")
    return {k: e[k] for k in keys if k in e}


INIT_ALLOWANCE_S = 240.0      # first `import torch` on a fresh box (1-2 min) + RCCL init
STEP_BOUND_S = 5.0            # per launch: the slowest BASELINE workload takes ~0.15 s
CPU_BASELINE_ALLOWANCE_S = 120.0
RANK_STAGES = ("started", "init", "timed", "done")


def rank_deadline(args) -> float:
    if args.rank_deadline is not None:
        return float(args.rank_deadline)
    return INIT_ALLOWANCE_S + (STEP_BOUND_S * (args.warmup + args.steps) + CPU_BASELINE_ALLOWANCE_S) * len(args.lfs)


def report_stage(stage: str) -> None:
    """Tell the launcher (launch_ranks) that this rank reached `stage` (a marker file)."""
    d = os.environ.get("PRISMA_BENCH_REPORT_DIR")
    if d:
        with open(os.path.join(d, f"rank{os.environ.get('RANK', '0')}.{stage}"), "w") as fh:
            fh.write(f"{time.time()}\n")


def launch_ranks(n: int, deadline_s: float) -> int:
    """Start n child ranks of this script (one per GPU) and wait for them.  The parent touches no
    GPU (no torch import at all) and does not exec: it runs the ranks as subprocesses with the
    torch.distributed env contract and returns the worst exit status; a failing rank stops the rest.
    Each rank reports its stages (started, init, timed, done) as marker files; if the ranks are not
    all finished `deadline_s` after the start, every rank is terminated (killed after a 10-s grace),
    the ranks that had not reached "done" are named with their last stage, and the exit status is 124."""
    import tempfile
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    rep = tempfile.mkdtemp(prefix="prisma_bench_ranks_")
    procs = []
    t_start = time.monotonic()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PRISMA_BENCH_REPORT_DIR=rep)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))

    def last_stage(r):
        got = [st for st in RANK_STAGES if os.path.exists(os.path.join(rep, f"rank{r}.{st}"))]
        return got[-1] if got else "not started"

    def stop_all(live):
        for q in live:
            q.terminate()
        t_kill = time.monotonic() + 10.0
        for q in live:
            try:
                q.wait(timeout=max(0.1, t_kill - time.monotonic()))
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()

    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0:
                rc = rc or c
                stop_all(live)
                live = []
        if live and time.monotonic() - t_start > deadline_s:
            stuck = [f"rank {r} (last stage: {last_stage(r)})" for r, p in enumerate(procs) if p in live]
            print(f"bench.py: rank deadline of {deadline_s:.0f} s expired; not finished: {', '.join(stuck)}; "
                  f"terminating all {n} ranks", file=sys.stderr, flush=True)
            stop_all(live)
            live = []
            rc = 124
        time.sleep(0.2)
    for f in os.listdir(rep):
        os.unlink(os.path.join(rep, f))
    os.rmdir(rep)
    return rc


def rendezvous_only(args, world: int, rank: int) -> None:
    """--rendezvous-only: initialise the process group, all-gather each rank's replica count and
    print one JSON line on rank 0 (a check of the N-rank plumbing: spawn, rendezvous, collective)."""
    import torch
    import torch.distributed as dist
    from prisma_amd.dist import shard
    backend = args.backend or ("gloo" if args.same_device else "nccl")
    for k, v in (("MASTER_ADDR", "127.0.0.1"), ("RANK", str(rank)), ("WORLD_SIZE", str(world))):
        os.environ.setdefault(k, v)
    if "MASTER_PORT" not in os.environ:                     # one rank without the launcher
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
        sk.close()
    if backend == "nccl":
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
    else:
        dev = torch.device("cpu")
        dist.init_process_group("gloo")
    report_stage("init")
    _, R = shard(args.replicas * world, rank, world)
    t = torch.zeros(world, dtype=torch.int64, device=dev)
    t[rank] = R
    dist.all_reduce(t)
    report_stage("timed")
    if rank == 0:
        print(json.dumps({"rendezvous": "ok", "backend": backend, "world_size": dist.get_world_size(),
                          "replicas_gathered": int(t.sum().item()), "per_rank_replicas": t.cpu().tolist(),
                          "workload": {"preset": args.preset, "topology": args.topology, "policy": args.policy,
                                       "replicas_per_gpu": args.replicas, "ping_as_obs": args.ping_as_obs,
                                       "load_factors": args.lfs, "hops": args.hops, "warmup": args.warmup}}),
              flush=True)
    dist.destroy_process_group()
    report_stage("done")


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, rank_deadline(args)))
    report_stage("started")
    stall = os.environ.get("PRISMA_BENCH_STALL_RANK")       # test hook: this rank hangs before init
    if stall is not None and stall == os.environ.get("RANK"):
        time.sleep(3600)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.rendezvous_only:
        rendezvous_only(args, world, rank)
        return
    import torch
    import torch.distributed as dist

    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    backend = args.backend or ("gloo" if args.same_device else "nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    use_dist = world > 1 or args.force_dist
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:                 # a 1-rank group of its own (--force-dist)
            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            sk.close()
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    report_stage("init")
    coll_dev = dev if backend == "nccl" else torch.device("cpu")

    for lf in args.lfs:
        measure(args, lf, world, rank, use_dist, backend, coll_dev, dev, local)
    if use_dist:
        dist.destroy_process_group()
    report_stage("done")


def measure(args, lf, world, rank, use_dist, backend, coll_dev, dev, local):
    """One workload (the arguments at load factor lf): W untimed steps, K timed steps bracketed by a
    barrier and device synchronisation, the max over ranks; rank 0 prints its JSON line."""
    import torch
    import torch.distributed as dist
    from prisma_amd.config import engine_params
    from prisma_amd.dist import gather_replica_stats, shard
    from prisma_amd.engine import PrismaEngine, build_id
    from prisma_amd.policies import StackedQNet
    from prisma_amd.topology import Topology, sp_next_hop_table

    topo = Topology.example(args.topology, args.tm, lf)
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
    if use_dist:
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
    if use_dist:
        dist.barrier()
    t1 = time.perf_counter()
    report_stage("timed")
    elapsed = t1 - t0
    if use_dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    c1 = eng.counters()
    hops_local = int((c1["hops_total"] - c0["hops_total"]).sum())
    deg_avg = float(c1["hop_deg_sum"].sum()) / max(1, int(c1["hops"].sum()))   # mean deg(u) over hops
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    errors = int(c1["error"].max())
    stats = gather_replica_stats(c1, world, device=coll_dev)   # RCCL all-gather (outside the timed region)
    per_rank = [hops_local]
    if use_dist:
        ht = torch.zeros(world, dtype=torch.int64, device=coll_dev)
        ht[rank] = hops_local
        dist.all_reduce(ht)
        per_rank = [int(x) for x in ht.cpu().tolist()]
        er = torch.tensor([errors], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(er, op=dist.ReduceOp.MAX)
        errors = int(er.item())
    hops_total = int(sum(per_rank))

    if rank == 0:
        # per-launch algorithmic bytes: the hops one launch executes on this rank x B_hop at their mean degree
        hops_per_launch = hops_local / args.steps
        alg_bytes = algorithmic_bytes(int(round(hops_per_launch)), int(round(hops_per_launch * deg_avg)))
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        bid = build_id()
        traffic = pmc_traffic(args.topology, args.replicas, args.hops, bid)
        metric = METRIC if (args.topology, args.replicas) == ("abilene", 4096) else \
            f"packet-hop transitions/sec at {args.replicas} {topo.name} replicas; achieved HBM GB/s"
        workload = (f"{args.topology} tm{args.tm} lf{lf} {args.policy} greedy, {args.replicas} replicas/GPU x "
                    f"{args.hops} hops/step, pingAsObs={args.ping_as_obs}, simTime 60 s auto-reset")
        result = {
            "metric": metric,
            "value": hops_total / elapsed,
            "unit": "hops/s",
            "n_gpus": 1 if args.same_device else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": f"synthetic (Poisson traffic from the shipped {topo.name} TM{args.tm} x load_factor "
                    f"{lf}; {'random-init ' + args.policy + ' weights' if args.policy != 'sp' else 'SP table'})",
            "config": {
                "workload": workload, "preset": args.preset, "load_factor": lf,
                "topology": args.topology, "replicas_per_gpu": args.replicas, "hops_per_step": args.hops,
                "policy": args.policy, "parallelism": f"replica-sharded x{world}"
                + (" (ranks share cuda:0 over gloo: rehearsal, not a scaling figure)" if args.same_device else ""),
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": eng.kernel_name_mlp if args.policy == "dqn_buffer" else eng.kernel_name,
                "kernel_ms": kern_ms, "build_id": bid,
                "alg_bytes_per_launch": alg_bytes, "hops_per_launch": hops_per_launch,
                # the binding resource: instruction issue (committed SQ counters of this build)
                "issue": issue_roofline(args.topology, args.replicas, args.hops, bid),
            },
            "errors": errors,
            "dist": {"world_size": dist.get_world_size() if use_dist else 1, "backend": backend if use_dist else None,
                     "replicas_gathered": int(stats["stats"].shape[0])},
            "episodes_completed": stats["episodes_completed"],
            "replicas_total": int(stats["stats"].shape[0]),
            "per_rank_hops_s": [h / elapsed for h in per_rank],
        }
        if args.cpu_baseline and world == 1:
            kind = "mlp" if args.policy == "dqn_buffer" else "table"
            # warm-up equal to the GPU line's (hops per replica before the timed steps)
            warm = args.warmup * args.hops if args.topology == "er256" else 0
            result["cpu_baseline"] = cpu_baseline(topo, dict(params, auto_reset=0), kind, policy().cpu().numpy(),
                                                  args.cpu_hops, args.cpu_hops_1core, threads=args.replicas,
                                                  warm_hops=warm, workload=workload)
        print(json.dumps(result), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
