"""Quick GPU-vs-oracle check + first timing (diagnostic script, prints details)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import torch
from prisma_amd.config import engine_params
from prisma_amd.engine import PrismaEngine
from prisma_amd.topology import Topology, sp_next_hop_table
import oracle as O


def first_diff(a, b):
    for i in range(min(len(a), len(b))):
        if a[i].tobytes() != b[i].tobytes():
            return i
    return None if len(a) == len(b) else min(len(a), len(b))


def check_table(name, topo, params, R, H):
    eng = PrismaEngine(topo, params, R)
    table = sp_next_hop_table(topo)
    eng.reset(0)
    eng.run(torch.from_numpy(table).cuda(), H)
    torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    ok = True
    for r in range(R):
        o = O.OracleSim(topo, params, replica=r)
        o.run_table(table, H)
        ref = o.records()
        n = min(len(ref), eng.log_capacity)
        got = eng.records(r, 0, int(cnt[r]["dec_count"]), log_host=log) if cnt[r]["dec_count"] <= eng.log_capacity else None
        oc = o.counters()
        bad = [k for k in cnt.dtype.names if k not in ("hops_total", "events_total") and cnt[r][k] != oc[k]]
        if got is None or got.tobytes() != ref.tobytes() or bad or cnt[r]["error"]:
            ok = False
            print(f"[{name}] replica {r}: MISMATCH err={cnt[r]['error']} gpu_dec={cnt[r]['dec_count']} ref_dec={len(ref)} badcounters={bad}")
            for k in bad:
                print("   ", k, cnt[r][k], oc[k])
            if got is not None:
                i = first_diff(got, ref)
                if i is not None:
                    print("   first record diff at", i)
                    for j in range(max(0, i - 2), min(i + 3, len(ref), len(got))):
                        print("     gpu", got[j])
                        print("     ref", ref[j])
            if r > 2:
                break
    print(f"[{name}] {'OK' if ok else 'FAIL'} R={R} H={H}")
    eng.close()
    return ok


def check_external(name, topo, params, R, steps, seed=0):
    eng = PrismaEngine(topo, params, R)
    eng.reset(0)
    rng = np.random.default_rng(seed)
    orcs = [O.OracleSim(topo, params, replica=r) for r in range(R)]
    ref_obs = [o.step(-1) for o in orcs]
    obs, mask = eng.step(None)
    torch.cuda.synchronize()
    ok = True
    deg = topo.degrees
    for s in range(steps):
        g = obs.cpu().numpy(); m = mask.cpu().numpy()
        for r in range(R):
            ro = ref_obs[r]
            if (ro is None) != (m[r] == 0) or (ro is not None and not np.array_equal(ro, g[r])):
                print(f"[{name}] step {s} replica {r}: obs mismatch gpu={g[r]} mask={m[r]} ref={ro}")
                ok = False
                break
        if not ok:
            break
        # random action in [0, deg] (deg => discarded), mostly valid
        cnt = eng.counters()
        acts = np.zeros(R, dtype=np.int32)
        # node of pending decision = from oracle records last
        for r in range(R):
            recs = orcs[r].records()
            node = int(recs[-1]["node"]) if len(recs) else 0
            acts[r] = rng.integers(0, deg[node] + (1 if rng.random() < 0.02 else 0))
        ref_obs = [orcs[r].step(int(acts[r])) for r in range(R)]
        obs, mask = eng.step(torch.from_numpy(acts).cuda())
        torch.cuda.synchronize()
    cnt = eng.counters()
    log = eng.log_tensor().cpu().numpy()
    for r in range(R):
        ref = orcs[r].records()
        got = eng.records(r, 0, len(ref), log_host=log)
        if got.tobytes() != ref.tobytes():
            ok = False
            i = first_diff(got, ref)
            print(f"[{name}] replica {r} records differ at {i}: gpu={got[i]} ref={ref[i]}")
            break
    print(f"[{name}] {'OK' if ok else 'FAIL'} R={R} steps={steps}")
    eng.close()
    return ok


def timing(topo, params, R, H, iters=3):
    eng = PrismaEngine(topo, params, R)
    table = torch.from_numpy(sp_next_hop_table(topo)).cuda()
    eng.reset(0)
    eng.run(table, 64)
    torch.cuda.synchronize()
    c0 = eng.counters()["hops_total"].sum()
    t0 = time.time()
    for _ in range(iters):
        eng.run(table, H)
    torch.cuda.synchronize()
    dt = time.time() - t0
    c1 = eng.counters()
    hops = int(c1["hops_total"].sum() - c0)
    print(f"[timing] {topo.name} R={R} H={H}x{iters}: {hops} hops in {dt:.3f}s = {hops/dt:.3e} hops/s; "
          f"state {eng.state_bytes} B, lds {eng.lds_bytes} B, err={int(c1['error'].max())}, "
          f"events/hop={(c1['events_total'].sum())/max(1,c1['hops_total'].sum()):.2f}")
    eng.close()


if __name__ == "__main__":
    ab = Topology.example("abilene", 0, 1.0)
    ge = Topology.example("geant", 0, 1.0)
    allok = True
    allok &= check_table("abilene-sp-ping", ab, engine_params(ab, sim_time_s=20.0, ping_as_obs=1), 8, 2000)
    allok &= check_table("abilene-sp-buf", ab, engine_params(ab, sim_time_s=20.0, ping_as_obs=0), 8, 2000)
    allok &= check_table("geant-sp-ping", ge, engine_params(ge, sim_time_s=10.0, ping_as_obs=1), 4, 3000)
    allok &= check_table("abilene-lf2", Topology.example("abilene", 1, 2.0),
                         engine_params(Topology.example("abilene", 1, 2.0), sim_time_s=10.0, ping_as_obs=1), 4, 5000)
    allok &= check_external("abilene-ext", ab, engine_params(ab, sim_time_s=20.0, ping_as_obs=1), 16, 300)
    timing(ab, engine_params(ab, sim_time_s=60.0, ping_as_obs=1, auto_reset=1), 4096, 1000)
    timing(ab, engine_params(ab, sim_time_s=60.0, ping_as_obs=1, auto_reset=1), 4096, 4000)
    timing(ge, engine_params(ge, sim_time_s=60.0, ping_as_obs=1, auto_reset=1), 4096, 1000)
    print("ALL", "OK" if allok else "FAIL")
