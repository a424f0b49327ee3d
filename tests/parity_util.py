"""Shared parity machinery for the -m gpu tests: the engine (through the C-ABI) against the CPU
oracle, launch by launch, for as long as a workload needs (steady state, episode ends), and the
in-kernel DQN-buffer decisions against the fp32 torch model.

The oracle (oracle/, test infrastructure) is the checker here, never the thing measured."""
from __future__ import annotations

import numpy as np

from prisma_amd.records import COUNTERS_DTYPE, ST_DROPPED, ST_ENQUEUED

CNT_KEYS = [k for k in COUNTERS_DTYPE.names if k not in ("hops_total", "events_total")]


def assert_counters_equal(g, o, r, where=""):
    bad = [(k, g[k], o[k]) for k in CNT_KEYS if g[k] != o[k]]
    assert not bad, f"replica {r}{where}: counters differ {bad}"


class OracleChain:
    """One replica's oracle, continued into the next episode when one ends (params.auto_reset),
    with decision indices numbered across episodes the way the engine's log numbers them (the log
    position carries over an episode end: include/prisma.h prisma_step)."""

    def __init__(self, oracle_mod, topo, params, replica, policy):
        self.O, self.topo, self.params, self.replica = oracle_mod, topo, params, replica
        self.policy = policy                   # ("table", uint8 [N, N]) or ("mlp", fp32 packed)
        self.ep = 0
        self.base = 0                          # global index of the current episode's first record
        self.o = oracle_mod.OracleSim(topo, params, replica=replica, episode=0)
        self.done = []                         # finished episodes: (base, OracleSim, final counters)
        self.hops_total = 0
        self.events_done = 0                   # events of the finished episodes
        self.t_done = 0                        # simulated ns of the finished episodes
        self.end_diag = []                     # oracle diagnostics (or_diag) at each episode end

    def _run(self, hops):
        kind, pol = self.policy
        return self.o.run_table(pol, hops) if kind == "table" else self.o.run_mlp(pol, hops)

    def _next_episode(self):
        c = self.o.counters()
        assert int(c["episode_over"]) == 1
        if hasattr(self.o, "diag"):
            self.end_diag.append(self.o.diag())
        self.done.append((self.base, self.o, c))
        self.events_done += int(c["events"])
        self.t_done += int(c["now_ns"])
        self.base += int(c["dec_count"])
        self.ep += 1
        self.o = self.O.OracleSim(self.topo, self.params, replica=self.replica, episode=self.ep)

    def advance(self, hops):
        """Execute `hops` more hops, across episode ends when auto_reset is on."""
        left = int(hops)
        while left > 0:
            got = self._run(left)
            left -= got
            self.hops_total += got
            if left > 0:
                assert int(self.o.counters()["episode_over"]) == 1, "oracle stopped short inside an episode"
                if not self.params["auto_reset"]:
                    break
                self._next_episode()
        return int(hops) - left

    def sync_episode(self, episode):
        """The engine has moved on to `episode`: the oracle's current episode must be over
        without further hops (its remaining events run here)."""
        while self.ep < episode:
            assert self._run(1) == 0, "engine ended an episode the oracle still has hops in"
            self._next_episode()

    def records(self, first, count):
        """Records [first, first + count) in global numbering (prev shifted by episode bases)."""
        parts = []
        eps = [(b, o) for b, o, _ in self.done] + [(self.base, self.o)]
        for k, (b, o) in enumerate(eps):
            end = eps[k + 1][0] if k + 1 < len(eps) else b + int(o.counters()["dec_count"])
            lo, hi = max(first, b), min(first + count, end)
            if lo >= hi:
                continue
            r = o.records(lo - b, hi - lo).copy()
            r["prev"] = np.where(r["prev"] >= 0, r["prev"] + b, r["prev"])
            parts.append(r)
        return np.concatenate(parts) if parts else np.zeros(0, dtype=self.o.rec_dtype)

    def counters(self):
        c = self.o.counters().copy()
        c["dec_count"] += self.base
        return c

    def drop_finished(self, upto):
        """Forget finished episodes whose records all lie before global index `upto`."""
        while self.done and self.done[0][0] + int(self.done[0][2]["dec_count"]) <= upto:
            self.done.pop(0)[1].close()


def decisions_of(recs):
    """Records that carry a policy decision (forwarded or dropped: the hops)."""
    return recs[(recs["status"] == ST_ENQUEUED) | (recs["status"] == ST_DROPPED)]


def check_near_ties(net_cpu, weights_host, checker, recs, rel_tol=1e-5):
    """In-kernel DQN-buffer decisions vs the fp32 torch model (models.py:258-306, learner.py:143-145).

    The kernel's actions equal the oracle's fixed-order restatement bit for bit (checked by the
    record comparison); here every decision is also evaluated by torch in fp32 on the CPU. Wherever
    the kernel's action differs from torch's argmin, the two actions must be a genuine near-tie
    under torch's own Q values: Q[a_kernel] - Q[a_torch] <= rel_tol * max(1, |Q[a_torch]|).
    Returns (decisions, disagreements, max |Q_restatement - Q_torch| over all decisions, worst gap)."""
    import torch
    dec = decisions_of(recs)
    if len(dec) == 0:
        return 0, 0, 0.0, 0.0
    W = dec["obs"].shape[1]
    obs = dec["obs"].astype(np.int64)
    node = dec["node"].astype(np.int64)
    with torch.no_grad():
        qt = net_cpu.q_values(torch.from_numpy(obs).to(torch.int32), torch.from_numpy(node)).numpy()
    qo, ao = checker.mlp_q_batch(weights_host, node.astype(np.int32), dec["obs"].astype(np.uint32).reshape(-1, W))
    ak = dec["action"].astype(np.int64)
    assert np.array_equal(ao, ak), "kernel actions differ from the restatement's (records said equal)"
    at = np.argmin(qt, axis=1)
    rows = np.arange(len(dec))
    finite = np.isfinite(qt)
    dq = np.abs(qo[finite] - qt[finite]).max()
    gap = qt[rows, ak] - qt[rows, at]
    tol = rel_tol * np.maximum(1.0, np.abs(qt[rows, at]))
    bad = np.nonzero(gap > tol)[0]
    assert bad.size == 0, (f"{bad.size} kernel decisions are not near-ties of torch's argmin: e.g. node "
                           f"{node[bad[0]]} obs {obs[bad[0]].tolist()} q {qt[bad[0]].tolist()} "
                           f"kernel {ak[bad[0]]} torch {at[bad[0]]}")
    return len(dec), int((ak != at).sum()), float(dq), float(gap.max())


def compare_steady(oracle_mod, eng, topo, params, policy, *, t_target_s, hops_per_launch, min_episode=0,
                   replicas=None, net_cpu=None, max_launches=400, label="", log_tail=False):
    """Run `eng` launch by launch (fused policy) and compare every new decision record and the
    counters of each checked replica with an OracleChain after EVERY launch, until every checked
    replica's simulated clock has passed t_target_s and its episode index reached min_episode.

    policy: ("table", uint8 [N, N] numpy) or ("mlp", packed fp32 numpy). The log is copied out per
    launch, so log_capacity only has to hold one launch's records -- unless log_tail: then a launch
    may write more records than the log ring holds (the bench's own shape: 32 768 hops per launch,
    8 192 records), and the last log_capacity records of each launch are compared (the earlier
    ones were overwritten on the device; the counters still cover the whole launch). Returns a
    summary dict."""
    import torch
    R = eng.R
    picks = list(range(R)) if replicas is None else list(replicas)
    kind, pol = policy
    dev_pol = torch.from_numpy(np.ascontiguousarray(pol)).cuda()
    chains = {r: OracleChain(oracle_mod, topo, params, params["replica_base"] + r, policy) for r in picks}
    checked = {r: 0 for r in picks}
    prev_hops = np.zeros(R, dtype=np.uint64)
    n_cmp = 0
    short = 0                                  # (launch, replica) pairs that executed fewer hops than asked
    tail_launches = 0                          # (launch, replica) pairs compared on the log's tail only
    ties = [0, 0, 0.0, 0.0]
    max_clock = 0
    for launch in range(max_launches):
        eng.run(dev_pol, hops_per_launch)
        torch.cuda.synchronize()
        cnt = eng.counters()
        log = eng.log_tensor().cpu().numpy()
        delta = cnt["hops_total"] - prev_hops
        prev_hops = cnt["hops_total"].copy()
        assert np.all(delta <= hops_per_launch)
        short += int((delta[picks] < hops_per_launch).sum())
        for r in picks:
            c = cnt[r]
            assert int(c["error"]) == 0, (label, r, int(c["error"]))
            ch = chains[r]
            got = ch.advance(int(delta[r]))
            assert got == int(delta[r]), (label, r, got, int(delta[r]))
            ch.sync_episode(int(c["episode"]))
            total = int(c["dec_count"])
            new = total - checked[r]
            first = checked[r]
            if new > eng.log_capacity:
                assert log_tail, (label, "a launch wrote more records than the log holds")
                first, new = total - eng.log_capacity, eng.log_capacity
                tail_launches += 1
            ref = ch.records(first, new)
            assert len(ref) == new, (label, r, len(ref), new)
            got_rec = eng.records(r, first, new, log_host=log)
            if got_rec.tobytes() != ref.tobytes():
                bad = next(i for i in range(new) if got_rec[i].tobytes() != ref[i].tobytes())
                raise AssertionError(f"{label} replica {r} launch {launch}: record {first + bad} differs "
                                     f"(t = {int(ref[bad]['t_ns']) / 1e9:.6f} s)\n engine {got_rec[bad]}\n "
                                     f"oracle {ref[bad]}")
            if kind == "mlp" and net_cpu is not None:
                d, dis, dq, gap = check_near_ties(net_cpu, pol, ch.o, got_rec)
                ties[0] += d
                ties[1] += dis
                ties[2] = max(ties[2], dq)
                ties[3] = max(ties[3], gap)
            n_cmp += new
            checked[r] = total
            assert_counters_equal(c, ch.counters(), r, f" ({label}, launch {launch})")
            assert int(c["hops_total"]) == ch.hops_total
            assert int(c["events_total"]) == ch.events_done + int(ch.o.counters()["events"])
            ch.drop_finished(checked[r])
            max_clock = max(max_clock, int(c["now_ns"]))
        print(f"  [{label}] launch {launch}: t = {min(chains[r].t_done + int(cnt[r]['now_ns']) for r in picks) / 1e9:.2f} s,"
              f" {n_cmp} records compared", flush=True)
        done = all(int(cnt[r]["episode"]) >= min_episode and
                   chains[r].t_done + int(cnt[r]["now_ns"]) >= int(t_target_s * 1e9) for r in picks)
        if done:
            break
    else:
        raise AssertionError(f"{label}: {max_launches} launches did not reach t = {t_target_s} s")
    t_min = min(chains[r].t_done + int(cnt[r]["now_ns"]) for r in picks) / 1e9
    out = dict(label=label, launches=launch + 1, records=n_cmp, t_compared_s=t_min,
               episodes=[int(cnt[r]["episode"]) for r in picks], max_clock_s=max_clock / 1e9,
               hops=int(sum(int(cnt[r]["hops_total"]) for r in picks)), short_launches=short,
               tail_launches=tail_launches, end_diag=[d for r in picks for d in chains[r].end_diag],
               relay_drops=sum(sum(d["relay_drops"] for d in chains[r].end_diag) + chains[r].o.diag()["relay_drops"]
                               for r in picks))
    if kind == "mlp" and net_cpu is not None:
        out.update(mlp_decisions=ties[0], torch_disagreements=ties[1], max_abs_dq=ties[2], max_tie_gap=ties[3])
    print(f"\n[steady] {label}: compared up to t = {t_min:.3f} s of simulated time per replica "
          f"({out['records']} records, {out['launches']} launches, episodes {out['episodes']})"
          + (f"; torch fp32: {ties[1]} of {ties[0]} decisions differ, all near-ties (max gap {ties[3]:.3g}), "
             f"max |Q_restatement - Q_torch| = {ties[2]:.3g}" if kind == "mlp" and net_cpu is not None else ""))
    return out
