"""Replay buffers and the Q-routing trainer (prisma_amd/trainer.py) against the
reference's own ReplayBuffer (fixture) and restatements of learner.py / trainer.py math, on CPU."""
import copy
import json
import os

import numpy as np
import pytest
import torch

from prisma_amd.topology import Topology
from prisma_amd.trainer import LinearSchedule, QRoutingTrainer, ReplayBuffers, huber


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "replay_buffer.json")


def _batch(bt, W):
    return {"node": torch.tensor(bt["node"], dtype=torch.int64),
            "obs": torch.tensor(bt["obs"], dtype=torch.int32).reshape(-1, W),
            "next_obs": torch.tensor(bt["next_obs"], dtype=torch.int32).reshape(-1, W),
            "action": torch.tensor(bt["action"], dtype=torch.int64),
            "reward": torch.tensor(bt["reward"], dtype=torch.float64),
            "done": torch.tensor(bt["done"], dtype=torch.bool)}


def test_replay_buffers_match_reference_fixture():
    """Per-node rings against the states the reference's own ReplayBuffer.add reached on the
    same transition sequence (replay_buffer.py:12-37; tests/golden/make_replay_golden.py)."""
    fx = json.load(open(GOLDEN))
    N, size, W = fx["n_nodes"], fx["size"], fx["obs_width"]
    buf = ReplayBuffers(N, size, W, device="cpu")
    for bt, st in zip(fx["batches"], fx["states"]):
        buf.add(_batch(bt, W))
        for u in range(N):
            assert int(buf.count[u]) == st[u]["len"]
            assert int(buf.next_idx[u]) == st[u]["next_idx"]
            assert int(buf.total[u]) == st[u]["total_samples"]
            assert buf.obs[u, :st[u]["len"], 0].tolist() == st[u]["tags"]
    for u in range(N):
        for i, d in enumerate(fx["final"][u]):
            assert buf.obs[u, i].tolist() == d["obs"]
            assert buf.next_obs[u, i].tolist() == d["next_obs"]
            assert int(buf.action[u, i]) == d["action"]
            assert float(buf.reward[u, i]) == float(np.float32(d["reward"]))   # rings store f32 rewards
            assert bool(buf.done[u, i]) == d["done"]
    o, a, r, no, dn = buf.sample(16, torch.Generator().manual_seed(1))
    assert o.shape == (N, 16, W) and a.shape == (N, 16)
    for u in range(N):                                    # samples come from the node's own ring
        assert set(o[u, :, 0].tolist()) <= set(fx["states"][-1][u]["tags"])


def test_linear_schedule():
    s = LinearSchedule(3000, 1.0, 0.1)
    v = s.value(torch.tensor([0, 1500, 3000, 9000]))
    assert torch.allclose(v, torch.tensor([1.0, 0.55, 0.1, 0.1], dtype=torch.float64))


def test_huber_and_infinite_targets():
    x = torch.tensor([-3.0, -0.5, 0.0, 0.5, 3.0, -float("inf")], requires_grad=True)
    y = huber(x)
    assert torch.allclose(y[:5], torch.tensor([2.5, 0.125, 0.0, 0.125, 2.5]))
    y[:5].sum().backward(retain_graph=True)
    x.grad = None
    y.sum().backward()
    assert torch.isfinite(x.grad).all() and x.grad[-1] == -1.0


def test_targets_match_per_sample_restatement():
    """trainer.py:60-72 + learner.py:231-255: the next node's target Q, v's interface back
    to u filtered out, min over the rest; done -> reward."""
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "buffer", seed=3, device="cpu", batch_size=8)
    rng = np.random.default_rng(2)
    B = 64
    node = torch.from_numpy(rng.integers(0, 11, B))
    action = torch.tensor([int(rng.integers(0, topo.degrees[u])) for u in node.tolist()])
    reward = torch.from_numpy(rng.random(B).astype(np.float32))
    nobs = torch.from_numpy(rng.integers(0, 16000, (B, topo.obs_width)).astype(np.int32))
    nobs[:, 0] = torch.from_numpy(rng.integers(0, 11, B).astype(np.int32))
    done = torch.from_numpy(rng.random(B) < 0.25)
    got = tr.targets(node, action, reward, nobs, done)
    for i in range(B):
        u, a = int(node[i]), int(action[i])
        v = topo.neighbors(u)[a]
        if bool(done[i]):
            assert float(got[i]) == float(reward[i])
            continue
        q = tr.q_target.q_values(nobs[i:i + 1], torch.tensor([v]))[0]
        keep = [j for j, w in enumerate(topo.neighbors(v)) if w != u]
        want = float(reward[i]) + min(float(q[j]) for j in keep)
        assert abs(float(got[i]) - want) < 1e-6


def test_keras_adam_per_node_and_idle_nodes_untouched():
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "routing", seed=4, device="cpu", batch_size=4, lr=1e-3)
    W0 = tr.q.W2.detach().clone()
    g1 = torch.randn_like(tr.q.W2)
    g2 = torch.randn_like(tr.q.W2)
    ready1 = torch.zeros(11, dtype=torch.bool)
    ready1[[1, 4]] = True
    ready2 = torch.ones(11, dtype=torch.bool)
    for g, rd in ((g1, ready1), (g2, ready2)):
        for p in tr.params:
            p.grad = torch.zeros_like(p)
        tr.q.W2.grad = g.clone()
        tr._adam(rd)
    W = tr.q.W2.detach()
    for u in range(11):                                     # numpy Keras Adam per node
        m = np.zeros(W0[u].shape)
        v = np.zeros(W0[u].shape)
        w = W0[u].numpy().astype(np.float64)
        t = 0
        for g, rd in ((g1, ready1), (g2, ready2)):
            if not rd[u]:
                continue
            t += 1
            gu = g[u].numpy().astype(np.float64)
            m = 0.9 * m + 0.1 * gu
            v = 0.999 * v + 0.001 * gu * gu
            lr_t = 1e-3 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
            w = w - lr_t * m / (np.sqrt(v) + 1e-7)
        assert np.allclose(W[u].numpy(), w, atol=1e-6), u


def test_train_step_reduces_td_error_on_a_fixed_batch():
    """Repeated steps on one node's buffer of synthetic transitions lower its loss."""
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "buffer", seed=5, device="cpu", batch_size=32, lr=1e-3)
    rng = np.random.default_rng(5)
    n = 400
    node = torch.from_numpy(rng.integers(0, 11, n))
    obs = torch.from_numpy(rng.integers(0, 16000, (n, topo.obs_width)).astype(np.int32))
    obs[:, 0] = torch.from_numpy(rng.integers(0, 11, n).astype(np.int32))
    act = torch.tensor([int(rng.integers(0, topo.degrees[u])) for u in node.tolist()])
    tr.observe({"node": node, "obs": obs, "next_obs": obs.clone(), "action": act,
                "reward": torch.full((n,), 0.01), "done": torch.ones(n, dtype=torch.bool)})
    first = tr.train_step()
    for _ in range(60):
        last = tr.train_step()
    ok = ~torch.isnan(first)
    assert ok.any() and bool((last[ok] < first[ok]).all())


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")
def test_training_loop_on_the_engine():
    """End to end on the device: the engine steps 256 Abilene replicas under the trainer's
    epsilon-greedy policy, transitions flow into the per-node buffers, every node trains."""
    from prisma_amd.env import VecRoutingEnv
    from prisma_amd.trainer import train
    env = VecRoutingEnv("abilene", n_replicas=256, sim_time_s=30.0, ping_as_obs=0)
    tr = QRoutingTrainer(env.topo, "buffer", batch_size=64, buffer_size=4096, seed=0, n_replicas=256,
                         sync_step=0.05)
    w0 = tr.q.W2.detach().clone()
    losses = train(env, tr, steps=200, train_every=4)
    env.close()
    assert losses and np.all(np.isfinite(losses))
    assert int(tr.buffers.total.sum()) > 200 * 256 // 2
    assert bool((tr.steps > 0).all())                       # every Abilene node trained
    assert not torch.equal(w0, tr.q.W2.detach())


def _restated_target(topo, copies, node, action, reward, nobs, done, gamma=1.0):
    """learner.py:231-255 per sample with node u's own copy of neighbour i (a state dict)."""
    from prisma_amd.policies import StackedQNet
    net = StackedQNet(topo, "buffer", seed=0, device="cpu")
    out = []
    with torch.no_grad():
        for j in range(len(node)):
            u, a = int(node[j]), int(action[j])
            if bool(done[j]):
                out.append(float(reward[j]))
                continue
            v = topo.neighbors(u)[a]
            net.load_state_dict(copies[(u, a)])
            q = net.q_values(nobs[j:j + 1], torch.tensor([v]))[0]
            keep = [k for k, w in enumerate(topo.neighbors(v)) if w != u]
            out.append(float(reward[j]) + gamma * min(float(q[k]) for k in keep))
    return out


def test_nn_signaling_copies_follow_the_reference_rules():
    """trainer.py:101-171 + learner.py:257-295 + forwarder.py:251-263: per (node, neighbour)
    target / upcoming / temp copies, restated literally with state dicts."""
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "buffer", seed=3, device="cpu", signaling_type="NN", nn_max_seg_index=68)
    snap = lambda: {k: t.detach().clone() for k, t in tr.q.state_dict().items()}
    q0 = snap()
    pairs = [(u, i) for u in range(11) for i in range(int(topo.degrees[u]))]
    cp = {p: {"t": q0, "up": q0, "tmp": q0} for p in pairs}
    counter = np.full(11, -1, dtype=int)                     # Agent.sync_counters start at -1 (forwarder.py:123)
    rng = np.random.default_rng(4)
    g = torch.Generator().manual_seed(1)
    for step in range(6):
        with torch.no_grad():                                       # "training" between syncs
            for p in tr.q.parameters():
                p.add_(0.05 * torch.randn(p.shape, generator=g))
        now = snap()
        for p in pairs:
            cp[p]["tmp"], cp[p]["up"] = cp[p]["up"], now
        counter += 1
        tr.sync()
        for _ in range(12):
            v = int(rng.integers(0, 11))
            i = int(rng.integers(0, topo.degrees[v]))
            src = topo.neighbors(v)[i]
            nn = int(counter[v] - rng.integers(1, 3))
            seg = 68 if rng.random() < 0.7 else int(rng.integers(0, 68))
            if seg == 68:
                cp[(v, i)]["t"] = cp[(v, i)]["tmp"] if nn == counter[v] - 1 else cp[(v, i)]["up"]
            tr.on_big_signal(v, src, nn, seg)
    with pytest.raises(ValueError):
        tr.on_big_signal(0, topo.neighbors(0)[0], 0, 69)
    B = 96
    node = torch.from_numpy(rng.integers(0, 11, B))
    action = torch.tensor([int(rng.integers(0, topo.degrees[u])) for u in node.tolist()])
    reward = torch.from_numpy(rng.random(B).astype(np.float32))
    nobs = torch.from_numpy(rng.integers(0, 16000, (B, topo.obs_width)).astype(np.int32))
    nobs[:, 0] = torch.from_numpy(rng.integers(0, 11, B).astype(np.int32))
    done = torch.from_numpy(rng.random(B) < 0.2)
    got = tr.targets(node, action, reward, nobs, done)
    want = _restated_target(topo, {p: c["t"] for p, c in cp.items()}, node, action, reward, nobs, done)
    assert np.allclose(got.numpy(), np.array(want, dtype=np.float32), atol=1e-6)
    assert len(tr.snapshots) <= 3 * len(pairs) + 1


def _hop_batch(topo, rng, n, replicas=3):
    node = torch.from_numpy(rng.integers(0, 11, n))
    obs = torch.from_numpy(rng.integers(0, 16000, (n, topo.obs_width)).astype(np.int32))
    obs[:, 0] = torch.from_numpy(rng.integers(0, 11, n).astype(np.int32))
    return {"node": node.int(), "obs": obs, "next_obs": obs.flip(0).clone(),
            "action": torch.tensor([int(rng.integers(0, topo.degrees[u])) for u in node.tolist()], dtype=torch.int32),
            "reward": torch.from_numpy(rng.random(n)), "done": torch.from_numpy(rng.random(n) < 0.2),
            "replica": torch.from_numpy(rng.integers(0, replicas, n)).int(),
            "uid": torch.arange(100, 100 + n, dtype=torch.int64) + (1 << 21) * 5,   # above 21 bits
            "hop": torch.from_numpy(rng.random(n) < 0.75)}


def _echo_rows(tr_batch, idx, R, W):
    """Control notifications of one env step: the echo of transition idx[k] at replica k."""
    obs = torch.zeros((R, W), dtype=torch.int32)
    node = torch.full((R,), -1, dtype=torch.int32)
    ctrl = torch.zeros(R, dtype=torch.bool)
    for j in idx:
        r = int(tr_batch["replica"][j])
        obs[r, 0], obs[r, 1], obs[r, 2] = 1000, int(tr_batch["uid"][j]) & ((1 << 21) - 1), 54
        node[r], ctrl[r] = tr_batch["node"][j], True
    return obs, {"control": ctrl, "node": node}


@pytest.mark.parametrize("kind", ["NN", "target"])
def test_hop_transitions_wait_for_their_echo(kind):
    """forwarder.py:380-410 + 246-250: with "NN" / "target" signalling a hop transition
    enters u's buffer when its packet's echo is back at u (loss transitions at once); a
    "target" transition carries the next node's online-network target."""
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "buffer", seed=6, device="cpu", signaling_type=kind, batch_size=4, n_replicas=3)
    rng = np.random.default_rng(8)
    b = _hop_batch(topo, rng, 40)
    hop = b["hop"].numpy()
    tr.observe(b)
    assert int(tr.buffers.total.sum()) == int((~hop).sum())
    want_t = None
    if kind == "target":
        h = np.nonzero(hop)[0]
        want_t = _restated_target(topo, {(u, i): tr.q.state_dict() for u in range(11)
                                         for i in range(int(topo.degrees[u]))},
                                  b["node"][h], b["action"][h], b["reward"][h].float(), b["next_obs"][h], b["done"][h])
    released = 0
    for j in np.nonzero(hop)[0]:
        # an echo at another node releases nothing, the right one releases exactly its transition
        obs, info = _echo_rows(b, [j], 3, topo.obs_width)
        info["node"] = (info["node"] + 1) % 11
        tr.on_control(obs, info)
        assert int(tr.buffers.total.sum()) == int((~hop).sum()) + released
        obs, info = _echo_rows(b, [j], 3, topo.obs_width)
        tr.on_control(obs, info)
        released += 1
        assert int(tr.buffers.total.sum()) == int((~hop).sum()) + released
    assert tr._pend_key.numel() == 0
    if kind == "target":
        got = []
        for j in np.nonzero(hop)[0]:
            u = int(b["node"][j])
            rows = tr.buffers.reward[u, :int(tr.buffers.count[u])]
            acts = tr.buffers.action[u, :int(tr.buffers.count[u])]
            obs_u = tr.buffers.obs[u, :int(tr.buffers.count[u])]
            k = [m for m in range(len(rows)) if int(acts[m]) == int(b["action"][j]) and
                 torch.equal(obs_u[m], b["obs"][j])][0]
            got.append(float(rows[k]))
        assert np.allclose(got, np.array(want_t, dtype=np.float32), atol=1e-6)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")
def test_training_loop_with_nn_signaling():
    """End to end with "NN" signalling on the engine (train + notify_dest + big signalling):
    hop transitions enter the buffers as their echoes come back, completed NN copies swap
    the per-neighbour target copies, every step's loss is finite."""
    from prisma_amd.env import VecRoutingEnv
    from prisma_amd.trainer import train
    env = VecRoutingEnv("abilene", n_replicas=64, sim_time_s=30.0, ping_as_obs=1, train=1, notify_dest=1,
                        signaling_type="NN", big_signaling=1, sync_step_s=0.05, big_signaling_bytes=1024)
    tr = QRoutingTrainer(env.topo, "buffer", batch_size=32, buffer_size=4096, seed=0, signaling_type="NN",
                         big_signaling_size=1024, n_replicas=64, sync_step=0.05)
    losses = train(env, tr, steps=600, train_every=4)
    env.close()
    assert losses and np.all(np.isfinite(losses))
    assert int(tr.buffers.total.sum()) > 0
    assert bool((tr.tgt_ver > 0).any())


# ---- PrioritizedReplayBuffer (replay_buffer.py:393-534) ----------------------------------
PRIO_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "prio_replay_buffer.json")


def test_prioritized_replay_matches_reference_fixture():
    """Per-node prioritized rings against the states the reference's own PrioritizedReplayBuffer
    reached on the same operation script (tests/golden/make_prio_replay_golden.py): priorities of
    the stored slots (sum-tree leaves), the tree total (bit for bit: the same pairwise sums), max
    priority, latest gradient steps, the per-action slot lists, and the importance weights of the
    samples the reference drew (fed the same indices)."""
    fx = json.load(open(PRIO_GOLDEN))
    deg, size, W = fx["degrees"], fx["size"], fx["obs_width"]
    N = len(deg)
    buf = ReplayBuffers(N, size, W, device="cpu", prioritized=True, max_deg=max(deg), alpha=fx["alpha"])
    n_samples = 0
    for op, rec in zip(fx["ops"], fx["trace"]):
        u = op["node"]
        if op["op"] == "add":
            buf.add({"node": torch.tensor([u]), "obs": torch.tensor([op["obs"]], dtype=torch.int32),
                     "next_obs": torch.tensor([op["next_obs"]], dtype=torch.int32),
                     "action": torch.tensor([op["action"]]), "reward": torch.tensor([op["reward"]]),
                     "done": torch.tensor([op["done"]]), "prio": torch.tensor([op["prio"]], dtype=torch.float64)})
        elif op["op"] == "grad":
            buf.gradient_step(u, op["action"], op["step"])
        elif not rec.get("skipped"):
            B = len(rec["idx"])
            idx = torch.zeros((N, B), dtype=torch.int64)
            idx[u] = torch.tensor(rec["idx"])
            smp = buf.sample_full(B, idx=idx)
            assert smp["obs"][u, :, 0].tolist() == rec["tags"]
            assert smp["weights"][u].tolist() == rec["weights"]
            n_samples += 1
        st = rec["state"]
        n = st["len"]
        assert int(buf.count[u]) == n and int(buf.next_idx[u]) == st["next_idx"]
        assert int(buf.total[u]) == st["total_samples"]
        assert buf.obs[u, :n, 0].tolist() == st["tags"]
        assert buf.prio[u, :n].tolist() == st["prio"] == st["prio_min"]
        assert float(buf.tree_sum()[u]) == st["tree_sum"]
        assert float(buf.max_prio[u]) == st["max_priority"]
        assert buf.latest[u, :deg[u]].tolist() == st["latest_gradient_step"]
        for a in range(deg[u]):
            assert set(torch.nonzero(buf.member[u, a]).squeeze(1).tolist()) == set(st["neighbors_idx"][a])
    assert n_samples >= 10


def test_prioritized_batch_add_equals_one_by_one():
    """A batch add (several nodes, overflowing rings) equals the same transitions added one by one."""
    rng = np.random.default_rng(3)
    N, size, W, D = 4, 5, 4, 3
    n = 37
    tr = {"node": torch.from_numpy(rng.integers(0, N, n)), "obs": torch.from_numpy(rng.integers(0, 99, (n, W))).int(),
          "next_obs": torch.from_numpy(rng.integers(0, 99, (n, W))).int(),
          "action": torch.from_numpy(rng.integers(0, D, n)), "reward": torch.from_numpy(rng.random(n)),
          "done": torch.from_numpy(rng.random(n) < 0.3), "prio": torch.from_numpy(rng.integers(1, 5, n)).double()}
    a = ReplayBuffers(N, size, W, device="cpu", prioritized=True, max_deg=D)
    b = ReplayBuffers(N, size, W, device="cpu", prioritized=True, max_deg=D)
    a.gradient_step(1, 2, 3)
    b.gradient_step(1, 2, 3)
    a.add(tr)
    for i in range(n):
        b.add({k: t[i:i + 1] for k, t in tr.items()})
    for f in ("obs", "action", "count", "next_idx", "total", "prio", "orig", "member", "max_prio"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


def test_prioritized_loss_is_importance_weighted():
    """learner.py:179: mean(weights * huber) per node, weights from the prioritized buffer."""
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "buffer", seed=5, device="cpu", batch_size=8, lr=1e-3, prioritized_replay=True)
    rng = np.random.default_rng(6)
    n = 200
    node = torch.from_numpy(rng.integers(0, 11, n))
    obs = torch.from_numpy(rng.integers(0, 16000, (n, topo.obs_width)).astype(np.int32))
    obs[:, 0] = torch.from_numpy(rng.integers(0, 11, n).astype(np.int32))
    act = torch.tensor([int(rng.integers(0, topo.degrees[u])) for u in node.tolist()])
    tr.observe({"node": node, "obs": obs, "next_obs": obs.clone(), "action": act,
                "reward": torch.full((n,), 0.01), "done": torch.ones(n, dtype=torch.bool)})
    for u in range(11):                                     # newer steps for action 0: priorities below 1
        tr.buffers.gradient_step(u, 0, 4)
    g = torch.Generator().manual_seed(9)
    tr.gen = torch.Generator().manual_seed(9)
    s = tr.buffers.sample_full(8, g)
    per = tr.train_step()
    N, B = 11, 8
    q = StackedQNet_copy = None
    assert per is not None and torch.isfinite(per[~torch.isnan(per)]).all()
    w = s["weights"]
    assert bool((w[s["action"] == 0] < 1.0).any()) and bool((w[s["action"] != 0] >= 1.0).all())


# ---- signalingSim=0: the agents' own signalling delays (forwarder.py:94-108, trainer.py) -----
class _RefAgents:
    """A literal per-replica restatement of the reference's signalingSim=0 bookkeeping: one
    upcoming-event list per node kept sorted by time (forwarder.py:434-442), released while its
    head's time <= Agent.curr_time (forwarder.py:444-464), then the sync check (trainer.py:101-112,
    155-171); target copies as version numbers."""

    def __init__(self, topo, R, sync_step, small_delay, big_delay):
        self.topo, self.R = topo, R
        self.sync_step, self.small_delay, self.big_delay = sync_step, small_delay, big_delay
        N = topo.n_nodes
        self.upcoming = [[[] for _ in range(N)] for _ in range(R)]
        self.counter = np.full((R, N), -1)
        D = topo.max_deg
        self.tgt = np.zeros((R, N, D), dtype=int)
        self.up = np.zeros((R, N, D), dtype=int)
        self.tmp = np.zeros((R, N, D), dtype=int)
        self.buffers = [[] for _ in range(N)]
        self.version = 0

    def push(self, r, u, item):
        item["seq"] = self.seq = getattr(self, "seq", 0) + 1
        self.upcoming[r][u].append(item)
        self.upcoming[r][u].sort(key=lambda e: e["time"])

    def step(self, clock):
        released = []
        for r in range(self.R):
            for u in range(self.topo.n_nodes):
                q = self.upcoming[r][u]
                while q and q[0]["time"] <= clock[r]:
                    e = q.pop(0)
                    if "tag" in e:
                        released.append((e["time"], e["seq"], u, e["tag"]))
                    else:
                        self.tgt[r, u, e["i"]] = self.up[r, u, e["i"]]
        # the replicas are separate simulations sharing the per-node buffers: one step's releases
        # enter them in time order across replicas (the trainer's choice; one simulation has no
        # such merge)
        for _, _, u, tg in sorted(released):
            self.buffers[u].append(tg)
        due = [(r, u) for r in range(self.R) for u in range(self.topo.n_nodes)
               if self.topo.degrees[u] > 0 and clock[r] > (self.counter[r, u] + 1) * self.sync_step]
        if due:
            self.version += 1
        for r, u in due:
            for i in range(int(self.topo.degrees[u])):
                self.tmp[r, u, i] = self.up[r, u, i]
                self.up[r, u, i] = self.version
                self.push(r, u, {"time": clock[r] + self.big_delay[u], "i": i})
            self.counter[r, u] += 1


def test_signaling_sim0_nn_queues_follow_the_reconstruction():
    """signalingSim=0 with "NN" (a reconstruction of the reference's intent: its own path raises
    AttributeError, trainer.py module docstring): hop transitions reach u's buffer
    small_signaling_delay(v) after their notification, every sync queues the neighbours' NNs for
    big_signaling_delay(u), and the target copies follow, per replica, against the literal
    restatement above."""
    topo = Topology.example("abilene")
    R = 3
    tr = QRoutingTrainer(topo, "buffer", seed=2, device="cpu", signaling_type="NN", signaling_sim=0,
                         n_replicas=R, sync_step=0.3, batch_size=4)
    # forwarder.py:94-108: sizes and delays
    for u in range(11):
        d = int(topo.degrees[u])
        assert tr.small_size[u] == 64 + 8 + 8 * (d + 1)
        assert tr.nn_size[u] == 32 * sum(int(p[u].numel()) for p in (tr.q.W1[:, :topo.n_overlay], tr.q.b1)) \
            + 32 * ((d * 32 + 32) + (64 * 64 + 64) * 2 + 64 * d + d)
        assert tr.small_delay[u] == tr.small_size[u] / 500000 + 0.001
        assert tr.big_delay[u] == tr.nn_size[u] / 500000 + 0.001
    ref = _RefAgents(topo, R, 0.3, tr.small_delay, tr.big_delay)
    rng = np.random.default_rng(11)
    clock = np.zeros(R)
    tag = 0
    for step in range(120):
        clock = clock + rng.random(R) * 0.03
        n = int(rng.integers(0, 6))
        node = rng.integers(0, 11, n)
        act = np.array([int(rng.integers(0, topo.degrees[u])) for u in node], dtype=np.int64)
        rep = rng.integers(0, R, n)
        t_ns = np.array([int((clock[r] - rng.random() * 0.01) * 1e9) for r in rep], dtype=np.int64)
        hop = rng.random(n) < 0.8
        obs = np.zeros((n, topo.obs_width), dtype=np.int32)
        obs[:, 0] = np.arange(tag, tag + n)
        for j in range(n):
            v = topo.neighbors(int(node[j]))[act[j]]
            if hop[j]:
                ref.push(int(rep[j]), int(node[j]), {"time": t_ns[j] / 1e9 + tr.small_delay[v], "tag": tag + j})
            else:
                ref.buffers[int(node[j])].append(tag + j)
        tag += n
        batch = {"node": torch.from_numpy(node).int(), "obs": torch.from_numpy(obs), "next_obs": torch.from_numpy(obs),
                 "action": torch.from_numpy(act).int(), "reward": torch.full((n,), 0.01, dtype=torch.float64),
                 "done": torch.zeros(n, dtype=torch.bool), "replica": torch.from_numpy(rep).int(),
                 "uid": torch.arange(n, dtype=torch.int64), "hop": torch.from_numpy(hop), "t_ns": torch.from_numpy(t_ns)}
        # the reference releases transitions pushed in an earlier round only: push first, then step
        tr.advance_clock(torch.from_numpy((clock * 1e9).astype(np.int64)))
        tr.on_step(torch.zeros((R, topo.obs_width), dtype=torch.int32), {"transitions": batch})
        ref.step(clock)
        for u in range(11):
            cnt = int(tr.buffers.count[u])
            got = tr.buffers.obs[u, :cnt, 0].tolist()
            assert got == (ref.buffers[u][-cnt:] if cnt else []), (step, u, got, ref.buffers[u])
        valid = np.arange(topo.max_deg)[None, None, :] < topo.degrees[None, :, None]
        assert np.array_equal(tr.tgt_ver * valid, ref.tgt) and np.array_equal(tr.up_ver * valid, ref.up), step
    assert tr.big_pkts > 0 and tr.small_pkts > 0 and bool((tr.tgt_ver > 0).any())


def test_compute_sync_step_restates_trainer_formula():
    """trainer.py:114-134's formula, nn_size / (sum(TM) * ratio - pkts_per_s * small_signaling_pkt_size)
    (parity unpinned: the reference never reaches it -- Forwarder calls _compute_sync_step, which
    only Trainer defines, and trainer.py:106 syncs on Agent.sync_step = -1)."""
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "buffer", seed=0, device="cpu", signaling_type="NN", sync_step=-1, sync_ratio=0.1)
    from prisma_amd.trainer import convert_bps_to_data_rate
    data = sum(convert_bps_to_data_rate(x) for x in np.asarray(topo.tm_strings, dtype=object).ravel())
    for u in range(11):
        want = tr.nn_size[u] / (data * 0.1 - data / (512 * 8) * (64 + 8 + 8 * (topo.degrees[u] + 1)))
        assert abs(tr.sync_step[u] - want) <= 1e-12 * abs(want)
    assert convert_bps_to_data_rate("12.5Kbps") == 12500.0 and convert_bps_to_data_rate("3Mbps") == 3e6


def test_echo_releases_only_the_first_queued_match_and_new_episode_drops_the_queue():
    """forwarder.py:477-490 pops ONE element per echo (the first in time order); a replica that
    starts a new episode forgets its queued transitions (agent.py:141-145)."""
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "buffer", seed=6, device="cpu", signaling_type="NN", batch_size=4, n_replicas=2)
    obs = torch.zeros((3, topo.obs_width), dtype=torch.int32)
    obs[:, 0] = torch.tensor([7, 8, 9], dtype=torch.int32)
    b = {"node": torch.tensor([3, 3, 3], dtype=torch.int32), "obs": obs, "next_obs": obs,
         "action": torch.tensor([0, 0, 0], dtype=torch.int32), "reward": torch.zeros(3, dtype=torch.float64),
         "done": torch.zeros(3, dtype=torch.bool), "replica": torch.tensor([0, 0, 1], dtype=torch.int32),
         "uid": torch.tensor([5, 5, 5]), "hop": torch.ones(3, dtype=torch.bool),
         "t_ns": torch.tensor([2_000_000, 1_000_000, 1_000_000])}
    tr.observe(b)
    eo = torch.zeros((2, topo.obs_width), dtype=torch.int32)
    eo[0, 0], eo[0, 1] = 1000, 5
    tr.on_control(eo, {"control": torch.tensor([True, False]), "node": torch.tensor([3, -1], dtype=torch.int32)})
    assert tr.buffers.obs[3, :int(tr.buffers.count[3]), 0].tolist() == [8]      # the earlier of the two
    tr.advance_clock(torch.tensor([5_000_000, 5_000_000]), torch.tensor([0, 1]))  # replica 1: next episode
    assert tr._pend_key.numel() == 1 and int(tr._pend["replica"][0]) == 0
    assert tr.sync_counter[1].max() == -1


def test_snapshot_generations_stay_bounded_with_drifting_clocks():
    """Thousands of replicas whose clocks drift apart sync at different steps: the stored weight
    generations stay within max_snapshots, syncs between two optimizer steps share one
    generation, and the targets still come from each copy's weights."""
    topo = Topology.example("abilene")
    R = 2048
    tr = QRoutingTrainer(topo, "buffer", seed=3, device="cpu", signaling_type="NN", n_replicas=R, sync_step=0.01,
                         batch_size=4, max_snapshots=8)
    rng = np.random.default_rng(5)
    clock = np.zeros(R)
    speed = rng.random(R) * 0.004
    g = torch.Generator().manual_seed(1)
    with pytest.warns(RuntimeWarning, match="max_snapshots=8 reached"):
        for step in range(60):
            clock += speed
            tr.advance_clock(torch.from_numpy((clock * 1e9).astype(np.int64)))
            tr.check_sync()
            if step % 3 == 0:                                       # an optimizer step now and then
                with torch.no_grad():
                    for p in tr.q.parameters():
                        p.add_(1e-3 * torch.randn(p.shape, generator=g))
            assert len(tr.snapshots) <= 8, (step, len(tr.snapshots))
    assert tr.stale_syncs > 0 and tr.stats()["stale_syncs"] == tr.stale_syncs   # the cap was forced
    assert len(set(tr.tgt_ver.ravel().tolist()) | set(tr.up_ver.ravel().tolist())) > 8   # many versions...
    # ...each resolving to stored weights, and targets() runs one pass per stored generation
    B = 64
    node = torch.from_numpy(rng.integers(0, 11, B))
    action = torch.tensor([int(rng.integers(0, topo.degrees[u])) for u in node.tolist()])
    nobs = torch.from_numpy(rng.integers(0, 16000, (B, topo.obs_width)).astype(np.int32))
    nobs[:, 0] = torch.from_numpy(rng.integers(0, 11, B).astype(np.int32))
    rep = torch.from_numpy(rng.integers(0, R, B))
    tr.tgt_ver[:] = tr.up_ver
    got = tr.targets(node, action, torch.zeros(B), nobs, torch.zeros(B, dtype=torch.bool), rep)
    for j in range(0, B, 8):
        net = copy.deepcopy(tr._eval)
        net.load_state_dict(tr.weights_of(int(tr.tgt_ver[rep[j], node[j], action[j]])))
        want = tr._bootstrap(net, node[j:j + 1], action[j:j + 1], torch.zeros(1), nobs[j:j + 1],
                             torch.zeros(1, dtype=torch.bool))
        assert torch.allclose(got[j:j + 1], want, rtol=1e-6, atol=1e-6), (got[j], want)


def test_syncs_copy_the_current_weights_without_a_cap():
    """Default (max_snapshots=None): every sync's copy is the online weights at that sync, as the
    reference's _sync_all copies them (trainer.py:101-171), and no sync is counted stale."""
    import warnings as _w
    topo = Topology.example("abilene")
    R = 64
    tr = QRoutingTrainer(topo, "buffer", seed=4, device="cpu", n_replicas=R, sync_step=0.01, batch_size=4)
    rng = np.random.default_rng(7)
    clock = np.zeros(R)
    speed = rng.random(R) * 0.004
    g = torch.Generator().manual_seed(2)
    syncs = 0
    with _w.catch_warnings():
        _w.simplefilter("error", RuntimeWarning)
        for step in range(60):
            clock += speed
            tr.advance_clock(torch.from_numpy((clock * 1e9).astype(np.int64)))
            v0 = tr.version
            tr.check_sync()
            cur = {k: t.detach().clone() for k, t in tr.q.state_dict().items()}
            if tr.version != v0:
                syncs += 1
                for k, t in tr.weights_of(tr.version).items():       # this sync's copy == the weights now
                    assert torch.equal(t, cur[k]), (step, k)
            with torch.no_grad():                                     # an optimizer step after every sync
                for p in tr.q.parameters():
                    p.add_(1e-3 * torch.randn(p.shape, generator=g))
    assert syncs > 32 and tr.stale_syncs == 0 and tr.stats()["stale_syncs"] == 0


def test_stored_bytes_warning_keeps_the_semantics():
    """warn_stored_bytes only reports: past the threshold one RuntimeWarning names the bytes, and
    every sync still copies the current weights (the default, uncapped semantics); stats() carries
    the stored and peak generation counts and bytes."""
    topo = Topology.example("abilene")
    R = 64
    tr = QRoutingTrainer(topo, "buffer", seed=4, device="cpu", n_replicas=R, sync_step=0.01, batch_size=4)
    gb = tr.generation_bytes
    assert gb == sum(t.numel() * t.element_size() for t in tr.q.state_dict().values()) > 0
    tr.warn_stored_bytes = 3 * gb
    rng = np.random.default_rng(7)
    clock = np.zeros(R)
    speed = rng.random(R) * 0.004
    g = torch.Generator().manual_seed(2)
    import warnings as _w
    with _w.catch_warnings(record=True) as caught:
        _w.simplefilter("always")
        for step in range(40):
            clock += speed
            tr.advance_clock(torch.from_numpy((clock * 1e9).astype(np.int64)))
            v0 = tr.version
            tr.check_sync()
            if tr.version != v0:
                cur = tr.q.state_dict()
                for k, t in tr.weights_of(tr.version).items():
                    assert torch.equal(t, cur[k]), (step, k)
            with torch.no_grad():
                for p in tr.q.parameters():
                    p.add_(1e-3 * torch.randn(p.shape, generator=g))
    msgs = [str(w.message) for w in caught if "warn_stored_bytes" in str(w.message)]
    assert len(msgs) == 1, msgs
    st = tr.stats()
    assert st["peak_generations"] > 3 and st["peak_stored_bytes"] == st["peak_generations"] * gb
    assert st["stored_bytes"] == st["stored_generations"] * gb <= st["peak_stored_bytes"]
    assert tr.stale_syncs == 0


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")
def test_stored_generations_at_4096_abilene_replicas():
    """The trainer's stored weight generations in a training run at the headline's replica count
    (4 096 Abilene replicas, the engine in external-action mode, an optimizer step every 4 env
    steps, syncs every 20 ms of each replica's simulated clock, "ideal" signalling; the default
    uncapped semantics). A copy lives until its (replica, node) syncs twice more, so the generations
    alive at once span about two sync periods of the slowest replica, not the replica count: the
    peak is bounded by the optimizer steps of that window. Stated bound for this run: 64
    generations (the run makes 150 optimizer steps)."""
    from prisma_amd.env import VecRoutingEnv
    from prisma_amd.trainer import train
    R, steps, every = 4096, 600, 4
    env = VecRoutingEnv("abilene", n_replicas=R, sim_time_s=60.0, ping_as_obs=0)
    tr = QRoutingTrainer(env.topo, "buffer", batch_size=512, buffer_size=50000, seed=0, n_replicas=R,
                         sync_step=0.02)
    losses = train(env, tr, steps=steps, train_every=every)
    env.close()
    st = tr.stats()
    print(f"\n[trainer] R={R}: {steps} env steps, {int(tr.steps.max())} optimizer steps, sim clock "
          f"{tr.clock.min():.3f}-{tr.clock.max():.3f} s, syncs (versions) {tr.version}, stored generations "
          f"{st['stored_generations']} ({st['stored_bytes']} B), peak {st['peak_generations']} "
          f"({st['peak_stored_bytes']} B, {tr.generation_bytes} B each)")
    assert losses and np.all(np.isfinite(losses))
    assert tr.version > 20                                   # many syncs happened
    assert st["peak_generations"] <= 64 and st["peak_stored_bytes"] == st["peak_generations"] * tr.generation_bytes
    assert st["stale_syncs"] == 0


def test_trainer_stats_tblog(tmp_path):
    from prisma_amd import tblog
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "buffer", seed=0, device="cpu")
    w = tblog.EventFileWriter(str(tmp_path))
    tblog.trainer_stats_writer(w, tr, 3)
    w.close()
    tags = {t for e in tblog.read_events(w.path) for (t, _, _) in e["values"]}
    assert tags == {f"trainer/{k}" for k in tr.stats()}


def test_trainer_replica_count_must_match_the_env():
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "buffer", seed=0, device="cpu", n_replicas=4)
    with pytest.raises(ValueError, match="n_replicas=4"):
        tr.advance_clock(torch.zeros(8, dtype=torch.int64))


def test_old_episode_hop_transitions_are_not_queued_and_sync_every_warns():
    """A step that crosses a replica's episode end reports its last old-episode transitions:
    they are not queued into the new episode (agent.py:141-145 drops the upcoming events)."""
    topo = Topology.example("abilene")
    tr = QRoutingTrainer(topo, "buffer", seed=6, device="cpu", signaling_type="NN", batch_size=4, n_replicas=2)
    obs = torch.zeros((2, topo.obs_width), dtype=torch.int32)
    b = {"node": torch.tensor([3, 3], dtype=torch.int32), "obs": obs, "next_obs": obs,
         "action": torch.tensor([0, 0], dtype=torch.int32), "reward": torch.zeros(2, dtype=torch.float64),
         "done": torch.zeros(2, dtype=torch.bool), "replica": torch.tensor([0, 1], dtype=torch.int32),
         "uid": torch.tensor([5, 6]), "hop": torch.ones(2, dtype=torch.bool),
         "t_ns": torch.tensor([1_000_000, 1_000_000]), "episode": torch.tensor([0, 0])}
    tr.on_step(torch.zeros((2, topo.obs_width), dtype=torch.int32),
               {"transitions": b, "now_ns": torch.tensor([2_000_000, 3_000]), "episode": torch.tensor([0, 1])})
    assert tr._pend_key.numel() == 1 and int(tr._pend["replica"][0]) == 0
    from prisma_amd.trainer import train

    class _Env:
        def reset(self):
            raise RuntimeError("reached")
    with pytest.warns(DeprecationWarning, match="sync_step"), pytest.raises(RuntimeError, match="reached"):
        train(_Env(), tr, 1, sync_every=5)
