"""Replay buffers and the Q-routing trainer (prisma_amd/trainer.py) against the
reference's own ReplayBuffer (fixture) and restatements of learner.py / trainer.py math, on CPU."""
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
    tr = QRoutingTrainer(env.topo, "buffer", batch_size=64, buffer_size=4096, seed=0)
    w0 = tr.q.W2.detach().clone()
    losses = train(env, tr, steps=200, train_every=4, sync_every=50)
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
    counter = np.zeros(11, dtype=int)
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
    tr = QRoutingTrainer(topo, "buffer", seed=6, device="cpu", signaling_type=kind, batch_size=4)
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
                         nn_max_seg_index=1024 // 512 - 1)
    losses = train(env, tr, steps=600, train_every=4, sync_every=20)
    env.close()
    assert losses and np.all(np.isfinite(losses))
    assert int(tr.buffers.total.sum()) > 0
    assert bool((tr.tgt_ver > 0).any())
