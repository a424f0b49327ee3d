"""GPU replay buffers and the Q-routing DQN trainer.

The reference learns with one TF agent per overlay node, fed by its Forwarder thread
and trained asynchronously by a Trainer thread (prisma/source/trainer.py:28-171,
learner.py:162-228, replay_buffer.py:12-86).  Here the same math runs batched over all
nodes on the device, fed by ``VecRoutingEnv.transitions()``:

* ``ReplayBuffers`` — one FIFO ring of ``size`` transitions per node
  (replay_buffer.py:29-37: append until full, then overwrite the oldest;
  ``Agent.replay_buffer[index]``), stored as [N, size, ...] tensors; ``sample`` draws
  ``batch_size`` indices uniformly per node (replay_buffer.py:55-76).
* ``QRoutingTrainer.train_step`` — for every node whose buffer has received at least
  ``batch_size`` transitions (trainer.py:42): the Q-routing target of each sampled
  transition is ``r + gamma * (1 - done) * min_a' Q'_v(s', a')`` evaluated by the
  target network of the NEXT node v (the neighbour the action led to, ``ideal``
  signalling: learner.py:231-255), with v's interface back to this node filtered out
  (trainer.py:60-72); the loss is the Huber loss of ``Q_u(s, a) - target``
  (learner.py:81-87,171-179) averaged per node; each node's weights take one Keras-Adam
  step (learner.py:104, TF 2.8 defaults beta1 0.9, beta2 0.999, epsilon 1e-7 on the
  uncorrected second moment).  Nodes that do not train keep their weights and Adam
  state untouched, as separate per-node optimizers would.
* ``sync`` copies the online networks into the target networks (trainer.py:101-112;
  with ``ideal`` signalling every node's copy of a neighbour equals that neighbour's
  network at the last sync, so one stacked target copy serves all nodes).
* ``act`` is epsilon-greedy with the reference's ``LinearSchedule`` over each node's own
  transition count (forwarder.py:129-142, utils.py:101-124: 1.0 -> 0.1 over
  ``iterationNum`` = 3000 transitions).

Deliberate differences (documented in DESIGN.md): the reference's trainer threads wake at
random times (trainer.py:34); here the caller decides when all nodes train together.
When v's only interface leads back (degree 1) the filtered minimum is empty; TF's
``reduce_min`` returns +inf there and ``(1 - done) * inf`` makes the target NaN for
``done`` transitions -- here a done transition's target is its reward and an empty
minimum of a non-done one is +inf (its Huber gradient stays finite).
"""
from __future__ import annotations

import copy
from typing import Optional

import numpy as np
import torch

from .policies import StackedQNet
from .topology import Topology


class ReplayBuffers:
    def __init__(self, n_nodes: int, size: int, obs_width: int, device="cuda"):
        self.N, self.size, self.W = int(n_nodes), int(size), int(obs_width)
        z = lambda *s, dt: torch.zeros(*s, dtype=dt, device=device)
        self.obs = z(self.N, self.size, self.W, dt=torch.int32)
        self.next_obs = z(self.N, self.size, self.W, dt=torch.int32)
        self.action = z(self.N, self.size, dt=torch.int64)
        self.reward = z(self.N, self.size, dt=torch.float32)
        self.done = z(self.N, self.size, dt=torch.bool)
        self.next_idx = z(self.N, dt=torch.int64)
        self.count = z(self.N, dt=torch.int64)          # len(storage)
        self.total = z(self.N, dt=torch.int64)          # total_samples
        self.device = device

    def add(self, tr: dict):
        """Append transitions (dict of device tensors with a ``node`` field, in the order
        the Forwarders would have added them) to their node's ring."""
        node = tr["node"].to(self.device).long()
        n = node.numel()
        if n == 0:
            return
        order = torch.sort(node, stable=True).indices
        nd = node[order]
        counts = torch.bincount(nd, minlength=self.N)
        first = torch.cumsum(counts, 0) - counts
        rank = torch.arange(n, device=self.device) - first[nd]
        keep = rank >= counts[nd] - self.size          # an overflowing batch keeps its last `size`
        src = order[keep]
        u = nd[keep]
        slot = (self.next_idx[u] + rank[keep]) % self.size
        self.obs[u, slot] = tr["obs"][src].to(torch.int32)
        self.next_obs[u, slot] = tr["next_obs"][src].to(torch.int32)
        self.action[u, slot] = tr["action"][src].long()
        self.reward[u, slot] = tr["reward"][src].to(torch.float32)
        self.done[u, slot] = tr["done"][src].bool()
        self.next_idx = (self.next_idx + counts) % self.size
        self.count = torch.clamp(self.count + counts, max=self.size)
        self.total += counts

    def sample(self, batch_size: int, generator: Optional[torch.Generator] = None):
        """Uniform indices in [0, len) per node: tensors [N, batch_size, ...]."""
        r = torch.rand((self.N, batch_size), generator=generator, device=self.device, dtype=torch.float64)
        idx = torch.clamp((r * self.count.clamp_min(1)[:, None]).long(), max=self.size - 1)
        g = lambda t: torch.gather(t, 1, idx.view(self.N, batch_size, *([1] * (t.dim() - 2))).expand(
            self.N, batch_size, *t.shape[2:]))
        return g(self.obs), g(self.action), g(self.reward), g(self.next_obs), g(self.done)


def huber(x: torch.Tensor, delta: float = 1.0) -> torch.Tensor:
    """learner.py:81-87 (the quadratic branch on the clamped error, so an infinite error --
    an empty filtered minimum -- has the linear branch's finite gradient, not 0 * inf)."""
    ax = x.abs()
    xq = torch.clamp(x, -delta, delta)
    return torch.where(ax < delta, 0.5 * xq * xq, delta * (ax - 0.5 * delta))


class LinearSchedule:
    """utils.py:101-124 (baselines): p = initial + min(t / T, 1) * (final - initial)."""

    def __init__(self, schedule_timesteps: int = 3000, initial_p: float = 1.0, final_p: float = 0.1):
        self.T, self.p0, self.p1 = schedule_timesteps, initial_p, final_p

    def value(self, t):
        frac = torch.clamp(t.to(torch.float64) / self.T, max=1.0)
        return self.p0 + frac * (self.p1 - self.p0)


class QRoutingTrainer:
    def __init__(self, topo: Topology, kind: str = "buffer", lr: float = 1e-4, gamma: float = 1.0,
                 batch_size: int = 512, buffer_size: int = 50000, seed: int = 0, device="cuda",
                 iteration_num: int = 3000, eps_initial: float = 1.0, eps_final: float = 0.1):
        self.topo = topo
        self.device = torch.device(device)
        self.q = StackedQNet(topo, kind, seed=seed, device=self.device)
        self.q_target = copy.deepcopy(self.q)
        for p in self.q_target.parameters():
            p.requires_grad_(False)
        self.lr, self.gamma, self.batch_size = float(lr), float(gamma), int(batch_size)
        self.beta1, self.beta2, self.eps = 0.9, 0.999, 1e-7      # tf.keras.optimizers.Adam defaults
        self.params = list(self.q.parameters())
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        N, D = topo.n_nodes, topo.max_deg
        self.steps = torch.zeros(N, dtype=torch.int64, device=self.device)       # Adam step per node
        self.buffers = ReplayBuffers(N, buffer_size, topo.obs_width, self.device)
        # next node of (u, a) and the action of that node leading back to u
        nbr = torch.zeros((N, D), dtype=torch.int64)
        back = torch.full((N, D), -1, dtype=torch.int64)
        for u in range(N):
            nb = topo.neighbors(u)
            for a, v in enumerate(nb):
                nbr[u, a] = v
                nv = topo.neighbors(v)
                back[u, a] = nv.index(u) if u in nv else -1
        self.nbr, self.back = nbr.to(self.device), back.to(self.device)
        self.deg = torch.from_numpy(topo.degrees.astype(np.int64)).to(self.device)
        self.explore = LinearSchedule(iteration_num, eps_initial, eps_final)
        self.transitions_seen = torch.zeros(N, dtype=torch.int64, device=self.device)
        self.gen = torch.Generator(device=self.device).manual_seed(int(seed) + 1)

    # -- acting ---------------------------------------------------------------
    @torch.no_grad()
    def act(self, obs: torch.Tensor, node: torch.Tensor, explore: bool = True) -> torch.Tensor:
        """argmin_a Q (learner.py:142-159), epsilon-greedy per the deciding node's schedule."""
        node = node.long().clamp_min(0)
        a = self.q.act(obs, node).long()
        if explore:
            eps = self.explore.value(self.transitions_seen[node])
            r = torch.rand(node.shape, generator=self.gen, device=self.device, dtype=torch.float64)
            ra = (torch.rand(node.shape, generator=self.gen, device=self.device, dtype=torch.float64)
                  * self.deg[node].clamp_min(1)).long()
            a = torch.where(r < eps, ra, a)
        return a.to(torch.int32)

    def observe(self, tr: dict):
        self.buffers.add(tr)
        self.transitions_seen += torch.bincount(tr["node"].long(), minlength=self.topo.n_nodes)

    # -- learning -------------------------------------------------------------
    def targets(self, node, action, reward, next_obs, done) -> torch.Tensor:
        """r + gamma * (1 - done) * min over the next node's filtered actions of its target Q."""
        v = self.nbr[node, action]
        qn = self.q_target.q_values(next_obs, v)                      # [B, D], padding = +inf
        bk = self.back[node, action]
        hit = torch.arange(qn.shape[1], device=qn.device)[None, :] == bk[:, None]
        qn = qn.masked_fill(hit, float("inf"))
        best = qn.min(dim=1).values
        return torch.where(done, reward, reward + self.gamma * best)

    def train_step(self) -> Optional[torch.Tensor]:
        """One gradient step on every node whose buffer received >= batch_size transitions.
        Returns the per-node mean Huber loss (nan for nodes that did not train)."""
        N, B = self.topo.n_nodes, self.batch_size
        ready = (self.buffers.total >= B) & (self.deg > 0)
        if not bool(ready.any()):
            return None
        obs, act, rew, nobs, done = self.buffers.sample(B, self.gen)
        node = torch.arange(N, device=self.device).repeat_interleave(B)
        obs, act, rew = obs.reshape(N * B, -1), act.reshape(-1), rew.reshape(-1)
        nobs, done = nobs.reshape(N * B, -1), done.reshape(-1)
        with torch.no_grad():
            tgt = self.targets(node, act, rew, nobs, done)
        q = self.q.q_values(obs, node)
        qsel = q.gather(1, act[:, None]).squeeze(1)
        per = huber(qsel - tgt).view(N, B).mean(dim=1)               # tf.reduce_mean per node
        loss = torch.where(ready, per, torch.zeros_like(per)).sum()
        for p in self.params:
            p.grad = None
        loss.backward()
        self._adam(ready)
        return torch.where(ready, per.detach(), torch.full_like(per, float("nan")))

    @torch.no_grad()
    def _adam(self, ready: torch.Tensor):
        """Keras Adam per node: lr_t = lr sqrt(1 - b2^t) / (1 - b1^t);
        p -= lr_t m / (sqrt(v) + eps), applied only to the rows of nodes that trained."""
        self.steps += ready.long()
        t = self.steps.to(torch.float64)
        lr_t = (self.lr * torch.sqrt(1 - self.beta2 ** t) / (1 - self.beta1 ** t)).to(torch.float32)
        for p, m, v in zip(self.params, self.m, self.v):
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            sh = (-1,) + (1,) * (p.dim() - 1)
            r = ready.view(sh)
            m.copy_(torch.where(r, self.beta1 * m + (1 - self.beta1) * g, m))
            v.copy_(torch.where(r, self.beta2 * v + (1 - self.beta2) * g * g, v))
            upd = lr_t.nan_to_num(0.0).view(sh) * m / (torch.sqrt(v) + self.eps)
            p.copy_(torch.where(r, p - upd, p))

    @torch.no_grad()
    def sync(self):
        self.q_target.load_state_dict(self.q.state_dict())


def train(env, trainer: QRoutingTrainer, steps: int, train_every: int = 1, sync_every: int = 100):
    """Drive a VecRoutingEnv (external-action mode) with the trainer's epsilon-greedy
    policy: each step applies one action per replica, adds the completed transitions to
    the buffers, and trains every ``train_every`` steps; returns per-step mean losses."""
    obs, info = env.reset()
    losses = []
    for s in range(steps):
        a = trainer.act(obs, info["node"])
        obs, _, _, info = env.step(a)
        trainer.observe(info["transitions"])
        if s % train_every == 0:
            per = trainer.train_step()
            if per is not None:
                losses.append(float(torch.nanmean(per)))
        if (s + 1) % sync_every == 0:
            trainer.sync()
    return losses
