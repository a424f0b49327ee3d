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

Signalling types (argument_parser.py:72, with the simulated signalling of run_ns3.py's
``signalingSim=1``, i.e. an engine with ``train=1, notify_dest=1`` and, for "NN",
``big_signaling=1``):

* "ideal" -- as above: a hop transition enters node u's buffer when it completes, and every
  node's copy of a neighbour is that neighbour's network at the last sync.
* "NN" (forwarder.py:380-391, 251-263; trainer.py:101-171; learner.py:231-295) -- a hop
  transition waits until the small-signalling echo of its packet is back at u
  (``_get_upcoming_events_real``: lost echoes lose their transition); u keeps per neighbour i
  a target copy, an upcoming copy and the one before (temp): every sync moves upcoming to
  temp and takes the neighbour's current network as upcoming, and the target copy changes
  only when the neighbour's NN arrives over big signalling (segment index
  ``nn_max_seg_index``): to temp if the NN index is u's sync counter - 1, else to upcoming.
  Copies are versions of the stacked online networks (one snapshot per sync).
* "target" (forwarder.py:393-410, trainer.py:52-55) -- the next node v computes the target
  ``r + gamma (1 - done) min_filtered Q_v(s')`` with its ONLINE network when it is notified
  (learner.py:199-229), the transition carries it back on the echo and the training step
  uses it as is.

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
                 iteration_num: int = 3000, eps_initial: float = 1.0, eps_final: float = 0.1,
                 signaling_type: str = "ideal", nn_max_seg_index: int = 35328 // 512 - 1,
                 pending_cap: int = 1 << 20):
        if signaling_type not in ("ideal", "NN", "target"):
            raise ValueError("signaling_type must be 'ideal', 'NN' or 'target'")
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
        # signalling (module docstring)
        self.signaling = signaling_type
        self.nn_max_seg = int(nn_max_seg_index)       # agent.py:81: bigSignalingSize / packet_size - 1
        self.pending_cap = int(pending_cap)
        self._pend = None                             # hop transitions waiting for their echo
        self._pend_key = None
        self.snapshots = {0: self._snapshot()}        # version -> stacked online weights
        self.version = 0
        self.tgt_ver = torch.zeros((N, D), dtype=torch.int64)      # host: per (node, action) copy
        self.up_ver = torch.zeros((N, D), dtype=torch.int64)
        self.tmp_ver = torch.zeros((N, D), dtype=torch.int64)
        self.sync_counter = np.zeros(N, dtype=np.int64)
        self._eval = copy.deepcopy(self.q)
        for p in self._eval.parameters():
            p.requires_grad_(False)

    # -- acting ---------------------------------------------------------------
    @torch.no_grad()
    def act(self, obs: torch.Tensor, node: torch.Tensor, explore: bool = True) -> torch.Tensor:
        """argmin_a Q (learner.py:142-159), epsilon-greedy per the deciding node's schedule."""
        node = node.long().clamp_min(0)
        ctrl = obs[:, 0] == 1000                       # control notification: the action is ignored
        if bool(ctrl.any()):
            obs = obs.clone()
            obs[ctrl, 0] = 0
        a = self.q.act(obs, node).long()
        if explore:
            eps = self.explore.value(self.transitions_seen[node])
            r = torch.rand(node.shape, generator=self.gen, device=self.device, dtype=torch.float64)
            ra = (torch.rand(node.shape, generator=self.gen, device=self.device, dtype=torch.float64)
                  * self.deg[node].clamp_min(1)).long()
            a = torch.where(r < eps, ra, a)
        return a.to(torch.int32)

    def observe(self, tr: dict):
        """Completed transitions (VecRoutingEnv.transitions()).  "ideal": into the buffers at
        once; "NN" / "target": loss transitions at once (forwarder.py:214-244), hop transitions
        when their echo is back (on_control)."""
        if self.signaling == "ideal" or "hop" not in tr:
            self._add(tr)
            return
        hop = tr["hop"].to(self.device)
        self._add({k: t[~hop.to(t.device)] for k, t in tr.items()})
        h = {k: t[hop.to(t.device)].to(self.device) for k, t in tr.items()}
        if h["node"].numel() == 0:
            return
        if self.signaling == "target":                # v's target, computed when v is notified
            with torch.no_grad():
                h["reward"] = self._bootstrap(self.q, h["node"].long(), h["action"].long(),
                                              h["reward"].to(torch.float32), h["next_obs"], h["done"].bool())
        key = self._key(h["replica"], h["node"], h["uid"])
        if self._pend is None:
            self._pend, self._pend_key = h, key
        else:
            self._pend = {k: torch.cat([self._pend[k], h[k].to(self._pend[k].dtype)]) for k in self._pend}
            self._pend_key = torch.cat([self._pend_key, key])
        extra = self._pend_key.numel() - self.pending_cap
        if extra > 0:                                 # echoes that never came back: oldest first
            self._pend = {k: t[extra:] for k, t in self._pend.items()}
            self._pend_key = self._pend_key[extra:]

    def _add(self, tr: dict):
        if tr["node"].numel() == 0:
            return
        self.buffers.add(tr)
        self.transitions_seen += torch.bincount(tr["node"].long().to(self.device), minlength=self.topo.n_nodes)

    @staticmethod
    def _key(replica, node, uid):
        """(replica, node, uid mod 2^21): the engine's echo carries 21 uid bits (engine_layout.h)."""
        return (replica.long() << 29) | (node.long() << 21) | (uid.long() & ((1 << 21) - 1))

    def on_control(self, obs: torch.Tensor, info: dict):
        """Control notifications of a VecRoutingEnv step (obs rows [1000, a, b, c],
        include/prisma.h): an echo releases the hop transition of its packet at this node
        (forwarder.py:246-250); a big-signalling segment that completes a neighbour's NN swaps
        this node's target copy of it (forwarder.py:251-263)."""
        ctrl = info["control"].to(self.device)
        if not bool(ctrl.any()):
            return
        obs = obs.to(self.device)
        node = info["node"].to(self.device).long()
        big = ctrl & ((obs[:, 3] & 0x10000) != 0)
        echo = ctrl & ~big
        if self._pend is not None and bool(echo.any()):
            rep = torch.nonzero(echo).squeeze(1)
            keys = self._key(rep, node[echo], obs[echo, 1].long())
            hit = torch.isin(self._pend_key, keys)
            if bool(hit.any()):
                self._add({k: t[hit] for k, t in self._pend.items()})
                self._pend = {k: t[~hit] for k, t in self._pend.items()}
                self._pend_key = self._pend_key[~hit]
        if self.signaling == "NN" and bool(big.any()):
            rows = obs[big].cpu().numpy()
            for v, (_, nn, seg, c) in zip(node[big].cpu().tolist(), rows[:, :4].tolist()):
                self.on_big_signal(v, int(self.topo.overlay_nodes[c & 0xFFFF]), nn, seg)

    def on_big_signal(self, v: int, src: int, nn_index: int, seg_index: int):
        """Node v received segment seg_index of NN nn_index of neighbour src (underlay id)."""
        if seg_index > self.nn_max_seg:
            raise ValueError(f"segIndex > {self.nn_max_seg}")       # forwarder.py:256-257
        if seg_index != self.nn_max_seg:
            return
        i = self.topo.neighbors(v).index(src)
        if nn_index == self.sync_counter[v] - 1:                   # agent.py:168-175, with_temp
            self.tgt_ver[v, i] = self.tmp_ver[v, i]
        else:
            self.tgt_ver[v, i] = self.up_ver[v, i]
        self._gc()

    # -- learning -------------------------------------------------------------
    def targets(self, node, action, reward, next_obs, done) -> torch.Tensor:
        """r + gamma * (1 - done) * min over the next node's filtered actions of its target Q
        ("NN": node u's copy of that neighbour; "ideal": the stacked target networks)."""
        if self.signaling != "NN":
            return self._bootstrap(self.q_target, node, action, reward, next_obs, done)
        ver = self.tgt_ver.to(node.device)[node, action]
        out = torch.empty_like(reward)
        for k in torch.unique(ver).tolist():
            sel = ver == k
            self._eval.load_state_dict(self.snapshots[int(k)])
            out[sel] = self._bootstrap(self._eval, node[sel], action[sel], reward[sel], next_obs[sel], done[sel])
        return out

    def _bootstrap(self, net, node, action, reward, next_obs, done) -> torch.Tensor:
        v = self.nbr[node, action]
        qn = net.q_values(next_obs, v)                                 # [B, D], padding = +inf
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
            # "target" signalling: the buffer holds the targets the next nodes computed
            tgt = rew if self.signaling == "target" else self.targets(node, act, rew, nobs, done)
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
        """trainer.py:101-171 for every node: "ideal" -- each copy of a neighbour becomes its
        current network; "NN" -- the upcoming copies move to temp and take the neighbours'
        current networks, the target copies wait for the NN over big signalling; "target" --
        each node's own target network is refreshed (update_target)."""
        self.q_target.load_state_dict(self.q.state_dict())
        if self.signaling != "NN":
            return
        self.version += 1
        self.snapshots[self.version] = self._snapshot()
        self.tmp_ver.copy_(self.up_ver)
        self.up_ver.fill_(self.version)
        self.sync_counter += 1
        self._gc()

    def _snapshot(self) -> dict:
        return {k: t.detach().clone() for k, t in self.q.state_dict().items()}

    def _gc(self):
        live = set(torch.cat([self.tgt_ver.view(-1), self.up_ver.view(-1), self.tmp_ver.view(-1)]).tolist())
        for k in [k for k in self.snapshots if k not in live]:
            del self.snapshots[k]


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
        trainer.on_control(obs, info)
        if s % train_every == 0:
            per = trainer.train_step()
            if per is not None:
                losses.append(float(torch.nanmean(per)))
        if (s + 1) % sync_every == 0:
            trainer.sync()
    return losses
