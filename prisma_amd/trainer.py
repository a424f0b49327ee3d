"""GPU replay buffers and the Q-routing DQN trainer.

The reference learns with one TF agent per overlay node, fed by its Forwarder thread
and trained asynchronously by a Trainer thread (prisma/source/trainer.py:28-171,
learner.py:162-228, replay_buffer.py:12-86, 393-534).  Here the same math runs batched over all
nodes on the device, fed by ``VecRoutingEnv`` steps (``QRoutingTrainer.on_step``):

* ``ReplayBuffers`` -- one FIFO ring of ``size`` transitions per node
  (replay_buffer.py:29-37: append until full, then overwrite the oldest;
  ``Agent.replay_buffer[index]``), stored as [N, size, ...] tensors; ``sample`` draws
  ``batch_size`` indices uniformly per node (replay_buffer.py:55-76).  With
  ``prioritized=True`` it is the reference's ``PrioritizedReplayBuffer`` (alpha 1, one
  priority class per neighbour, agent.py:66-67): each slot's sum-tree priority, the prio of
  the FIRST transition ever written to the slot (``original_prios`` is appended to and
  indexed by slot, so later writes never replace it), the slots ever written under each
  action (``neighbors_idx``), ``latest_gradient_step`` per action and ``_max_priority``;
  ``sample`` returns the importance weights ``prio[idx] / sum(prio) * len`` of uniformly
  drawn indices (replay_buffer.py:469-503), and the loss is weighted by them (learner.py:179).
  Pinned by a fixture generated from the reference class (tests/golden/make_prio_replay_golden.py).
* ``QRoutingTrainer.train_step`` -- for every node whose buffer has received at least
  ``batch_size`` transitions (trainer.py:42): the Q-routing target of each sampled
  transition is ``r + gamma * (1 - done) * min_a' Q'_v(s', a')`` evaluated by node u's copy
  of the NEXT node v's network (learner.py:231-255), with v's interface back to u filtered out
  (trainer.py:60-72); the loss is the importance-weighted Huber loss of ``Q_u(s, a) - target``
  (learner.py:81-87,171-179) averaged per node; each node's weights take one Keras-Adam
  step (learner.py:104, TF 2.8 defaults beta1 0.9, beta2 0.999, epsilon 1e-7 on the
  uncorrected second moment).  Nodes that do not train keep their weights and Adam
  state untouched, as separate per-node optimizers would.
* ``act`` is epsilon-greedy with the reference's ``LinearSchedule`` over each node's own
  transition count (forwarder.py:129-142, utils.py:101-124: 1.0 -> 0.1 over
  ``iterationNum`` = 3000 transitions).

Time.  The reference runs ONE simulation and its agents read one clock, ``Agent.curr_time``,
the time of the latest notification.  Here every replica is its own simulation: the trainer
keeps a clock per replica (the engine's clock at that replica's latest notification), and
everything the reference schedules in simulated time is kept per replica: the sync counters
and each node's copies of its neighbours' networks, the upcoming-event queues.  The networks
themselves are shared by all replicas (the per-node agents learn from every replica's
transitions); a copy is a version number into snapshots of the stacked online networks.

Syncs (trainer.py:101-112): node u of replica r syncs when its clock passes
``(sync_counter + 1) * sync_step`` (sync counters start at -1, forwarder.py:123, so the first
sync is at the first notification): the upcoming copy of every neighbour moves to temp and
takes the neighbour's current network, then the counter advances; with "ideal" signalling the
target copies take the upcoming ones at once.  ``sync_step < 0`` sizes the step from the
control/data ratio ``sync_ratio`` (trainer.py:114-134).

Signalling types (argument_parser.py:72) and where the signalling happens (``signalingSim``,
argument_parser.py:41):

* "ideal" -- a hop transition enters node u's buffer when it completes.
* "NN" -- a hop transition reaches u's buffer only through the small-signalling packet that
  the next node v sends back; u keeps per neighbour i a target copy, an upcoming copy and the
  one before (temp), and the target copy changes only when neighbour i's whole NN has reached
  u through big signalling.
  - signalingSim=1 (the engine simulates the packets: ``train=1, notify_dest=1,
    big_signaling=1``): the echo of the packet releases the transition
    (``_get_upcoming_events_real``, forwarder.py:477-490: the first queued match; lost echoes
    lose it); the NN's last segment (``nn_max_seg_index``) sets the target copy to temp if the
    NN index is u's sync counter - 1, else to upcoming (forwarder.py:251-263).
  - signalingSim=0 (the reference's default: the agents model the delays). RECONSTRUCTION OF
    INTENT, parity unpinned: in the reference this path cannot run. Trainer.run calls
    self._get_upcoming_events, which only Forwarder defines; Trainer._sync_all uses
    self._push_upcoming_event and self.big_signaling_delay, which Trainer lacks; Forwarder calls
    self._compute_sync_step, which only Trainer defines (each an AttributeError), and
    trainer.py:106 reads the class attribute Agent.sync_step (-1), not the per-node value
    computed from it. What follows is the behaviour those lines evidently intend: the transition is
    queued at u for ``now + small_signaling_delay(v)`` with the packet size
    64 + 8 + 8 (deg(v) + 1) bytes (forwarder.py:101-103, 380-391), and every sync of u queues,
    per neighbour, the arrival of that neighbour's NN at ``now + big_signaling_delay(u)``
    (trainer.py:160-167; nn_size = trainable parameters x 32 bits, forwarder.py:94-98); queued
    events are released once u's clock has reached them (``_get_upcoming_events``,
    forwarder.py:444-464), a released NN setting the target copy to upcoming.
* "target" (forwarder.py:393-410, trainer.py:52-55) -- the next node v computes the target
  ``r + gamma (1 - done) min_filtered Q_v(s')`` with its ONLINE network when it is notified
  (learner.py:199-229); the transition carries it back (signalingSim=1: on the echo;
  signalingSim=0: queued for ``now + small_signaling_delay``, packet 64 + 8 + 8 bytes) and the
  training step uses it as is.  With the prioritized buffer it carries the gradient step of v's
  network as its priority, and a newer one raises ``latest_gradient_step`` and re-weights the
  action's slots (forwarder.py:495-505).

Deliberate differences (documented in DESIGN.md): the reference's trainer threads wake at
random times (trainer.py:34); here the caller decides when all nodes train together, and the
sync / release checks run at every ``on_step``.  When v's only interface leads back (degree 1)
the filtered minimum is empty; TF's ``reduce_min`` returns +inf there and ``(1 - done) * inf``
makes the target NaN for ``done`` transitions -- here a done transition's target is its reward
and an empty minimum of a non-done one is +inf (its Huber gradient stays finite).  The
reference never gives a queued "target" transition its "gradient_step" (forwarder.py:501 reads
a key nothing sets) and adds hop transitions of the other types without a priority (a
TypeError with the prioritized buffer): here those get v's gradient step, resp. the action's
latest gradient step (priority 1, as the loss transitions of forwarder.py:227-233).
"""
from __future__ import annotations

import copy
import warnings
from typing import Optional

import numpy as np
import torch

from .policies import StackedQNet
from .topology import Topology


class ReplayBuffers:
    def __init__(self, n_nodes: int, size: int, obs_width: int, device="cuda", prioritized: bool = False,
                 max_deg: int = 1, alpha: float = 1.0):
        self.N, self.size, self.W = int(n_nodes), int(size), int(obs_width)
        z = lambda *s, dt: torch.zeros(*s, dtype=dt, device=device)
        self.obs = z(self.N, self.size, self.W, dt=torch.int32)
        self.next_obs = z(self.N, self.size, self.W, dt=torch.int32)
        self.action = z(self.N, self.size, dt=torch.int64)
        self.reward = z(self.N, self.size, dt=torch.float32)
        self.done = z(self.N, self.size, dt=torch.bool)
        self.replica = z(self.N, self.size, dt=torch.int64)   # which simulation a transition came from
        self.next_idx = z(self.N, dt=torch.int64)
        self.count = z(self.N, dt=torch.int64)          # len(storage)
        self.total = z(self.N, dt=torch.int64)          # total_samples
        self.device = device
        self.prioritized = bool(prioritized)
        if self.prioritized:
            D = max(int(max_deg), 1)
            self.alpha = float(alpha)
            self.prio = z(self.N, self.size, dt=torch.float64)        # sum-tree leaves (== min-tree leaves)
            self.orig = z(self.N, self.size, dt=torch.float64)        # original_prios[slot]
            self.member = z(self.N, D, self.size, dt=torch.bool)      # neighbors_idx[action] as slot sets
            self.latest = torch.ones((self.N, D), dtype=torch.int64, device=device)   # latest_gradient_step
            self.max_prio = torch.ones(self.N, dtype=torch.float64, device=device)   # _max_priority

    def add(self, tr: dict):
        """Append transitions (dict of device tensors with a ``node`` field, in the order
        the Forwarders would have added them) to their node's ring.  With the prioritized
        buffer, ``tr["prio"]`` is each transition's priority (default: the action's latest
        gradient step, forwarder.py:227-233)."""
        node = tr["node"].to(self.device).long()
        n = node.numel()
        if n == 0:
            return
        order = torch.sort(node, stable=True).indices
        nd = node[order]
        counts = torch.bincount(nd, minlength=self.N)
        first = torch.cumsum(counts, 0) - counts
        rank = torch.arange(n, device=self.device) - first[nd]
        slot_all = (self.next_idx[nd] + rank) % self.size
        keep = rank >= counts[nd] - self.size          # an overflowing batch keeps its last `size`
        src = order[keep]
        u = nd[keep]
        slot = slot_all[keep]
        act = tr["action"].to(self.device).long()
        self.obs[u, slot] = tr["obs"][src].to(self.device, torch.int32)
        self.next_obs[u, slot] = tr["next_obs"][src].to(self.device, torch.int32)
        self.action[u, slot] = act[src]
        self.reward[u, slot] = tr["reward"][src].to(self.device, torch.float32)
        self.done[u, slot] = tr["done"][src].to(self.device).bool()
        rep = tr.get("replica")
        self.replica[u, slot] = rep[src].to(self.device).long() if rep is not None else 0
        if self.prioritized:
            a_all = act[order]
            prio = tr.get("prio")
            prio = (self.latest[nd, a_all].to(torch.float64) if prio is None
                    else prio.to(self.device, torch.float64)[order])
            k_all = self.total[nd] + rank                     # the add's number: original_prios index
            fst = k_all < self.size
            self.orig[nd[fst], slot_all[fst]] = prio[fst]
            self.member[nd, a_all, slot_all] = True
            self.prio[u, slot] = self.max_prio[u] ** self.alpha
        self.next_idx = (self.next_idx + counts) % self.size
        self.count = torch.clamp(self.count + counts, max=self.size)
        self.total += counts

    def gradient_step(self, node: int, action: int, step: int):
        """A transition from a newer gradient step of neighbour `action` reached `node`:
        forwarder.py:502-505 + update_priorities (replay_buffer.py:515-534) over the slots ever
        written under that action."""
        if int(step) <= int(self.latest[node, action]):
            return
        self.latest[node, action] = int(step)
        m = self.member[node, action]
        if bool(m.any()):
            vals = (self.orig[node, m] / float(step)) ** self.alpha
            self.prio[node, m] = vals
            self.max_prio[node] = torch.maximum(self.max_prio[node], vals.max())

    def tree_sum(self) -> torch.Tensor:
        """[N] sum-tree roots: the pairwise sums the reference's SumSegmentTree keeps (leaves
        padded to a power of two with zeros), bit for bit."""
        cap = 1
        while cap < self.size:
            cap *= 2
        x = torch.zeros((self.N, cap), dtype=torch.float64, device=self.device)
        x[:, :self.size] = self.prio
        while x.shape[1] > 1:
            x = x[:, 0::2] + x[:, 1::2]
        return x[:, 0]

    def sample_full(self, batch_size: int, generator: Optional[torch.Generator] = None, idx=None) -> dict:
        """Uniform indices in [0, len) per node (or the given idx [N, batch]): tensors
        [N, batch_size, ...] plus the importance weights (ones without priorities)."""
        if idx is None:
            r = torch.rand((self.N, batch_size), generator=generator, device=self.device, dtype=torch.float64)
            idx = torch.clamp((r * self.count.clamp_min(1)[:, None]).long(), max=self.size - 1)
        idx = idx.to(self.device).long()
        g = lambda t: torch.gather(t, 1, idx.view(self.N, batch_size, *([1] * (t.dim() - 2))).expand(
            self.N, batch_size, *t.shape[2:]))
        out = {"obs": g(self.obs), "action": g(self.action), "reward": g(self.reward), "next_obs": g(self.next_obs),
               "done": g(self.done), "replica": g(self.replica), "idx": idx}
        if self.prioritized:
            tot = self.tree_sum()
            out["weights"] = torch.gather(self.prio, 1, idx) / tot.clamp_min(1e-300)[:, None] * \
                self.count.to(torch.float64)[:, None]
        else:
            out["weights"] = torch.ones((self.N, batch_size), dtype=torch.float64, device=self.device)
        return out

    def sample(self, batch_size: int, generator: Optional[torch.Generator] = None):
        s = self.sample_full(batch_size, generator)
        return s["obs"], s["action"], s["reward"], s["next_obs"], s["done"]


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


def convert_bps_to_data_rate(text: str) -> float:
    """utils.py:141-159: the float reading of a traffic-matrix entry ("12.5Kbps" -> 12500.0)."""
    unit = str(text).rstrip("bps")
    names = ("K", "M", "G", "T")
    if unit and unit[-1] in names:
        return float(unit[:-1]) * 1000.0 ** (names.index(unit[-1]) + 1)
    return float(unit)


def nn_param_count(topo: Topology, u: int, kind: str) -> int:
    """Trainable parameters of node u's Keras model (models.py:258-306, 360-392); the
    LayerNormalization has none (center=False, scale=False)."""
    no, d = topo.n_overlay, int(topo.degrees[u])
    n = no * 32 + 32 + 64 * 64 + 64 + 64 * d + d
    return n + ((d * 32 + 32) + (64 * 64 + 64) if kind == "buffer" else (32 * 64 + 64))


class QRoutingTrainer:
    def __init__(self, topo: Topology, kind: str = "buffer", lr: float = 1e-4, gamma: float = 1.0,
                 batch_size: int = 512, buffer_size: int = 50000, seed: int = 0, device="cuda",
                 iteration_num: int = 3000, eps_initial: float = 1.0, eps_final: float = 0.1,
                 signaling_type: str = "ideal", nn_max_seg_index: Optional[int] = None,
                 big_signaling_size: int = 512, packet_size: int = 512, pending_cap: int = 1 << 20,
                 n_replicas: int = 1, signaling_sim: int = 1, sync_step: float = 1.0, sync_ratio: float = 0.1,
                 link_cap: int = 500000, link_delay_ms: float = 1.0, prioritized_replay: bool = False,
                 max_snapshots: Optional[int] = None, warn_stored_bytes: Optional[int] = 1 << 30):
        if signaling_type not in ("ideal", "NN", "target"):
            raise ValueError("signaling_type must be 'ideal', 'NN' or 'target'")
        self.topo = topo
        self.kind = kind
        self.device = torch.device(device)
        self.q = StackedQNet(topo, kind, seed=seed, device=self.device)
        self.lr, self.gamma, self.batch_size = float(lr), float(gamma), int(batch_size)
        self.beta1, self.beta2, self.eps = 0.9, 0.999, 1e-7      # tf.keras.optimizers.Adam defaults
        self.params = list(self.q.parameters())
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        N, D = topo.n_nodes, topo.max_deg
        self.N, self.D = N, D
        self.steps = torch.zeros(N, dtype=torch.int64, device=self.device)       # Adam step per node
        self.prioritized = bool(prioritized_replay)
        self.buffers = ReplayBuffers(N, buffer_size, topo.obs_width, self.device, prioritized=self.prioritized,
                                     max_deg=D)
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
        self.nbr_host = nbr.numpy()
        self.deg = torch.from_numpy(topo.degrees.astype(np.int64)).to(self.device)
        self.deg_host = topo.degrees.astype(np.int64)
        self.explore = LinearSchedule(iteration_num, eps_initial, eps_final)
        self.transitions_seen = torch.zeros(N, dtype=torch.int64, device=self.device)
        self.gen = torch.Generator(device=self.device).manual_seed(int(seed) + 1)
        # ---- signalling (module docstring) ----
        self.signaling = signaling_type
        self.signaling_sim = int(signaling_sim)
        # agent.py:81: bigSignalingSize / packet_size - 1
        self.nn_max_seg = int(big_signaling_size // packet_size - 1) if nn_max_seg_index is None else int(nn_max_seg_index)
        self.pending_cap = int(pending_cap)
        self.link_cap, self.link_delay_s = float(link_cap), float(link_delay_ms) * 0.001
        self.packet_size = int(packet_size)
        self.nn_size = np.array([nn_param_count(topo, u, kind) * 32 if topo.degrees[u] > 0 else 0
                                 for u in range(N)], dtype=np.float64)               # bits, forwarder.py:96
        self.big_delay = self.nn_size / self.link_cap + self.link_delay_s           # forwarder.py:97
        if signaling_type == "NN":                                                   # forwarder.py:101-108
            self.small_size = 64 + 8 + 8 * (self.deg_host + 1)
        else:
            self.small_size = np.full(N, 64 + 8 + 8, dtype=np.int64)
        self.small_delay = self.small_size / self.link_cap + self.link_delay_s
        self.sync_ratio = float(sync_ratio)
        if sync_step < 0:
            self.sync_step = np.array([self.compute_sync_step(u, self.sync_ratio) if topo.degrees[u] > 0 else np.inf
                                       for u in range(N)])
        else:
            self.sync_step = np.full(N, float(sync_step))
        self.small_overhead = 0.0                    # Agent.small_signaling_overhead_counter (bytes)
        self.small_pkts = 0
        self.big_overhead = 0.0                      # Agent.big_signaling_overhead_counter (bits, forwarder.py:96)
        self.big_pkts = 0
        # ---- per-replica simulated time and network copies ----
        self.R = int(n_replicas)
        self.clock = np.zeros(self.R)                # Agent.curr_time per simulation (s)
        self.episode = np.zeros(self.R, dtype=np.int64)
        self.sync_counter = np.full((self.R, N), -1, dtype=np.int64)
        # A copy is a version number; a version maps to one stored generation of the stacked online
        # weights. The weights only change in place (train_step's Adam, a caller's edits), so syncs
        # between two changes share one stored generation (keyed on the parameters' in-place
        # version counters). Replica clocks drift apart, so the live versions grow towards O(R);
        # max_snapshots (opt-in; None = unbounded, every sync copies the current weights as the
        # reference's _sync_all does) caps the stored generations: at the cap a sync takes the
        # newest stored generation instead of the current weights. Such syncs are counted in
        # stale_syncs (stats(), tblog.trainer_stats_writer) and the first one warns.
        self.max_snapshots = None if max_snapshots is None else int(max_snapshots)
        self.stale_syncs = 0                         # syncs that received an older stored generation
        self._stale_warned = False
        # what the stored generations cost: their bytes, the peak count and bytes (stats()), and a
        # one-time warning past warn_stored_bytes (None: never) -- a report, the semantics unchanged
        self.generation_bytes = sum(t.numel() * t.element_size() for t in self.q.state_dict().values())
        self.warn_stored_bytes = None if warn_stored_bytes is None else int(warn_stored_bytes)
        self.peak_generations = 0
        self._bytes_warned = False
        self._gen_w = {}                             # generation key -> stacked weights
        self._snap_gen = {}                          # version -> generation key
        self.version = 0
        self._snap_gen[0] = self._capture()
        self.tgt_ver = np.zeros((self.R, N, D), dtype=np.int64)      # per (replica, node, action) copy
        self.up_ver = np.zeros((self.R, N, D), dtype=np.int64)
        self.tmp_ver = np.zeros((self.R, N, D), dtype=np.int64)
        self._pend = None                            # hop transitions waiting for their echo / arrival time
        self._pend_key = None
        self._pend_time = None
        self._pend_seq = None
        self._seq = 0
        self._big = []                               # signalingSim=0 "NN": (time, seq, replica, node, action)
        self._eval = copy.deepcopy(self.q)
        for p in self._eval.parameters():
            p.requires_grad_(False)

    # -- helpers ----------------------------------------------------------------
    def compute_sync_step(self, u: int, ratio: float = 0.1) -> float:
        """trainer.py:114-134 for node u: nn_size / (data_load * ratio - control_load), the data
        load being the sum of the raw traffic matrix (utils.py convert_bps_to_data_rate, no load
        factor) and the control load one small-signalling packet per data packet."""
        tm = self.topo.tm_strings
        if tm is None:
            raise ValueError("sync_step < 0 needs the topology's traffic matrix (Topology.tm_strings)")
        data = float(np.sum(np.vectorize(convert_bps_to_data_rate)(np.asarray(tm, dtype=object))))
        pkts = data / (self.packet_size * 8)
        control = pkts * float(self.small_size[u])
        return float(self.nn_size[u] / (data * ratio - control))

    @property
    def q_target(self):
        """The networks the "ideal" targets of replica 0 read (the last sync's snapshot)."""
        net = copy.deepcopy(self._eval)
        net.load_state_dict(self.weights_of(int(self.tgt_ver[0].max())))
        return net

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

    # -- one env step -----------------------------------------------------------
    def on_step(self, obs: torch.Tensor, info: dict):
        """Everything the Forwarder and Trainer threads do between two notifications: the
        replicas' clocks move to their new notifications (info["now_ns"]), a replica that
        started a new episode drops its queued signalling, the completed transitions enter the
        buffers or the queues (observe), control notifications release their transitions or
        complete NN copies (on_control), then the releases and syncs that are due run, in the
        Trainer thread's order (trainer.py:33-39)."""
        if "now_ns" in info:
            self.advance_clock(info["now_ns"], info.get("episode"))
        if "transitions" in info:
            self.observe(info["transitions"])
        self.on_control(obs, info)
        self.release_due()                           # Trainer.run: _get_upcoming_events, then _check_sync
        self.check_sync()

    def advance_clock(self, now_ns, episode=None):
        t = np.asarray(now_ns.cpu() if torch.is_tensor(now_ns) else now_ns, dtype=np.float64).reshape(-1) / 1e9
        if t.shape != (self.R,):
            raise ValueError(f"the env reports {t.size} replica clocks but the trainer was built with "
                             f"n_replicas={self.R}: pass QRoutingTrainer(..., n_replicas=env.R)")
        if episode is not None:
            ep = np.asarray(episode.cpu() if torch.is_tensor(episode) else episode, dtype=np.int64).reshape(-1)
            new = ep != self.episode
            if new.any():
                self.new_episode(np.nonzero(new)[0])
                self.episode = ep.copy()
        self.clock = t

    def new_episode(self, replicas):
        """Replicas that started a new episode (Forwarder.reset: sync counters back to -1,
        forwarder.py:123; agent.py:141-145 empties the upcoming events): their queued
        transitions and NN arrivals are dropped; their copies stay."""
        reps = np.asarray(replicas, dtype=np.int64)
        self.sync_counter[reps] = -1
        if self._pend is not None:
            keep = ~torch.isin(self._pend["replica"].long().to(self.device),
                               torch.from_numpy(reps).to(self.device))
            self._take_pending(keep)
        if self._big:
            rs = set(reps.tolist())
            self._big = [e for e in self._big if e[2] not in rs]

    def observe(self, tr: dict):
        """Completed transitions (VecRoutingEnv.transitions()).  "ideal": into the buffers at
        once; "NN" / "target": loss transitions at once (forwarder.py:214-244), hop transitions
        when their small-signalling packet is back (on_control / release_due)."""
        if self.signaling == "ideal" or "hop" not in tr:
            self._add(tr)
            return
        hop = tr["hop"].to(self.device)
        self._add({k: t[~hop.to(t.device)] for k, t in tr.items()})
        h = {k: t[hop.to(t.device)].to(self.device) for k, t in tr.items()}
        if "episode" in h and h["node"].numel():
            # a hop transition completed in an episode its replica has already left (reported in the
            # step that crossed the episode end): Agent.reset drops the upcoming events
            # (agent.py:141-145), so it is not queued into the new episode
            cur = torch.from_numpy(self.episode % 256).to(self.device)[h["replica"].long()]
            fresh = (h["episode"].long() % 256) == cur
            if not bool(fresh.all()):
                h = {k: t[fresh] for k, t in h.items()}
        n = h["node"].numel()
        if n == 0:
            return
        if self.signaling == "target":                # v's target, computed when v is notified
            v = self.nbr[h["node"].long(), h["action"].long()]
            with torch.no_grad():
                h["reward"] = self._bootstrap(self.q, h["node"].long(), h["action"].long(),
                                              h["reward"].to(torch.float32), h["next_obs"], h["done"].bool())
            h["prio"] = (self.steps[v] + 1).to(torch.float64)      # v's gradient_step_idx (trainer.py:27,99)
        rep = h["replica"].long()
        v_host = self.nbr_host[h["node"].long().cpu().numpy(), h["action"].long().cpu().numpy()]
        if "t_ns" in h:
            t_not = h["t_ns"].double().cpu().numpy() / 1e9
        else:
            t_not = self.clock[rep.cpu().numpy()]
        due = t_not + self.small_delay[v_host]        # signalingSim=0: Agent.curr_time + small_signaling_delay
        if self.signaling_sim == 0:
            self.small_overhead += float(self.small_size[v_host].sum())     # forwarder.py:389-391, 410-412
            self.small_pkts += n
        key = self._key(h["replica"], h["node"], h["uid"])
        seq = torch.arange(self._seq, self._seq + n, dtype=torch.int64, device=self.device)
        self._seq += n
        due_t = torch.from_numpy(due).to(self.device)
        if self._pend is None:
            self._pend, self._pend_key, self._pend_time, self._pend_seq = h, key, due_t, seq
        else:
            self._pend = {k: torch.cat([self._pend[k], h[k].to(self._pend[k].dtype)]) for k in self._pend}
            self._pend_key = torch.cat([self._pend_key, key])
            self._pend_time = torch.cat([self._pend_time, due_t])
            self._pend_seq = torch.cat([self._pend_seq, seq])
        extra = self._pend_key.numel() - self.pending_cap
        if extra > 0:                                 # echoes that never came back: oldest first
            keep = torch.ones(self._pend_key.numel(), dtype=torch.bool, device=self.device)
            keep[:extra] = False
            self._take_pending(keep)

    def _queue_order(self, idx: torch.Tensor) -> torch.Tensor:
        """idx (pending positions) in queue order: by time, ties in arrival order (the upcoming
        list is kept sorted by "time" with a stable sort, forwarder.py:441-442)."""
        idx = idx[torch.argsort(self._pend_seq[idx], stable=True)]
        return idx[torch.argsort(self._pend_time[idx], stable=True)]

    def _take_pending(self, keep: torch.Tensor):
        self._pend = {k: t[keep] for k, t in self._pend.items()}
        self._pend_key = self._pend_key[keep]
        self._pend_time = self._pend_time[keep]
        self._pend_seq = self._pend_seq[keep]

    def _release(self, sel: torch.Tensor):
        """Move the selected pending hop transitions into the buffers, in queue order (time,
        then arrival), applying "target" gradient steps as the Forwarder does per element."""
        if not bool(sel.any()):
            return
        idx = torch.nonzero(sel).squeeze(1)
        order = self._queue_order(idx)
        batch = {k: t[order] for k, t in self._pend.items()}
        if self.prioritized and self.signaling == "target":
            # add, then a newer gradient step re-weights the action's slots (forwarder.py:495-505):
            # element by element where a step rises, in between as one batch
            u_h = batch["node"].long().cpu().numpy()
            a_h = batch["action"].long().cpu().numpy()
            g_h = batch["prio"].long().cpu().numpy()
            lat = self.buffers.latest.cpu().numpy().copy()
            start = 0
            for j in range(len(u_h)):
                if g_h[j] > lat[u_h[j], a_h[j]]:
                    self._add({k: t[start:j + 1] for k, t in batch.items()})
                    self.buffers.gradient_step(int(u_h[j]), int(a_h[j]), int(g_h[j]))
                    lat[u_h[j], a_h[j]] = g_h[j]
                    start = j + 1
            if start < len(u_h):
                self._add({k: t[start:] for k, t in batch.items()})
        else:
            self._add(batch)
        self._take_pending(~sel)

    def _add(self, tr: dict):
        if tr["node"].numel() == 0:
            return
        if self.prioritized and "prio" not in tr:
            # loss transitions and the hop transitions of "ideal" / "NN": the action's latest step
            tr = dict(tr, prio=self.buffers.latest[tr["node"].long().to(self.device),
                                                   tr["action"].long().to(self.device)].to(torch.float64))
        if not self.prioritized and "prio" in tr:
            tr = {k: t for k, t in tr.items() if k != "prio"}
        self.buffers.add(tr)
        self.transitions_seen += torch.bincount(tr["node"].long().to(self.device), minlength=self.N)

    @staticmethod
    def _key(replica, node, uid):
        """(replica, node, uid mod 2^21): the engine's echo carries 21 uid bits (engine_layout.h)."""
        return (replica.long() << 29) | (node.long() << 21) | (uid.long() & ((1 << 21) - 1))

    def on_control(self, obs: torch.Tensor, info: dict):
        """Control notifications of a VecRoutingEnv step (obs rows [1000, a, b, c],
        include/prisma.h), signalingSim=1: an echo releases the first queued hop transition of
        its packet at this node (forwarder.py:246-250, 477-490); a big-signalling segment that
        completes a neighbour's NN swaps this node's target copy of it (forwarder.py:251-263)."""
        if "control" not in info:
            return
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
            # the first queued match of each echo (the queue is in time order, arrival order
            # breaking ties): one transition per echo, as the reference pops one element
            hit = torch.isin(self._pend_key, keys)
            if bool(hit.any()):
                cand = self._queue_order(torch.nonzero(hit).squeeze(1))
                uk, inv = torch.unique(self._pend_key[cand], return_inverse=True)
                pos = torch.arange(cand.numel(), device=self.device)
                firstpos = torch.full((uk.numel(),), cand.numel(), dtype=torch.int64, device=self.device)
                firstpos = firstpos.scatter_reduce(0, inv, pos, reduce="amin")
                sel = torch.zeros(self._pend_key.numel(), dtype=torch.bool, device=self.device)
                sel[cand[firstpos]] = True
                self._release(sel)
        if self.signaling == "NN" and bool(big.any()):
            rows = obs[big].cpu().numpy()
            reps = torch.nonzero(big).squeeze(1).cpu().tolist()
            for r, v, (_, nn, seg, c) in zip(reps, node[big].cpu().tolist(), rows[:, :4].tolist()):
                self.on_big_signal(v, int(self.topo.overlay_nodes[c & 0xFFFF]), nn, seg, replica=r)

    def on_big_signal(self, v: int, src: int, nn_index: int, seg_index: int, replica: int = 0):
        """Node v of `replica` received segment seg_index of NN nn_index of neighbour src
        (underlay id), forwarder.py:251-263."""
        if seg_index > self.nn_max_seg:
            raise ValueError(f"segIndex > {self.nn_max_seg}")       # forwarder.py:256-257
        if seg_index != self.nn_max_seg:
            return
        i = self.topo.neighbors(v).index(src)
        if nn_index == self.sync_counter[replica, v] - 1:           # agent.py:168-175, with_temp
            self.tgt_ver[replica, v, i] = self.tmp_ver[replica, v, i]
        else:
            self.tgt_ver[replica, v, i] = self.up_ver[replica, v, i]
        self._gc()

    # -- syncs and signalingSim=0 arrivals -----------------------------------------
    def check_sync(self, force: bool = False):
        """trainer.py:101-112 for every (replica, node): sync when the replica's clock is past
        (sync_counter + 1) * sync_step (force: every node of every replica now)."""
        deg = self.deg_host > 0
        if force:
            due = np.broadcast_to(deg[None, :], self.sync_counter.shape).copy()
        else:
            due = (self.clock[:, None] > (self.sync_counter + 1) * self.sync_step[None, :]) & deg[None, :]
        if not due.any():
            return
        self._gc()
        self.version += 1
        self._snap_gen[self.version] = self._capture()
        r_idx, u_idx = np.nonzero(due)
        self.tmp_ver[r_idx, u_idx] = self.up_ver[r_idx, u_idx]        # sync_neighbor_upcoming_target_q_network
        self.up_ver[r_idx, u_idx] = self.version
        self.sync_counter[r_idx, u_idx] += 1
        if self.signaling == "ideal":                                  # _sync_all(update_upcoming=False)
            self.tgt_ver[r_idx, u_idx] = self.up_ver[r_idx, u_idx]
        elif self.signaling == "NN" and self.signaling_sim == 0:       # trainer.py:160-167
            for r, u in zip(r_idx.tolist(), u_idx.tolist()):
                t = self.clock[r] + self.big_delay[u]
                for i in range(int(self.deg_host[u])):
                    self._big.append((t, self._seq, r, u, i))
                    self._seq += 1
                    self.big_overhead += self.nn_size[u]
                    self.big_pkts += 1
        self._gc()

    def sync(self):
        """Sync every node of every replica now (tests / callers that schedule syncs themselves)."""
        self.check_sync(force=True)

    def release_due(self):
        """signalingSim=0 (_get_upcoming_events, forwarder.py:444-475): the queued hop
        transitions and NN arrivals whose time has come (time <= the replica's clock), in time
        order."""
        if self.signaling_sim != 0:
            return
        if self._pend is not None and self._pend_key.numel():
            clk = torch.from_numpy(self.clock).to(self.device)
            due = self._pend_time <= clk[self._pend["replica"].long()]
            self._release(due)
        if self._big:
            keep = []
            for e in sorted(self._big):
                t, _, r, u, i = e
                if t <= self.clock[r]:
                    self.tgt_ver[r, u, i] = self.up_ver[r, u, i]     # _sync_current(neighbor_idx)
                else:
                    keep.append(e)
            self._big = keep
            self._gc()

    # -- learning -------------------------------------------------------------
    def targets(self, node, action, reward, next_obs, done, replica=None) -> torch.Tensor:
        """r + gamma * (1 - done) * min over the next node's filtered actions of node u's copy
        of that neighbour (per replica: the copy the replica's syncs and signalling gave u)."""
        rep = torch.zeros_like(node) if replica is None else replica.long()
        ver = self.tgt_ver[rep.cpu().numpy(), node.cpu().numpy(), action.cpu().numpy()]
        gens = {}
        for k in np.unique(ver).tolist():            # one forward pass per stored generation
            gens.setdefault(self._snap_gen[int(k)], []).append(k)
        gen_of = torch.from_numpy(ver).to(node.device)
        out = torch.empty_like(reward)
        for g, vs in gens.items():
            sel = torch.isin(gen_of, torch.tensor(vs, dtype=gen_of.dtype, device=node.device))
            self._eval.load_state_dict(self._gen_w[g])
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
        N, B = self.N, self.batch_size
        ready = (self.buffers.total >= B) & (self.deg > 0)
        if not bool(ready.any()):
            return None
        s = self.buffers.sample_full(B, self.gen)
        node = torch.arange(N, device=self.device).repeat_interleave(B)
        obs, act, rew = s["obs"].reshape(N * B, -1), s["action"].reshape(-1), s["reward"].reshape(-1)
        nobs, done, rep = s["next_obs"].reshape(N * B, -1), s["done"].reshape(-1), s["replica"].reshape(-1)
        w = s["weights"].reshape(N, B).to(torch.float32)
        with torch.no_grad():
            # "target" signalling: the buffer holds the targets the next nodes computed
            tgt = rew if self.signaling == "target" else self.targets(node, act, rew, nobs, done, rep)
        q = self.q.q_values(obs, node)
        qsel = q.gather(1, act[:, None]).squeeze(1)
        per = (w * huber(qsel - tgt).view(N, B)).mean(dim=1)          # learner.py:179, per node
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

    def _snapshot(self) -> dict:
        return {k: t.detach().clone() for k, t in self.q.state_dict().items()}

    def _weights_key(self):
        return tuple(int(p._version) for p in self.params)

    def _capture(self):
        """The generation key of the current online weights, stored if new. At the opt-in
        max_snapshots cap the newest stored generation instead (counted in stale_syncs)."""
        key = self._weights_key()
        if key not in self._gen_w:
            if self.max_snapshots is not None and len(self._gen_w) >= self.max_snapshots:
                self.stale_syncs += 1
                if not self._stale_warned:
                    warnings.warn(f"QRoutingTrainer: max_snapshots={self.max_snapshots} reached; syncs now copy "
                                  "the newest stored weight generation instead of the current weights (counted "
                                  "in stale_syncs). The reference copies the current weights at every sync "
                                  "(trainer.py:101-171): leave max_snapshots=None for that", RuntimeWarning,
                                  stacklevel=3)
                    self._stale_warned = True
                return self._snap_gen[max(self._snap_gen)]
            self._gen_w[key] = self._snapshot()
            n = len(self._gen_w)
            self.peak_generations = max(self.peak_generations, n)
            if (self.warn_stored_bytes is not None and not self._bytes_warned
                    and n * self.generation_bytes > self.warn_stored_bytes):
                warnings.warn(f"QRoutingTrainer: {n} stored weight generations hold {n * self.generation_bytes} bytes "
                              f"(> warn_stored_bytes={self.warn_stored_bytes}); replica clocks far apart keep old "
                              "copies alive. A smaller sync_step or train_every, or max_snapshots, bounds them",
                              RuntimeWarning, stacklevel=3)
                self._bytes_warned = True
        return key

    def stats(self) -> dict:
        """The trainer's own counters (not the reference's Agent statistics): signalling overheads,
        stored weight generations (now and at their peak, count and bytes) and the syncs that received
        an older generation (max_snapshots)."""
        return {"small_signaling_bytes": float(self.small_overhead), "small_signaling_pkts": int(self.small_pkts),
                "big_signaling_bits": float(self.big_overhead), "big_signaling_pkts": int(self.big_pkts),
                "stored_generations": len(self._gen_w), "stale_syncs": int(self.stale_syncs),
                "stored_bytes": len(self._gen_w) * self.generation_bytes,
                "peak_generations": int(self.peak_generations),
                "peak_stored_bytes": int(self.peak_generations) * self.generation_bytes}

    def weights_of(self, version: int) -> dict:
        """The stacked online weights copy `version` refers to."""
        return self._gen_w[self._snap_gen[int(version)]]

    @property
    def snapshots(self) -> dict:
        """Stored weight generations (bounded by max_snapshots when it is set)."""
        return self._gen_w

    def _gc(self):
        live = set(np.unique(np.concatenate([self.tgt_ver.ravel(), self.up_ver.ravel(), self.tmp_ver.ravel()])).tolist())
        live.add(self.version)
        for k in [k for k in self._snap_gen if k not in live]:
            del self._snap_gen[k]
        used = set(self._snap_gen.values())
        for g in [g for g in self._gen_w if g not in used]:
            del self._gen_w[g]


def train(env, trainer: QRoutingTrainer, steps: int, train_every: int = 1, sync_every: Optional[int] = None):
    """Drive a VecRoutingEnv (external-action mode) with the trainer's epsilon-greedy
    policy: each step applies one action per replica, hands the step's notifications and
    completed transitions to the trainer (on_step: clocks, buffers, signalling, syncs), and
    trains every ``train_every`` steps; returns per-step mean losses.

    ``sync_every`` (syncs every k env steps) is gone: syncs follow each replica's simulated
    clock and ``QRoutingTrainer(sync_step=...)`` (trainer.py:101-112). Passing it warns and
    is otherwise ignored."""
    if sync_every is not None:
        warnings.warn("train(sync_every=...) is ignored: syncs follow the replicas' simulated clocks; set "
                      "QRoutingTrainer(sync_step=seconds) instead", DeprecationWarning, stacklevel=2)
    obs, info = env.reset()
    trainer.advance_clock(info["now_ns"], info.get("episode"))
    losses = []
    for s in range(steps):
        a = trainer.act(obs, info["node"])
        obs, _, _, info = env.step(a)
        trainer.on_step(obs, info)
        if s % train_every == 0:
            per = trainer.train_step()
            if per is not None:
                losses.append(float(torch.nanmean(per)))
    return losses
