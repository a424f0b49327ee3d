"""Gym-style batched surface over the engine (the drop-in for Ns3Env at scale).

The reference drives one ``ns3env.Ns3Env`` per overlay node over ZMQ
(ns3env.py:378-455; forwarder.py:291-332): ``reset() -> obs``,
``step(action) -> (obs, reward, done, info)`` where ``obs`` is the next data
packet waiting at that node, ``done`` says it reached its destination and
the Q-routing reward is recovered by the agent from time stamps in ``info``.

``VecRoutingEnv`` keeps that contract for R replicas at once: every replica
always has exactly one pending notification (at whatever node the next data
packet arrives), ``step(actions)`` applies one action per replica and returns
``(obs, reward, done, info)`` for the next notifications.  What the reference forwarder
reconstructs from the info string — per-hop (obs, action, reward, next_obs,
done) transitions and the loss transitions — is produced on the device by
``transitions()``, joined from the engine's decision log.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .config import engine_params
from .engine import PrismaEngine
from .records import ST_DESTINATION, ST_DROPPED, ST_PENDING
from .topology import Topology


@dataclass
class Box:
    """gym.spaces.Box stand-in (gym is not installed): obs space of one node."""
    low: int
    high: int
    shape: tuple
    dtype: str = "uint32"


@dataclass
class Discrete:
    n: int


def decode_records(rec: torch.Tensor, W: int) -> dict:
    """Typed views of gathered records (torch uint8 [n, 32 + 4W] on any device)."""
    i32 = rec.view(torch.int32)
    i64 = rec.view(torch.int64)
    f64 = rec.view(torch.float64)
    nd = i32[:, 6]
    w7 = i32[:, 7]
    act = (w7 & 0xFF)
    act = torch.where(act >= 128, act - 256, act)
    return {
        "t_ns": i64[:, 0], "uid": i32[:, 2], "prev": i32[:, 3], "reward": f64[:, 2],
        "node": nd & 0xFF, "dst": (nd >> 8) & 0xFF, "start_s": (nd >> 16) & 0xFFFF, "action": act,
        "status": (w7 >> 8) & 0xFF, "ttl": (w7 >> 16) & 0xFF, "episode": (w7 >> 24) & 0xFF, "obs": i32[:, 8:8 + W],
    }


class VecRoutingEnv:
    def __init__(self, topology="abilene", tm_index: int = 0, load_factor: float = 1.0,
                 n_replicas: int = 1024, device: int = 0, topo: Optional[Topology] = None, **params):
        self.topo = topo if topo is not None else Topology.example(topology, tm_index, load_factor)
        self.params = engine_params(self.topo, **params)
        self.engine = PrismaEngine(self.topo, self.params, n_replicas, device)
        self.R = n_replicas
        self.W = self.engine.W
        self.device = self.engine.torch_device
        deg = self.topo.degrees
        # per-node spaces (data-packet-manager.cc:136-159)
        self.observation_spaces = [Box(0, 16260, (1 + int(d),)) for d in deg]
        self.action_spaces = [Discrete(int(d)) for d in deg]
        self.loss_penalty = float(self.params["loss_penalty"])
        self._consumed = torch.zeros(self.R, dtype=torch.int64, device=self.device)
        self._cnt_words = None

    # ------------------------------------------------------------------
    def reset(self, episode: int = 0):
        """Start `episode` on every replica -> (obs [R, W], info) of the first notifications."""
        self.engine.reset(episode)
        self._consumed.zero_()
        obs, mask, node = self.engine.step(None)
        return obs, self._info(obs, mask, node)[2]

    def step(self, actions: torch.Tensor):
        """Apply one action per replica -> (obs, reward, done, info), each batched over replicas.

        The per-node contract of Ns3Env.step (ns3env.py:417-420 -> get_state :410-415), for every
        replica's next notification:
          obs    int32 [R, W]: [dst, v_0..v_deg-1] of the notified packet (getObservation,
                 data-packet-manager.cc:171-206); [1000, uid, 0..] for a small-signalling arrival
                 (packet-routing-gym.cc:157, notify_dest with train only);
          reward f64 [R]: the Q-routing reward of the hop that brought the notified packet here,
                 curr_time - t_decision on the microsecond-formatted times (the value the Forwarder
                 computes from the info string, forwarder.py:352-360; the wire's own reward field
                 is the constant 1 of DataPacketManager::getReward, data-packet-manager.cc:219-222);
                 0.0 for a packet's first notification, control notifications and finished episodes;
          done   bool [R]: the notified packet is at its destination (getGameOver,
                 data-packet-manager.cc:225-227; only with notify_dest, otherwise destination
                 arrivals never stop the engine and done is always False);
          info   dict: mask (uint8, 0 = the replica's episode ended this call), node (deciding node,
                 -1 if none), uid / prev (packet uid and the record index of its previous decision,
                 -1 if fresh), control (bool), and "transitions": every replay transition completed
                 since the previous step (transitions(): hop transitions and loss transitions).
        """
        obs, mask, node = self.engine.step(actions.to(device=self.device, dtype=torch.int32))
        reward, done, info = self._info(obs, mask, node)
        info["transitions"] = self.transitions()
        return obs, reward, done, info

    def _info(self, obs, mask, node):
        """Reward, done and info of the current notifications, from their decision records (the
        record of a data notification is the replica's last one, written when it was notified)."""
        R = self.R
        cf = self._counter_fields()
        dec = cf["dec_count"]
        live = mask.to(torch.bool)
        control = live & (obs[:, 0] == 1000)
        data = live & ~control & (dec > 0)
        d = (dec - 1).clamp_min(0) % self.engine.log_capacity
        rec = decode_records(self.engine.gather_records(torch.arange(R, device=self.device, dtype=torch.int32),
                                                        d.to(torch.int32)), self.W)
        has_prev = data & (rec["prev"] >= 0)
        reward = torch.where(has_prev, rec["reward"], torch.zeros_like(rec["reward"]))
        done = data & (rec["status"] == ST_DESTINATION)
        info = {"mask": mask, "node": node, "control": control,
                "uid": torch.where(data, rec["uid"], torch.full_like(rec["uid"], -1)),
                "prev": torch.where(has_prev, rec["prev"], torch.full_like(rec["prev"], -1)),
                # the replica's clock at this notification (Agent.curr_time, forwarder.py:208) and
                # its episode index: the trainer schedules syncs and signalling delays on them
                "now_ns": cf["now_ns"], "episode": cf["episode"]}
        return reward, done, info

    def run(self, table: torch.Tensor, max_hops: int):
        self.engine.run(table, max_hops)

    def counters(self) -> np.ndarray:
        return self.engine.counters()

    def _counter_fields(self) -> dict:
        """dec_count, now_ns and episode of every replica (device int64 [R])."""
        from .records import COUNTERS_DTYPE
        raw = self.engine.counters_tensor()                         # [R, 152] bytes
        w32 = raw.view(torch.int32)
        w64 = raw.view(torch.int64)
        f = COUNTERS_DTYPE.fields
        return {"dec_count": w32[:, f["dec_count"][1] // 4].to(torch.int64) & 0xFFFFFFFF,
                "now_ns": w64[:, f["now_ns"][1] // 8].clone(),
                "episode": w32[:, f["episode"][1] // 4].to(torch.int64) & 0xFFFFFFFF}

    def _dec_counts(self) -> torch.Tensor:
        return self._counter_fields()["dec_count"]

    def transitions(self) -> dict:
        """Replay transitions completed since the previous call (device tensors).

        For every finalised decision d (not the trailing pending one):
          - if d has a predecessor p: (obs_p, action_p, reward_d, obs_d, done_d)
            (forwarder.py:352-379 with signaling_type="ideal");
          - if d was dropped: (obs_d, action_d, loss_penalty, [dst_d, 0..], True)
            (forwarder.py:214-240).
        """
        W = self.W
        cap = self.engine.log_capacity
        dec = self._dec_counts()
        lo = torch.maximum(self._consumed, dec - cap + 1)
        n = (dec - lo).clamp_min(0)
        total = int(n.sum().item())
        empty = {k: torch.zeros((0,) + s, dtype=t, device=self.device) for k, s, t in
                 [("obs", (W,), torch.int32), ("action", (), torch.int32), ("reward", (), torch.float64),
                  ("next_obs", (W,), torch.int32), ("done", (), torch.bool), ("node", (), torch.int32),
                  ("replica", (), torch.int32), ("uid", (), torch.int64), ("hop", (), torch.bool),
                  ("t_ns", (), torch.int64), ("episode", (), torch.int64)]}
        if total == 0:
            return empty
        rep = torch.repeat_interleave(torch.arange(self.R, device=self.device), n)
        start = torch.repeat_interleave(lo, n)
        offs = torch.arange(total, device=self.device) - torch.repeat_interleave(torch.cumsum(n, 0) - n, n)
        d = start + offs
        cur = decode_records(self.engine.gather_records(rep.to(torch.int32), d.to(torch.int32)), W)
        final = cur["status"] != ST_PENDING
        # consume everything up to (excluding) a trailing pending record
        last_pending = torch.zeros(self.R, dtype=torch.bool, device=self.device)
        ends = torch.cumsum(n, 0) - 1
        has = n > 0
        last_pending[has] = ~final[ends[has]]
        self._consumed = torch.where(has, dec - last_pending.to(torch.int64), self._consumed)
        rep_f, cur_f = rep[final], {k: v[final] for k, v in cur.items()}
        # hop transitions: predecessor record
        hp = cur_f["prev"] >= 0
        prev = decode_records(self.engine.gather_records(rep_f[hp].to(torch.int32), cur_f["prev"][hp].to(torch.int32)), W)
        # loss transitions
        dr = cur_f["status"] == ST_DROPPED
        loss_next = torch.zeros((int(dr.sum()), W), dtype=torch.int32, device=self.device)
        loss_next[:, 0] = cur_f["obs"][dr][:, 0]
        out = {
            "obs": torch.cat([prev["obs"], cur_f["obs"][dr]]),
            "action": torch.cat([prev["action"], cur_f["action"][dr]]).to(torch.int32),
            "reward": torch.cat([cur_f["reward"][hp], torch.full((int(dr.sum()),), self.loss_penalty,
                                                                 dtype=torch.float64, device=self.device)]),
            "next_obs": torch.cat([cur_f["obs"][hp], loss_next]),
            "done": torch.cat([cur_f["status"][hp] == ST_DESTINATION,
                               torch.ones(int(dr.sum()), dtype=torch.bool, device=self.device)]),
            "node": torch.cat([prev["node"], cur_f["node"][dr]]).to(torch.int32),
            "replica": torch.cat([rep_f[hp], rep_f[dr]]).to(torch.int32),
            # the packet's uid and whether this is a hop transition (False: a loss transition):
            # with "NN" / "target" signalling a hop transition waits for its echo (trainer.py)
            "uid": torch.cat([cur_f["uid"][hp], cur_f["uid"][dr]]).to(torch.int64),
            "hop": torch.cat([torch.ones(int(hp.sum()), dtype=torch.bool, device=self.device),
                              torch.zeros(int(dr.sum()), dtype=torch.bool, device=self.device)]),
            # when the transition completed: the next notification (hop) or the drop (loss)
            "t_ns": torch.cat([cur_f["t_ns"][hp], cur_f["t_ns"][dr]]).to(torch.int64),
            # the episode (mod 256) it completed in: the trainer does not queue an old episode's
            # hop transitions into the next one
            "episode": torch.cat([cur_f["episode"][hp], cur_f["episode"][dr]]).to(torch.int64),
        }
        return out

    def close(self):
        self.engine.close()
