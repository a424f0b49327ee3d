"""Per-node ``Ns3Env`` drop-in over one GPU replica (the reference's gym surface).

The reference runs one ns-3 process and, per overlay node, one
``ns3env.Ns3Env(port=basePort+index, stepTime, startSim, simSeed, simArgs,
debug)`` client (forwarder.py:47) that a Forwarder thread drives with
``reset()`` / ``step(action)`` (forwarder.py:291-332; ns3env.py:378-440):

* the constructor returns with the start-up state ([-1]) that every node's
  environment notifies during setup (sim.cc:546); the action answering it is
  ignored, and ``reset()`` returns that observation;
* ``step(action)`` applies the action to the packet this node was last shown,
  then blocks until the simulator notifies this node again and returns
  ``(obs, reward, done, info)``: obs = ``[dst, v_0..v_{deg-1}]``
  (data-packet-manager.cc:171-206), reward = ``getReward()`` = 1,
  done = packet at its destination (``getGameOver``, :219-227), info = the
  22-token string of ``DataPacketManager::getInfo`` (packet-manager.cc:119-176,
  data-packet-manager.cc:230-248) that ``Forwarder.treat_info`` parses;
* at simulation end ``connected`` turns False (ns3env.py:211-213).

Here the simulator is ``PrismaSession``: one replica of the HIP engine in
external-action mode.  At most one decision is pending at a time, exactly as
ns-3 blocks on each Notify; ``PrismaSession.apply`` hands the action to the
engine, which runs on the GPU to the next data notification (any node).  The
info string is rendered from the engine's decision record and counters.

This is the slow, one-decision-per-launch compatibility path for unmodified
agents; batched training/evaluation uses ``VecRoutingEnv`` (prisma_amd.env).
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional

import numpy as np

from .config import engine_params
from .engine import PrismaEngine
from .env import Box, Discrete
from .records import ST_DESTINATION, ST_DROPPED, ST_ENQUEUED, ST_PENDING
from .topology import Topology

_SESSIONS: List["PrismaSession"] = []


def _f(x: float) -> str:
    return "%f" % x


class InfoTracker:
    """State behind the info string that is not in one record: the packets a
    node lost since its last data notification (dropPacket ->
    "Packet Lost=", data-packet-manager.cc:88-98) and each packet's source."""

    def __init__(self, n_nodes: int, data_size: int):
        self.lost: Dict[int, List[int]] = {u: [] for u in range(n_nodes)}
        self.src: Dict[int, int] = {}
        self.data_size = int(data_size)

    def notified(self, rec):
        """A data notification (record just written, status PENDING or DESTINATION)."""
        if int(rec["prev"]) < 0:
            self.src[int(rec["uid"])] = int(rec["node"])

    def applied(self, rec):
        """The decision of `rec` was applied (final status)."""
        st = int(rec["status"])
        if st == ST_DROPPED:
            self.lost[int(rec["node"])].append(int(rec["uid"]))
            self.src.pop(int(rec["uid"]), None)
        elif st == ST_DESTINATION:
            self.src.pop(int(rec["uid"]), None)

    @staticmethod
    def _stats(cnt, now: float, start: float, size: int, uid: int, ptype: int) -> str:
        """PacketManager::getInfo tokens 0-17 (packet-manager.cc:119-176)."""
        e2e_n, cost_n = int(cnt["e2e_n"]), int(cnt["cost_n"])
        avg_e2e = np.float32(cnt["e2e_sum"]) / np.float32(e2e_n) if e2e_n else np.float32(0.0)
        avg_cost = np.float32(cnt["cost_sum"]) / np.float32(cost_n) if cost_n else np.float32(0.0)
        bd = int(cnt["bytes_data"])
        sig = np.float32(int(cnt["bytes_signaling"])) / np.float32(bd) if bd else np.float32(0.0)
        lost, inj, arr = int(cnt["ov_lost"]), int(cnt["ov_injected"]), int(cnt["ov_arrived"])
        ul, ui, ua = int(cnt["un_lost"]), int(cnt["un_injected"]), int(cnt["un_arrived"])
        return (f"End to End Delay={_f(now - start)}, Packet Size={size}, "
                f"Current sim time ={_f(now)}, Pkt ID ={uid}, packetType ={ptype}"
                f", Avg End to End Delay ={_f(float(avg_e2e))}, Avg Cost ={_f(float(avg_cost))}, "
                f"Avg Underlay End to End Delay ={_f(0.0)}, Avg Underlay Cost ={_f(0.0)}"
                f", Packets dropped ={lost}, Packets delivered ={arr}, Packets injected ={inj},"
                f"Packets Buffered ={inj - (arr + lost)}"
                f", Packets dropped Underlay ={ul}, Packets delivered Underlay={ua}, Packets injected Underlay={ui},"
                f"Packets Buffered Underlay={ui - (ua + ul)}"
                f",Signaling overhead ={_f(float(sig))}")

    def render(self, rec, cnt) -> str:
        """DataPacketManager::getInfo for the notified data packet (22 tokens,
        data-packet-manager.cc:230-248)."""
        v = int(rec["node"])
        now = int(rec["t_ns"]) / 1e9
        lv = self.lost[v]
        lost_ids = "".join("%u;" % u for u in reversed(lv))
        lv.clear()
        uid = int(rec["uid"])
        return (self._stats(cnt, now, float(int(rec["start_s"])), self.data_size, uid, 0)
                + f", Packet Lost={lost_ids}, Source={self.src.get(uid, v)}, Destination={int(rec['dst'])}, node={v}")

    def render_ctrl(self, uid: int, cnt, size: int = 30) -> str:
        """SmallSignalingPacketManager::getInfo (small-signaling-packet-manager.cc:104-114): 20
        tokens.  Token 3 (the echo's own ns-3 packet uid) carries the signalled uid; size is the
        echo's size on the wire (30 B + its payload by signalling type, sim.cc:373-392)."""
        now = int(cnt["now_ns"]) / 1e9
        return self._stats(cnt, now, 0.0, size, uid, 2) + f", PacketIdSignaled={uid}, Arrived at final dest=1"

    def render_big(self, nn: int, seg: int, src_overlay: int, cnt) -> str:
        """BigSignalingPacketManager::getInfo (big-signaling-packet-manager.cc:111-123): 21 tokens,
        the NN-weight segment (542 B on the wire) of overlay node src_overlay.  Token 3 (the
        segment's ns-3 packet uid) is not modelled: 0."""
        now = int(cnt["now_ns"]) / 1e9
        return (self._stats(cnt, now, 0.0, 542, 0, 1)
                + f", NN Index={nn}, segment Index={seg}, NodeId Signaled={src_overlay}")

    def render_control(self, row, cnt) -> str:
        """Info string of a control notification from its engine obs row [1000, a, b, c]
        (include/prisma.h, prisma_params_t.notify_dest)."""
        if int(row[3]) & 0x10000:
            return self.render_big(int(row[1]), int(row[2]), int(row[3]) & 0xFFFF, cnt)
        return self.render_ctrl(int(row[1]), cnt, int(row[2]))


class PrismaSession:
    """One simulated network (one engine replica) shared by the per-node envs."""

    def __init__(self, topology: str = "abilene", tm_index: int = 0, load_factor: float = 1.0,
                 base_port: int = 6555, device: int = 0, replica: int = 0, topo: Optional[Topology] = None,
                 **params):
        self.topo = topo if topo is not None else Topology.example(topology, tm_index, load_factor)
        self.params = engine_params(self.topo, replica_base=replica, notify_dest=1, **params)
        self.engine = PrismaEngine(self.topo, self.params, 1, device)
        self.base_port = int(base_port)
        self.N = self.topo.n_nodes
        self.n_agents = self.topo.n_overlay                               # ports base .. base + NO - 1
        self.deg = [int(d) for d in self.topo.degrees]
        self.data_size = int(self.params["packet_size"]) + 30          # UDP 8 + IP 20 + PPP 2
        self._cv = threading.Condition()
        self.tracker = InfoTracker(self.N, self.data_size)
        self._last_done = [False] * self.N
        self._pending = None                                             # (node, obs, done, info, dec)
        self._over = False
        self._closed = 0
        self._inflight: Dict[int, int] = {}                              # tunnel hops not yet arrived: dec -> uid
        self.log: List[tuple] = []                                       # (node, obs, done, info) per notify
        self.engine.reset(0)
        self._advance(None)
        _SESSIONS.append(self)

    # -- simulator side ------------------------------------------------------
    def _advance(self, action: Optional[int]):
        import torch
        a = None if action is None else torch.tensor([int(action)], dtype=torch.int32, device=self.engine.torch_device)
        prev = self._pending
        obs, mask, node = self.engine.step(a)
        cnt = self.engine.counters()[0]
        if prev is not None and prev[4] is not None:
            rec = self.engine.records(0, prev[4], 1)[0]
            self.tracker.applied(rec)
            if not self.topo.identity and int(rec["status"]) == ST_ENQUEUED:
                self._inflight[prev[4]] = int(rec["uid"])
        if self._inflight:
            self._poll_tunnel_drops(int(cnt["dec_count"]))
        if int(mask.cpu()[0]) == 0:
            self._pending = None
            self._over = True
            return
        v = int(node.cpu()[0])
        row = obs.cpu().numpy()[0]
        if int(row[0]) == 1000:
            # control notification (--train small signalling, --signaling big signalling): obs
            # [1000]; GetGameOver reports the node's last data notification (packet-routing-gym.cc:143-148)
            self._pending = (v, [1000], self._last_done[v], self.tracker.render_control(row, cnt), None)
        else:
            d = int(cnt["dec_count"]) - 1
            rec = self.engine.records(0, d, 1)[0]
            assert int(rec["status"]) in (ST_PENDING, ST_DESTINATION)
            ob = [int(x) for x in row[:1 + self.deg[v]]]
            self._inflight.pop(int(rec["prev"]), None)                   # the hop arrived
            self.tracker.notified(rec)
            done = int(rec["status"]) == ST_DESTINATION
            self._last_done[v] = done
            self._pending = (v, ob, done, self.tracker.render(rec, cnt), d)
        self.log.append(self._pending[:4])

    def _poll_tunnel_drops(self, dec_count: int):
        """Tunnelled overlays: a packet can be dropped on an intermediate FIFO after its
        decision was applied; the engine then re-marks that record DROPPED (MacTxDrop ->
        the sender's dropPacket, data-packet-manager.cc:88-106).  Polled after every engine
        step, i.e. at the same point of the event stream as the reference; several such
        drops inside one step are listed in decision order (the reference: drop order)."""
        import torch
        cap = self.engine.log_capacity
        for d in [d for d in self._inflight if d < dec_count - cap // 2]:
            del self._inflight[d]                                         # TTL-expired, never arrives
        if not self._inflight:
            return
        ds = sorted(self._inflight)
        dev = self.engine.torch_device
        raw = self.engine.gather_records(torch.zeros(len(ds), dtype=torch.int32, device=dev),
                                         torch.tensor(ds, dtype=torch.int32, device=dev)).cpu().numpy()
        recs = raw.reshape(-1).view(self.engine.rec_dtype)
        for d, rec in zip(ds, recs):
            if int(rec["status"]) == ST_DROPPED:
                self.tracker.applied(rec)
                del self._inflight[d]

    # -- single-threaded driver (tests, notebooks) -----------------------------
    def pending(self):
        """(node, obs, done, info) of the decision the simulator waits for, or None at the end."""
        with self._cv:
            return None if self._pending is None else self._pending[:4]

    def apply(self, action: int):
        """Apply an action to the pending decision and run to the next notification."""
        with self._cv:
            if self._pending is None:
                raise RuntimeError("simulation over")
            self._advance(action)            # at a destination the action is ignored (:256-260)
            self._cv.notify_all()

    def over(self) -> bool:
        return self._over

    def counters(self):
        return self.engine.counters()[0]

    def close(self):
        with self._cv:
            self._closed += 1
            if self._closed >= self.n_agents or self._over:
                self._over = True
                self._cv.notify_all()

    # -- per-node blocking view ------------------------------------------------
    def _wait_for(self, node: int):
        with self._cv:
            while not self._over and (self._pending is None or self._pending[0] != node):
                self._cv.wait()
            return None if self._pending is None or self._pending[0] != node else self._pending[:4]

    def _step_node(self, node: int, action: int):
        with self._cv:
            if self._pending is not None and self._pending[0] == node:
                self._advance(action)
                self._cv.notify_all()
        return self._wait_for(node)


def session_for_port(port: int) -> PrismaSession:
    for s in reversed(_SESSIONS):
        if s.base_port <= port < s.base_port + s.n_agents:
            return s
    raise RuntimeError(f"no PrismaSession serves port {port}: create one with PrismaSession(base_port=...)")


class _BridgeShim:
    """The bits of Ns3ZmqBridge the Forwarder touches (send_close_command)."""

    def __init__(self, env: "Ns3Env"):
        self.env = env

    def send_close_command(self):
        self.env.session.close()
        return True


class Ns3Env:
    """ns3env.Ns3Env signature; overlay index = port - session.base_port (the env of overlay
    node i listens on openGymPort + i, sim.cc:528-535); `node` is its underlay id.

    Like the reference, the constructor returns at once with the start-up
    state every node's PacketRoutingEnv::initialize() notifies (sim.cc:546,
    packet-routing-gym.cc:216-219): obs [-1], reward -1, not done, info "-1,".
    The action answering it is ignored (ExecuteActions with the train-step
    flag, :200-201); later steps answer real data notifications."""

    def __init__(self, stepTime=0, port=0, startSim=True, simSeed=0, simArgs={}, debug=False,
                 session: Optional[PrismaSession] = None):
        self.stepTime, self.port, self.startSim = stepTime, port, startSim
        self.simSeed, self.simArgs, self.debug = simSeed, simArgs, debug
        self.session = session if session is not None else session_for_port(int(port))
        self.node = int(self.session.topo.overlay_nodes[int(port) - self.session.base_port])
        deg = self.session.deg[self.node]
        self.action_space = Discrete(deg)
        self.observation_space = Box(0, 16260, (1 + deg,))
        self.ns3ZmqBridge = _BridgeShim(self)
        self.connected = True
        self._startup = True
        self._state = ([-1], -1.0, False, "-1,")

    def _to_state(self, st):
        if st is None:
            self.connected = False
            return self._state
        v, obs, done, info = st
        return (list(obs), 1.0, bool(done), info)

    def reset(self):
        return self._state[0]

    def step(self, action):
        if self._startup:                    # the answer to the start-up state does nothing
            self._startup = False
            st = self.session._wait_for(self.node)
        else:
            st = self.session._step_node(self.node, int(action))
        self._state = self._to_state(st)
        return self._state

    def close(self):
        self.session.close()
