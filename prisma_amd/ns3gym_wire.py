"""The ns-3 side of the reference's ns3-gym wire protocol, backed by a GPU replica
(SURVEY 8f rank 3): an UNMODIFIED reference agent process -- ``Forwarder`` threads on
``ns3env.Ns3Env(port=basePort+index, startSim=0)`` (forwarder.py:47; ns3env.py:26-247),
which bind a ZMQ REP socket per node and wait for the simulator -- can be driven by
``OpenGymWire(PrismaSession(...)).start()`` instead of ``run_ns3`` + the ns-3 process.

Per overlay node the simulator side is a REQ socket connected to ``basePort + index``
(sim.cc:528-535) that plays ns3-gym's ``OpenGymInterface`` (the module is an un-vendored
submodule of the reference; its behaviour is pinned by the client it talks to,
ns3env.py:153-247):
  1. ``SimInitMsg`` {simProcessId, wafShellProcessId, obsSpace = Box(0, 16260,
     (1 + deg,), uint32), actSpace = Discrete(deg)} (data-packet-manager.cc:136-159),
     answered by ``SimInitAck``;
  2. the start-up state every PacketRoutingEnv notifies from ``initialize()``
     (packet-routing-gym.cc:151-163, 216-219): obs Box<int32> [-1], reward -1,
     isGameOver false, info "-1,"; its answer is ignored;
  3. per notification ``EnvStateMsg`` {obsData Box<uint32> [dst, v_0..v_{deg-1}] (or
     Box<int32> [1000] for a small-signalling packet), reward 1, isGameOver = packet at its
     destination, reason GameOver, info = the 22-token (20 for small signalling) string},
     answered by ``EnvActMsg`` {actData Discrete(action)} -- applied to that packet --
     or {stopSimReq} which stops the session;
  4. at simulation end ``EnvStateMsg`` {isGameOver, reason SimulationEnd}; the agent's
     ``send_close_command`` answers it.
Framing is ZMTP 3.0 (prisma_amd.zmtp), the messages the ns3opengym protobufs
(prisma_amd.opengym_pb).
"""
from __future__ import annotations

import os
import threading
from typing import List, Optional

from . import opengym_pb as pb
from .ns3env import PrismaSession
from .zmtp import ZmtpSocket


def space_messages(deg: int):
    obs = pb.SpaceDescription(type=pb.Box)
    obs.space.Pack(pb.BoxSpace(low=0.0, high=16260.0, dtype=pb.UINT, shape=[1 + deg]))
    act = pb.SpaceDescription(type=pb.Discrete)
    act.space.Pack(pb.DiscreteSpace(n=deg))
    return obs, act


def state_message(obs: List[int], shape: int, reward: float, over: bool, info: str, signed: bool,
                  reason: int = pb.GameOver) -> bytes:
    box = pb.BoxDataContainer(dtype=pb.INT if signed else pb.UINT, shape=[shape])
    if signed:
        box.intData.extend(int(x) for x in obs)
    else:
        box.uintData.extend(int(x) for x in obs)
    m = pb.EnvStateMsg(reward=reward, isGameOver=over, reason=reason, info=info)
    m.obsData.type = pb.Box
    m.obsData.data.Pack(box)
    return m.SerializeToString()


def action_of(raw: bytes):
    """(stop requested, action) of an EnvActMsg."""
    m = pb.EnvActMsg()
    m.ParseFromString(raw)
    if m.stopSimReq:
        return True, 0
    d = pb.DiscreteDataContainer()
    m.actData.data.Unpack(d)
    return False, int(d.data)


class OpenGymWire:
    def __init__(self, session: PrismaSession, host: str = "127.0.0.1"):
        self.session = session
        self.host = host
        self.threads: List[threading.Thread] = []
        self.errors: List[BaseException] = []

    def start(self) -> "OpenGymWire":
        for i, u in enumerate(int(x) for x in self.session.topo.overlay_nodes):
            t = threading.Thread(target=self._node, args=(i, u), daemon=True)
            t.start()
            self.threads.append(t)
        return self

    def join(self, timeout: Optional[float] = None) -> bool:
        for t in self.threads:
            t.join(timeout)
        return not any(t.is_alive() for t in self.threads)

    def _node(self, index: int, node: int):
        s = self.session
        deg = s.deg[node]
        sock = None
        try:
            sock = ZmtpSocket.connect(self.host, s.base_port + index, "REQ")
            init = pb.SimInitMsg(simProcessId=os.getpid(), wafShellProcessId=os.getppid())
            obs_space, act_space = space_messages(deg)
            init.obsSpace.CopyFrom(obs_space)
            init.actSpace.CopyFrom(act_space)
            sock.send(init.SerializeToString())
            ack = pb.SimInitAck()
            ack.ParseFromString(sock.recv())
            if ack.stopSimReq:
                s.close()
                return
            # start-up state (is_trainStep_flag = 1): its answer does nothing
            sock.send(state_message([-1], 1 + deg, -1.0, False, "-1,", signed=True))
            stop, _ = action_of(sock.recv())
            st = None if stop else s._wait_for(node)
            while st is not None:
                _, obs, done, info = st
                ctrl = len(obs) == 1 and obs[0] == 1000          # Box<int32> [1000] (packet-routing-gym.cc:155-156)
                sock.send(state_message(obs, 1 + deg, 1.0, done, info, signed=ctrl))
                stop, a = action_of(sock.recv())
                if stop:
                    break
                st = s._step_node(node, a)
            s.close()
            if not stop:                                          # NotifySimulationEnd
                sock.send(state_message([-1], 1 + deg, 1.0, True, "", signed=True, reason=pb.SimulationEnd))
                sock.recv()                                       # the agent's send_close_command
        except BaseException as e:                                # surfaced through self.errors
            self.errors.append(e)
            s.close()
        finally:
            if sock is not None:
                sock.close()
