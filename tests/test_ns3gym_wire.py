"""ns3-gym wire protocol (prisma_amd.zmtp, prisma_amd.opengym_pb, prisma_amd.ns3gym_wire).

CPU: ZMTP 3.0 known-answer bytes (RFC 23 greeting, NULL READY command), REQ/REP framing
round trips, protobuf encodings against hand-assembled wire bytes of the reference's
field numbers (messages.proto), and the whole per-node protocol driven by an
oracle-backed session with reference-like agent threads (REP sockets, Ns3ZmqBridge's
lock-step: SimInitMsg -> SimInitAck, state -> action, SimulationEnd -> close).
GPU: the same agents against a PrismaSession see the oracle's notification stream.
"""
import socket
import struct
import threading

import numpy as np
import pytest
import torch

from prisma_amd import opengym_pb as pb
from prisma_amd.config import engine_params
from prisma_amd.ns3gym_wire import OpenGymWire
from prisma_amd.topology import Topology
from prisma_amd.zmtp import ZmtpSocket, encode_frame, greeting, ready_command

from test_ns3env import oracle_stream, sp_policy


def test_zmtp_known_answers():
    g = greeting()
    assert len(g) == 64
    assert g[:10] == b"\xff\x00\x00\x00\x00\x00\x00\x00\x00\x7f" and g[10:12] == b"\x03\x00"
    assert g[12:32] == b"NULL" + b"\x00" * 16 and g[32] == 0 and g[33:] == b"\x00" * 31
    assert greeting(as_server=True)[32] == 1
    assert ready_command("REP") == (b"\x04\x19\x05READY\x0bSocket-Type\x00\x00\x00\x03REP")
    assert ready_command("REQ") == (b"\x04\x26\x05READY\x0bSocket-Type\x00\x00\x00\x03REQ"
                                    b"\x08Identity\x00\x00\x00\x00")
    assert encode_frame(b"ab", more=True) == b"\x01\x02ab"
    assert encode_frame(b"x" * 300) == b"\x02" + struct.pack(">Q", 300) + b"x" * 300


def test_zmtp_req_rep_round_trip():
    lst = socket.socket()
    lst.bind(("127.0.0.1", 0))
    lst.listen(1)
    port = lst.getsockname()[1]
    got = []

    def server():
        z = ZmtpSocket.accept(lst, "REP")
        assert z.peer_properties["Socket-Type"] == b"REQ"
        for _ in range(3):
            req = z.recv()
            got.append(req)
            z.send(req[::-1])
        z.close()

    t = threading.Thread(target=server)
    t.start()
    c = ZmtpSocket.connect("127.0.0.1", port, "REQ")
    assert c.peer_properties["Socket-Type"] == b"REP"
    for msg in (b"", b"hello", bytes(range(256)) * 3):
        c.send(msg)
        assert c.recv() == msg[::-1]
    t.join()
    c.close()
    lst.close()
    assert got[1] == b"hello"


def _varint(n):
    out = b""
    while True:
        b = n & 0x7F
        n >>= 7
        out += bytes([b | (0x80 if n else 0)])
        if not n:
            return out


def _ld(field, payload):                       # length-delimited field
    return _varint(field << 3 | 2) + _varint(len(payload)) + payload


def test_protobuf_field_numbers_match_messages_proto():
    """EnvActMsg{actData = DataContainer{type Discrete, data Any(DiscreteDataContainer{2})}}
    and EnvStateMsg bytes assembled by hand from messages.proto:44-123."""
    m = pb.EnvActMsg()
    m.actData.type = pb.Discrete
    m.actData.data.Pack(pb.DiscreteDataContainer(data=2))
    anyb = _ld(1, b"type.googleapis.com/ns3opengym.DiscreteDataContainer") + _ld(2, b"\x08\x02")
    want = _ld(1, b"\x08\x01" + _ld(2, anyb))
    assert m.SerializeToString() == want
    assert pb.EnvActMsg(stopSimReq=True).SerializeToString() == b"\x10\x01"
    s = pb.EnvStateMsg(reward=1.0, isGameOver=True, reason=pb.GameOver, info="a,b")
    box = pb.BoxDataContainer(dtype=pb.UINT, shape=[4], uintData=[3, 0, 30, 0])
    s.obsData.type = pb.Box
    s.obsData.data.Pack(box)
    boxb = b"\x08\x02" + _ld(2, b"\x04") + _ld(4, b"\x03\x00\x1e\x00")
    anyb = _ld(1, b"type.googleapis.com/ns3opengym.BoxDataContainer") + _ld(2, boxb)
    want = (_ld(1, b"\x08\x02" + _ld(2, anyb)) + b"\x15" + struct.pack("<f", 1.0) + b"\x18\x01" + b"\x20\x01"
            + _ld(5, b"a,b"))
    assert s.SerializeToString() == want
    i = pb.SimInitMsg(simProcessId=7)
    i.actSpace.type = pb.Discrete
    i.actSpace.space.Pack(pb.DiscreteSpace(n=3))
    anyb = _ld(1, b"type.googleapis.com/ns3opengym.DiscreteSpace") + _ld(2, b"\x08\x03")
    assert i.SerializeToString() == b"\x08\x07" + _ld(4, b"\x08\x01" + _ld(2, anyb))


def _agents(topo, base_port, policy, ready):
    """One reference-like agent per overlay node: binds its REP socket first
    (Ns3ZmqBridge.__init__, ns3env.py:41-55), then Ns3Env's lock-step + the Forwarder loop."""
    nodes = [int(x) for x in topo.overlay_nodes]
    seen = {u: [] for u in nodes}
    errors = []
    listeners = []
    for i in range(len(nodes)):
        lst = socket.socket()
        lst.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        lst.bind(("127.0.0.1", base_port + i))
        lst.listen(1)
        listeners.append(lst)

    def decode(raw):
        st = pb.EnvStateMsg()
        st.ParseFromString(raw)
        box = pb.BoxDataContainer()
        st.obsData.data.Unpack(box)
        obs = list(box.uintData) if box.dtype == pb.UINT else list(box.intData)
        return st, obs

    def agent(i, u):
        try:
            z = ZmtpSocket.accept(listeners[i], "REP")
            init = pb.SimInitMsg()
            init.ParseFromString(z.recv())                       # initialize_env (ns3env.py:153-168)
            box, disc = pb.BoxSpace(), pb.DiscreteSpace()
            init.obsSpace.space.Unpack(box)
            init.actSpace.space.Unpack(disc)
            assert init.obsSpace.type == pb.Box and list(box.shape) == [1 + topo.degrees[u]]
            assert box.dtype == pb.UINT and box.high == 16260.0 and disc.n == topo.degrees[u]
            z.send(pb.SimInitAck(done=True, stopSimReq=False).SerializeToString())
            st, obs = decode(z.recv())                           # start-up state
            assert obs == [-1] and st.reward == -1.0 and st.info == "-1," and not st.isGameOver
            action = 0                                           # its answer is ignored
            while True:
                act = pb.EnvActMsg()
                act.actData.type = pb.Discrete
                act.actData.data.Pack(pb.DiscreteDataContainer(data=action))
                z.send(act.SerializeToString())
                st, obs = decode(z.recv())
                if st.isGameOver and st.reason == pb.SimulationEnd:
                    z.send(pb.EnvActMsg(stopSimReq=True).SerializeToString())   # send_close_command
                    break
                seen[u].append((obs, bool(st.isGameOver), st.info))
                action = policy(u, obs)
            z.close()
        except Exception as e:                                   # pragma: no cover - surfaced below
            errors.append(e)

    ths = [threading.Thread(target=agent, args=(i, u), daemon=True) for i, u in enumerate(nodes)]
    for t in ths:
        t.start()
    ready.set()
    return ths, seen, errors, listeners


class OracleSession:
    """The slice of PrismaSession the wire uses, over the CPU oracle (notify mode)."""

    def __init__(self, oracle_mod, topo, params, base_port):
        self.topo, self.base_port = topo, base_port
        self.deg = [int(d) for d in topo.degrees]
        self.n_agents = topo.n_overlay
        self.o = oracle_mod.OracleSim(topo, params)
        self.cv = threading.Condition()
        self.last_done = [False] * topo.n_nodes
        self.over = False
        self._closed = 0
        self._set(self.o.step(-1))

    def _set(self, obs):
        if obs is None:
            self.pending = None
            self.over = True
            return
        v = self.o.pending_node()
        if int(obs[0]) == 1000:
            self.pending = (v, [1000], self.last_done[v], self.o.last_info())
        else:
            done = int(self.o.records()[-1]["status"]) == 3
            self.last_done[v] = done
            self.pending = (v, [int(x) for x in obs[:1 + self.deg[v]]], done, self.o.last_info())

    def _wait_for(self, node):
        with self.cv:
            while not self.over and self.pending[0] != node:
                self.cv.wait()
            return None if self.over else self.pending

    def _step_node(self, node, action):
        with self.cv:
            if not self.over and self.pending[0] == node:
                self._set(self.o.step(int(action)))
                self.cv.notify_all()
        return self._wait_for(node)

    def close(self):
        with self.cv:
            self._closed += 1
            if self._closed >= self.n_agents:
                self.over = True
            self.cv.notify_all()


def _run_wire(session, topo, base_port, pol):
    ready = threading.Event()
    ths, seen, errors, listeners = _agents(topo, base_port, pol, ready)
    ready.wait()
    wire = OpenGymWire(session).start()
    assert wire.join(timeout=600)
    for t in ths:
        t.join(timeout=60)
    for lst in listeners:
        lst.close()
    assert not wire.errors, wire.errors
    assert not errors, errors
    return seen


@pytest.mark.parametrize("name,lf,train", [("abilene", 2.0, 1), ("overlay_full_mesh_3n_abilene", 10.0, 0)])
def test_wire_protocol_over_the_oracle(oracle_mod, name, lf, train):
    topo = Topology.example(name, 0, lf)
    params = engine_params(topo, sim_time_s=0.6, ping_as_obs=1, notify_dest=1, train=train)
    pol = sp_policy(topo)
    seen = _run_wire(OracleSession(oracle_mod, topo, params, 17300), topo, 17300, pol)
    _, ref = oracle_stream(oracle_mod, topo, params, pol, 10 ** 9)
    for u in (int(x) for x in topo.overlay_nodes):
        assert seen[u] == [(obs, done, info) for (v, obs, done, info) in ref if v == u], u
    assert sum(len(x) for x in seen.values()) == len(ref) > 100


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")
def test_wire_protocol_over_the_engine(oracle_mod):
    from prisma_amd.ns3env import PrismaSession
    topo = Topology.example("abilene", 0, 2.0)
    kw = dict(sim_time_s=1.0, ping_as_obs=1, train=1)
    pol = sp_policy(topo)
    s = PrismaSession(topo=topo, base_port=17400, **kw)
    seen = _run_wire(s, topo, 17400, pol)
    _, ref = oracle_stream(oracle_mod, topo, engine_params(topo, notify_dest=1, **kw), pol, 10 ** 9)
    for u in range(topo.n_nodes):
        assert seen[u] == [(obs, done, info) for (v, obs, done, info) in ref if v == u], u
