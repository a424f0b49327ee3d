"""Minimal ZMTP 3.0 (ZeroMQ RFC 23) over TCP with the NULL mechanism: enough of REQ and
REP for the ns3-gym lock-step protocol (pyzmq / libzmq are not installed here).

Wire format (RFC 23/ZMTP):
  greeting  = %xFF 8%x00 %x7F, version %x03 %x00, mechanism "NULL" zero-padded to 20
              octets, as-server octet, 31 zero octets (64 octets);
  handshake = one READY command each way (NULL mechanism, RFC 23 §"NULL"): command-name
              "READY" and metadata properties (name-size octet, name, 4-octet big-endian
              value-size, value) -- "Socket-Type" and, for REQ, an empty "Identity";
  frame     = flags octet (bit 0 MORE, bit 1 LONG, bit 2 COMMAND), size (1 octet, or 8
              octets big-endian when LONG), body.
REQ prepends an empty delimiter frame to each request; REP returns the envelope it
received (everything up to and including the delimiter) ahead of its reply.
"""
from __future__ import annotations

import socket
import struct
import time
from typing import List, Tuple

FLAG_MORE, FLAG_LONG, FLAG_COMMAND = 0x01, 0x02, 0x04


def greeting(as_server: bool = False) -> bytes:
    return (b"\xff" + b"\x00" * 8 + b"\x7f" + b"\x03\x00" + b"NULL".ljust(20, b"\x00")
            + (b"\x01" if as_server else b"\x00") + b"\x00" * 31)


def encode_frame(body: bytes, more: bool = False, command: bool = False) -> bytes:
    flags = (FLAG_MORE if more else 0) | (FLAG_COMMAND if command else 0)
    if len(body) > 255:
        return bytes([flags | FLAG_LONG]) + struct.pack(">Q", len(body)) + body
    return bytes([flags, len(body)]) + body


def ready_command(socket_type: str) -> bytes:
    props = [(b"Socket-Type", socket_type.encode())]
    if socket_type == "REQ":
        props.append((b"Identity", b""))
    body = bytes([5]) + b"READY"
    for name, value in props:
        body += bytes([len(name)]) + name + struct.pack(">I", len(value)) + value
    return encode_frame(body, command=True)


def parse_properties(body: bytes) -> dict:
    """Metadata of a READY command body (after the command name)."""
    props, i = {}, 0
    while i < len(body):
        n = body[i]
        name = body[i + 1:i + 1 + n].decode()
        i += 1 + n
        (m,) = struct.unpack(">I", body[i:i + 4])
        props[name] = body[i + 4:i + 4 + m]
        i += 4 + m
    return props


class ZmtpSocket:
    """One ZMTP connection acting as a REQ or REP socket."""

    def __init__(self, sock: socket.socket, socket_type: str, as_server: bool):
        self.sock = sock
        self.type = socket_type
        self.sock.sendall(greeting(as_server))
        peer = self._recv_exact(64)
        if peer[0] != 0xFF or peer[9] != 0x7F or peer[10] < 3:
            raise ConnectionError("peer is not a ZMTP 3 endpoint")
        if peer[12:32].rstrip(b"\x00") != b"NULL":
            raise ConnectionError("peer does not use the NULL mechanism")
        self.sock.sendall(ready_command(socket_type))
        flags, body = self._recv_frame()
        if not flags & FLAG_COMMAND or body[1:1 + body[0]] != b"READY":
            raise ConnectionError("expected the peer's READY command")
        self.peer_properties = parse_properties(body[1 + body[0]:])
        self._envelope: List[bytes] = []

    # -- construction ---------------------------------------------------------
    @classmethod
    def connect(cls, host: str, port: int, socket_type: str = "REQ", timeout: float = 30.0) -> "ZmtpSocket":
        """Connect, retrying while the peer has not bound yet (as libzmq's connect does)."""
        deadline = time.monotonic() + timeout
        while True:
            try:
                s = socket.create_connection((host, port), timeout=timeout)
                break
            except OSError:
                if time.monotonic() > deadline:
                    raise
                time.sleep(0.02)
        s.settimeout(None)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        return cls(s, socket_type, as_server=False)

    @classmethod
    def accept(cls, listener: socket.socket, socket_type: str = "REP") -> "ZmtpSocket":
        s, _ = listener.accept()
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        return cls(s, socket_type, as_server=True)

    # -- framing ----------------------------------------------------------------
    def _recv_exact(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("ZMTP peer closed the connection")
            buf += chunk
        return bytes(buf)

    def _recv_frame(self) -> Tuple[int, bytes]:
        flags = self._recv_exact(1)[0]
        if flags & FLAG_LONG:
            (size,) = struct.unpack(">Q", self._recv_exact(8))
        else:
            size = self._recv_exact(1)[0]
        return flags, self._recv_exact(size)

    def _recv_message(self) -> List[bytes]:
        frames = []
        while True:
            flags, body = self._recv_frame()
            if flags & FLAG_COMMAND:
                continue                                   # e.g. PING / heartbeats: none expected
            frames.append(body)
            if not flags & FLAG_MORE:
                return frames

    def _send_message(self, frames: List[bytes]):
        out = b"".join(encode_frame(f, more=(i + 1 < len(frames))) for i, f in enumerate(frames))
        self.sock.sendall(out)

    # -- REQ / REP ----------------------------------------------------------------
    def send(self, body: bytes):
        if self.type == "REQ":
            self._send_message([b"", body])                # empty delimiter, then the request
        else:
            self._send_message(self._envelope + [body])

    def recv(self) -> bytes:
        frames = self._recv_message()
        if self.type == "REQ":
            if not frames or frames[0] != b"":
                raise ConnectionError("REP reply without the empty delimiter")
            return b"".join(frames[1:])
        k = frames.index(b"") + 1                          # envelope up to the delimiter
        self._envelope = frames[:k]
        return b"".join(frames[k:])

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass
