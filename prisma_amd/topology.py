"""Scenario construction: topology, links and Poisson flows of one replica.

Restates the reference's scenario builder (prisma/ns3/sim.cc) for the
identity-overlay configurations (every underlay node is an overlay node,
overlay adjacency == physical adjacency: the shipped abilene and geant
examples).  Everything here is host-side, run once per environment.

Reference behaviour mirrored (file:line relative to the reference root):
  * matrix readers stop at the first empty line and require square
    matrices (sim.cc:726-786, 952-1012);
  * traffic-matrix entries are ns-3 DataRate strings parsed with the
    truncating ns-3 rule ``(uint64_t)(r * multiplier)`` and scaled as
    ``ceil(rate * load_factor)`` (sim.cc:604, 623);
  * one flow per ordered overlay pair (i != j) with a non-zero parsed rate
    (sim.cc:494-514, 599-604), created in (i, j) order;
  * neighbour (action) order is ascending neighbour id (sim.cc:469-476,
    networkx adjacency order used by forwarder.py:191);
  * the access link host i -> switch i runs at 1e6 * link_cap * deg(i) b/s
    with zero delay (sim.cc:398-410);
  * loss_penalty = ((max_buffer + packet_size + 30) * 8 / cap + 0.001) * N
    (argument_parser.py:163).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")

# ns-3 DataRate::DoParse unit table (1000-based multipliers; "B" = bytes).
_RATE_UNITS = {
    "bps": 1.0, "b/s": 1.0, "Bps": 8.0, "B/s": 8.0,
    "kbps": 1e3, "Kbps": 1e3, "kb/s": 1e3, "Kb/s": 1e3,
    "kBps": 8e3, "KBps": 8e3, "kB/s": 8e3, "KB/s": 8e3,
    "Kibps": 1024.0, "KiBps": 8192.0, "Kib/s": 1024.0, "KiB/s": 8192.0,
    "Mbps": 1e6, "Mb/s": 1e6, "MBps": 8e6, "MB/s": 8e6,
    "Mibps": 1048576.0, "MiBps": 8388608.0,
    "Gbps": 1e9, "Gb/s": 1e9, "GBps": 8e9, "GB/s": 8e9,
    "Gibps": 1073741824.0, "GiBps": 8589934592.0,
}


def parse_data_rate(text: str) -> int:
    """ns-3 ``DataRate(std::string)``: leading number, unit trailer.

    The number is read as a double and multiplied by the unit factor, then
    truncated to an unsigned 64-bit integer, e.g. ``"32.66Kbps" -> 32659``
    (32.66 is 32.659999... in binary).  A bare number is bits/s.
    """
    s = text.strip()
    n = 0
    while n < len(s) and (s[n].isdigit() or s[n] == "."):
        n += 1
    if n == 0:
        raise ValueError(f"bad data rate {text!r}")
    r = float(s[:n])
    trailer = s[n:]
    if trailer == "":
        return int(r)
    if trailer not in _RATE_UNITS:
        raise ValueError(f"unknown data rate unit in {text!r}")
    mult = _RATE_UNITS[trailer]
    if mult == 1.0:
        return int(r)
    return int(r * mult)


def _read_rows(path: str) -> List[List[str]]:
    """Whitespace-split rows, stopping at the first empty line (sim.cc:742)."""
    rows: List[List[str]] = []
    with open(path, "r") as fh:
        for line in fh.read().split("\n"):
            if line == "":
                break
            rows.append(line.split())
    return rows


def read_square(path: str, kind=int) -> np.ndarray:
    rows = _read_rows(path)
    n = len(rows[0]) if rows else 0
    for i, r in enumerate(rows):
        if len(r) != n:
            raise ValueError(f"{path}: row {i} has {len(r)} entries, expected {n}")
    if len(rows) != n:
        raise ValueError(f"{path}: {len(rows)} rows and {n} columns")
    if kind is str:
        return np.array(rows, dtype=object)
    return np.array([[kind(float(x)) for x in r] for r in rows])


def read_map_overlay(path: str) -> np.ndarray:
    vals: List[int] = []
    for r in _read_rows(path):
        vals.extend(int(x) for x in r)
    return np.array(vals, dtype=np.int64)


def loss_penalty(max_buffer: int, packet_size: int, link_cap: int, n_nodes: int) -> float:
    """argument_parser.py:163 (the 512+30 there is packet_size + headers)."""
    return ((((max_buffer + packet_size + 30) * 8) / link_cap) + 0.001) * n_nodes


@dataclass
class Topology:
    """One replica's network: CSR links + flow table (host numpy arrays)."""

    n_nodes: int
    adjacency: np.ndarray            # [N, N] 0/1
    row_ptr: np.ndarray              # [N+1] int32
    link_dst: np.ndarray             # [E] int32
    link_src: np.ndarray             # [E] int32
    link_rev: np.ndarray             # [E] int32
    flow_src: np.ndarray             # [F] int32
    flow_dst: np.ndarray             # [F] int32
    flow_rate_bps: np.ndarray        # [F] uint64 (after load factor)
    flow_base_bps: np.ndarray        # [F] uint64 (parsed, before load factor)
    name: str = "custom"
    load_factor: float = 1.0
    overlay_index: Optional[np.ndarray] = None

    @property
    def n_links(self) -> int:
        return int(self.link_dst.shape[0])

    @property
    def n_flows(self) -> int:
        return int(self.flow_src.shape[0])

    @property
    def degrees(self) -> np.ndarray:
        return np.diff(self.row_ptr).astype(np.int32)

    @property
    def max_deg(self) -> int:
        return int(self.degrees.max())

    @property
    def obs_width(self) -> int:
        w = 1 + self.max_deg
        return (w + 3) & ~3

    def neighbors(self, u: int) -> List[int]:
        return [int(x) for x in self.link_dst[self.row_ptr[u]:self.row_ptr[u + 1]]]

    def link_id(self, u: int, v: int) -> int:
        nb = self.neighbors(u)
        return int(self.row_ptr[u]) + nb.index(v)

    # ------------------------------------------------------------------
    @classmethod
    def from_matrices(cls, adjacency, tm_strings, load_factor: float = 1.0,
                      name: str = "custom") -> "Topology":
        adj = (np.asarray(adjacency) != 0).astype(np.int32)
        n = adj.shape[0]
        if adj.shape != (n, n):
            raise ValueError("adjacency must be square")
        if np.any(np.diag(adj)):
            raise ValueError("self-loops are not supported")
        if not np.array_equal(adj, adj.T):
            raise ValueError("adjacency must be symmetric (p2p links are bidirectional)")
        tm = np.asarray(tm_strings, dtype=object)
        if tm.shape != (n, n):
            raise ValueError(f"traffic matrix shape {tm.shape} != ({n}, {n}) (sim.cc:310-313)")
        row_ptr = np.zeros(n + 1, dtype=np.int32)
        dst, src = [], []
        for u in range(n):
            nb = [v for v in range(n) if adj[u, v]]
            row_ptr[u + 1] = row_ptr[u] + len(nb)
            dst.extend(nb)
            src.extend([u] * len(nb))
        link_dst = np.array(dst, dtype=np.int32)
        link_src = np.array(src, dtype=np.int32)
        e = len(dst)
        index = {(int(link_src[l]), int(link_dst[l])): l for l in range(e)}
        link_rev = np.array([index[(int(link_dst[l]), int(link_src[l]))] for l in range(e)],
                            dtype=np.int32)
        if np.any(row_ptr[1:] - row_ptr[:-1] == 0):
            raise ValueError("every node needs at least one link")
        fs, fd, fr, fb = [], [], [], []
        for i in range(n):
            for j in range(n):
                if i == j:
                    continue
                base = parse_data_rate(str(tm[i, j])) if not isinstance(tm[i, j], (int, np.integer)) \
                    else int(tm[i, j])
                if base <= 0:
                    continue                       # sim.cc:604
                rate = int(math.ceil(float(base) * float(load_factor)))   # sim.cc:623
                if rate <= 0:
                    continue
                fs.append(i); fd.append(j); fr.append(rate); fb.append(base)
        return cls(n_nodes=n, adjacency=adj, row_ptr=row_ptr, link_dst=link_dst,
                   link_src=link_src, link_rev=link_rev,
                   flow_src=np.array(fs, dtype=np.int32), flow_dst=np.array(fd, dtype=np.int32),
                   flow_rate_bps=np.array(fr, dtype=np.uint64),
                   flow_base_bps=np.array(fb, dtype=np.uint64),
                   name=name, load_factor=float(load_factor),
                   overlay_index=np.arange(n, dtype=np.int32))

    @classmethod
    def from_files(cls, physical_adjacency: str, overlay_adjacency: str, map_overlay: str,
                   traffic_matrix: str, load_factor: float = 1.0, name: str = "custom") -> "Topology":
        phys = read_square(physical_adjacency)
        over = read_square(overlay_adjacency)
        mapo = read_map_overlay(map_overlay)
        tm = read_square(traffic_matrix, kind=str)
        identity = (phys.shape == over.shape and np.array_equal(phys != 0, over != 0)
                    and mapo.shape[0] == phys.shape[0]
                    and np.array_equal(mapo, np.arange(phys.shape[0])))
        if not identity:
            raise NotImplementedError(
                "only identity overlays (map_overlay = 0..N-1, overlay == physical adjacency) are "
                "supported by this build; tunnelled overlays (SURVEY 8a A15) are a next item")
        return cls.from_matrices(phys, tm, load_factor=load_factor, name=name)

    @classmethod
    def example(cls, name: str = "abilene", tm_index: int = 0, load_factor: float = 1.0) -> "Topology":
        root = os.path.join(DATA_DIR, name)
        tf = os.path.join(root, "topology_files")
        return cls.from_files(os.path.join(tf, "physical_adjacency_matrix.txt"),
                              os.path.join(tf, "overlay_adjacency_matrix.txt"),
                              os.path.join(tf, "map_overlay.txt"),
                              os.path.join(root, "traffic_matrices", f"node_intensity_normalized_{tm_index}.txt"),
                              load_factor=load_factor, name=name)


# ----------------------------------------------------------------------
# Shortest-path agent (forwarder.py:190-191): nx.shortest_path(G, u, dst)[1]
# on the unweighted overlay graph.  networkx answers that with its
# bidirectional BFS; the tie-break among equal-length paths is part of the
# agent's behaviour, so it is restated exactly and pinned
# against networkx-generated fixtures in tests/golden/.
# ----------------------------------------------------------------------
def _bidirectional_path(adj_lists: List[List[int]], s: int, t: int) -> List[int]:
    if s == t:
        return [s]
    pred = {s: None}
    succ = {t: None}
    forward = [s]
    reverse = [t]
    meet = None
    while forward and reverse and meet is None:
        if len(forward) <= len(reverse):
            this_level = forward
            forward = []
            for v in this_level:
                for w in adj_lists[v]:
                    if w not in pred:
                        forward.append(w)
                        pred[w] = v
                    if w in succ:
                        meet = w
                        break
                if meet is not None:
                    break
        else:
            this_level = reverse
            reverse = []
            for v in this_level:
                for w in adj_lists[v]:
                    if w not in succ:
                        succ[w] = v
                        reverse.append(w)
                    if w in pred:
                        meet = w
                        break
                if meet is not None:
                    break
    if meet is None:
        raise ValueError(f"no path {s} -> {t}")
    path = []
    w = meet
    while w is not None:
        path.append(w)
        w = pred[w]
    path.reverse()
    w = succ[path[-1]]
    while w is not None:
        path.append(w)
        w = succ[w]
    return path


def sp_next_hop_table(topo: Topology) -> np.ndarray:
    """[N, N] uint8 action table: index (into neighbors(u)) of the SP next hop.

    Diagonal entries (packet at its destination) are 0, the action the
    reference agent sends there (forwarder.py:149-150).
    """
    n = topo.n_nodes
    adj_lists = [topo.neighbors(u) for u in range(n)]
    table = np.zeros((n, n), dtype=np.uint8)
    for u in range(n):
        for d in range(n):
            if u == d:
                continue
            nxt = _bidirectional_path(adj_lists, u, d)[1]
            table[u, d] = adj_lists[u].index(nxt)
    return table


def sp_paths(topo: Topology) -> dict:
    n = topo.n_nodes
    adj_lists = [topo.neighbors(u) for u in range(n)]
    return {(u, d): _bidirectional_path(adj_lists, u, d) for u in range(n) for d in range(n) if u != d}
