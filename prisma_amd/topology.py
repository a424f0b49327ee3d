"""Scenario construction: topology, links, overlay tunnels and Poisson flows of one replica.

Restates the reference's scenario builder (prisma/ns3/sim.cc).  Everything
here is host-side, run once per environment.

Reference behaviour mirrored (file:line relative to the reference root):
  * matrix readers stop at the first empty line and require square
    matrices (sim.cc:726-786, 952-1012);
  * traffic-matrix entries are ns-3 DataRate strings parsed with the
    truncating ns-3 rule ``(uint64_t)(r * multiplier)`` and scaled as
    ``ceil(rate * load_factor)`` (sim.cc:604, 623);
  * one flow per ordered pair of OVERLAY nodes (i != j, underlay ids, in
    (i, j) underlay order) with a non-zero parsed rate (sim.cc:494-514,
    599-604);
  * the overlay neighbour (action) list of overlay node i is its overlay
    neighbours in ascending overlay index, stored as underlay ids
    (sim.cc:469-476); identity overlays give ascending neighbour ids
    (networkx adjacency order used by forwarder.py:191);
  * the access link host i -> switch i runs at 1e6 * link_cap * deg(i) b/s
    (deg = PHYSICAL degree, sim.cc:341-349) with zero delay (sim.cc:398-410);
  * loss_penalty = ((max_buffer + packet_size + 30) * 8 / cap + 0.001) * N
    with N = number of overlay nodes (argument_parser.py:127-128,163).

Tunnelled overlays: an overlay hop u -> w is IP-forwarded
along the underlay route that ns-3 global routing installs for the host
10.2.2.(w+1) (sim.cc:683, data-packet-manager.cc:271-287).  With unit link
metrics, ns-3's SPF (equal-distance candidates popped first-in-first-out,
link records in device order = ascending neighbour id, first root exit
direction used when RandomEcmpRouting is off) picks at every node x the
LOWEST-id neighbour that lies on some shortest path to w; ``route_tables``
restates that rule (pinned by a hand-checked known answer on the shipped
overlay_full_mesh_3n_abilene example, tests/test_topology.py).
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


def route_tables(adj: np.ndarray):
    """ns-3 global routing restated for unit metrics (module docstring).

    Returns (next_hop [N, N] int32, dist [N, N] int32): next_hop[x, y] is the
    neighbour x forwards to for destination y (-1 on the diagonal), the
    lowest-id neighbour n of x with dist[n, y] == dist[x, y] - 1."""
    n = adj.shape[0]
    nb = [[v for v in range(n) if adj[u, v]] for u in range(n)]
    dist = np.full((n, n), -1, dtype=np.int32)
    for y in range(n):                      # BFS from every destination
        dist[y, y] = 0
        frontier = [y]
        while frontier:
            nxt = []
            for u in frontier:
                for v in nb[u]:
                    if dist[v, y] < 0:
                        dist[v, y] = dist[u, y] + 1
                        nxt.append(v)
            frontier = nxt
    if np.any(dist < 0):
        raise ValueError("the physical topology must be connected")
    hop = np.full((n, n), -1, dtype=np.int32)
    for x in range(n):
        for y in range(n):
            if x != y:
                hop[x, y] = min(v for v in nb[x] if dist[v, y] == dist[x, y] - 1)
    return hop, dist


@dataclass
class Topology:
    """One replica's network: physical CSR links, overlay tunnels, flow table
    (host numpy arrays).

    Links (row_ptr/link_dst/link_src/link_rev) are the PHYSICAL directed
    switch links.  Decisions happen at overlay nodes over TUNNELS: tunnel t
    of node u = ov_row_ptr[u] + a (a = action index) goes to overlay
    neighbour tun_dst[t] (underlay id) along next_hop; its first link is
    tun_link[t] and it crosses tun_len[t] links.  For identity overlays
    tunnels == links (t == l)."""

    n_nodes: int
    adjacency: np.ndarray            # [N, N] 0/1 physical
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
    overlay_index: Optional[np.ndarray] = None     # [N] overlay index of node x, -1 if none
    overlay_nodes: Optional[np.ndarray] = None     # [N_o] underlay id of overlay node i
    overlay_adj: Optional[np.ndarray] = None       # [N_o, N_o] 0/1
    ov_row_ptr: Optional[np.ndarray] = None        # [N+1] tunnels per node (0 for non-overlay)
    tun_src: Optional[np.ndarray] = None           # [T]
    tun_dst: Optional[np.ndarray] = None           # [T]
    tun_link: Optional[np.ndarray] = None          # [T] first physical link
    tun_len: Optional[np.ndarray] = None           # [T] links crossed
    next_hop: Optional[np.ndarray] = None          # [N, N] routing (route_tables)
    dist: Optional[np.ndarray] = None              # [N, N] hop distance
    tm_strings: Optional[np.ndarray] = None        # [N, N] the traffic matrix as given (trainer's auto sync step)

    @property
    def n_links(self) -> int:
        return int(self.link_dst.shape[0])

    @property
    def n_flows(self) -> int:
        return int(self.flow_src.shape[0])

    @property
    def n_tunnels(self) -> int:
        return int(self.tun_dst.shape[0])

    @property
    def n_overlay(self) -> int:
        return int(self.overlay_nodes.shape[0])

    @property
    def identity(self) -> bool:
        """Every node is an overlay node and every tunnel is one link."""
        return self.n_overlay == self.n_nodes and bool(np.all(self.tun_len == 1)) and \
            bool(np.array_equal(self.overlay_nodes, np.arange(self.n_nodes)))

    @property
    def degrees(self) -> np.ndarray:
        """Overlay degree (number of actions) per underlay node, 0 off the overlay."""
        return np.diff(self.ov_row_ptr).astype(np.int32)

    @property
    def phys_degrees(self) -> np.ndarray:
        return np.diff(self.row_ptr).astype(np.int32)

    @property
    def max_deg(self) -> int:
        return int(self.degrees.max())

    @property
    def obs_width(self) -> int:
        w = 1 + self.max_deg
        return (w + 3) & ~3

    def neighbors(self, u: int) -> List[int]:
        """Overlay neighbours of u (underlay ids, action order)."""
        return [int(x) for x in self.tun_dst[self.ov_row_ptr[u]:self.ov_row_ptr[u + 1]]]

    def phys_neighbors(self, u: int) -> List[int]:
        return [int(x) for x in self.link_dst[self.row_ptr[u]:self.row_ptr[u + 1]]]

    def link_id(self, u: int, v: int) -> int:
        nb = self.phys_neighbors(u)
        return int(self.row_ptr[u]) + nb.index(v)

    def tunnel_path(self, t: int) -> List[int]:
        """Underlay nodes of tunnel t, origin first."""
        x, y = int(self.tun_src[t]), int(self.tun_dst[t])
        path = [x]
        while x != y:
            x = int(self.next_hop[x, y])
            path.append(x)
        return path

    # ------------------------------------------------------------------
    @classmethod
    def from_matrices(cls, adjacency, tm_strings, load_factor: float = 1.0,
                      name: str = "custom", map_overlay=None, overlay_adjacency=None) -> "Topology":
        """map_overlay[x] = overlay index of underlay node x or -1 (map_overlay.txt);
        default: identity overlay (overlay_adjacency = adjacency)."""
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
        if map_overlay is None:
            mapo = np.arange(n, dtype=np.int64)
            oadj = adj.copy()
        else:
            mapo = np.asarray(map_overlay, dtype=np.int64)
            oadj = (np.asarray(overlay_adjacency) != 0).astype(np.int32)
        if mapo.shape != (n,):
            raise ValueError(f"map_overlay has {mapo.shape[0]} entries for {n} underlay nodes")
        n_o = int((mapo >= 0).sum())
        if sorted(int(v) for v in mapo if v >= 0) != list(range(n_o)):
            raise ValueError("map_overlay must number the overlay nodes 0..N_o-1")
        if oadj.shape != (n_o, n_o) or np.any(np.diag(oadj)) or not np.array_equal(oadj, oadj.T):
            raise ValueError("overlay adjacency must be a symmetric N_o x N_o matrix without self-loops")
        overlay_nodes = np.zeros(n_o, dtype=np.int32)
        for x in range(n):
            if mapo[x] >= 0:
                overlay_nodes[mapo[x]] = x
        overlay_index = mapo.astype(np.int32)

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
        hop, dist = route_tables(adj)

        # tunnels: grouped by underlay id, each node's in ascending overlay index (sim.cc:469-476)
        ov_row_ptr = np.zeros(n + 1, dtype=np.int32)
        ts, td = [], []
        for u in range(n):
            if mapo[u] >= 0:
                i = int(mapo[u])
                nbr = [int(overlay_nodes[j]) for j in range(n_o) if oadj[i, j]]
                if not nbr:
                    raise ValueError(f"overlay node {i} has no overlay neighbour")
                ts.extend([u] * len(nbr))
                td.extend(nbr)
            ov_row_ptr[u + 1] = len(td)
        tun_src = np.array(ts, dtype=np.int32)
        tun_dst = np.array(td, dtype=np.int32)
        tun_link = np.array([index[(int(a), int(hop[a, b]))] for a, b in zip(ts, td)], dtype=np.int32)
        tun_len = np.array([int(dist[a, b]) for a, b in zip(ts, td)], dtype=np.int32)

        fs, fd, fr, fb = [], [], [], []
        for i in range(n):
            for j in range(n):
                if i == j or mapo[i] < 0 or mapo[j] < 0:
                    continue                       # activateUnderlayTraffic=0: overlay pairs only
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
                   overlay_index=overlay_index, overlay_nodes=overlay_nodes, overlay_adj=oadj,
                   ov_row_ptr=ov_row_ptr, tun_src=tun_src, tun_dst=tun_dst, tun_link=tun_link,
                   tun_len=tun_len, next_hop=hop, dist=dist, tm_strings=tm)

    @classmethod
    def from_files(cls, physical_adjacency: str, overlay_adjacency: str, map_overlay: str,
                   traffic_matrix: str, load_factor: float = 1.0, name: str = "custom") -> "Topology":
        phys = read_square(physical_adjacency)
        over = read_square(overlay_adjacency)
        mapo = read_map_overlay(map_overlay)
        tm = read_square(traffic_matrix, kind=str)
        return cls.from_matrices(phys, tm, load_factor=load_factor, name=name,
                                 map_overlay=mapo, overlay_adjacency=over)

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


def _overlay_lists(topo: Topology) -> List[List[int]]:
    n_o = topo.n_overlay
    return [[j for j in range(n_o) if topo.overlay_adj[i, j]] for i in range(n_o)]


def sp_next_hop_table(topo: Topology) -> np.ndarray:
    """[N, N] uint8 action table indexed by UNDERLAY ids (node, destination):
    index (into neighbors(u)) of the SP next hop on the overlay graph G
    (forwarder.py:190-191 runs nx.shortest_path on the overlay graph, in
    overlay indices, argument_parser.py:127).

    Diagonal entries (packet at its destination) and rows/columns of
    non-overlay nodes are 0 (forwarder.py:149-150 sends action 0 there).
    """
    n = topo.n_nodes
    lists = _overlay_lists(topo)
    on = topo.overlay_nodes
    table = np.zeros((n, n), dtype=np.uint8)
    for i in range(topo.n_overlay):
        for j in range(topo.n_overlay):
            if i == j:
                continue
            nxt = _bidirectional_path(lists, i, j)[1]
            table[on[i], on[j]] = lists[i].index(nxt)
    return table


def sp_paths(topo: Topology) -> dict:
    """SP paths on the overlay graph, in overlay indices."""
    lists = _overlay_lists(topo)
    n_o = topo.n_overlay
    return {(u, d): _bidirectional_path(lists, u, d) for u in range(n_o) for d in range(n_o) if u != d}


# ----------------------------------------------------------------------
# Config 5: Erdos-Renyi G(256, 8/255) overlay with a uniform TM.
# No reference counterpart (the reference's /24 addressing caps it below ~250
# nodes, sim.cc:443-447); its files are generated once by
# scripts/make_er256.py into data/er256 and shipped like the other examples.
# ----------------------------------------------------------------------
WIRE_BITS_PER_PAYLOAD_BIT = (512 + 30) / 512       # 542-B frames per 512-B payload


def erdos_renyi_adjacency(n: int = 256, p: float = 8 / 255, seed: int = 100) -> np.ndarray:
    """G(n, p) from numpy's PCG64 stream `seed`: the upper triangle is drawn as one
    n x n uniform matrix per attempt, attempts repeat until the graph is connected."""
    rng = np.random.default_rng(seed)
    while True:
        u = rng.random((n, n))
        a = np.triu((u < p).astype(np.int32), 1)
        a = a + a.T
        seen = np.zeros(n, dtype=bool)
        seen[0] = True
        frontier = [0]
        while frontier:
            nxt = np.flatnonzero(a[frontier].any(axis=0) & ~seen)
            seen[nxt] = True
            frontier = list(nxt)
        if seen.all() and a.sum(axis=1).min() > 0:
            return a


def sp_link_loads(topo: Topology, rates: np.ndarray, table: np.ndarray) -> np.ndarray:
    """Wire bits/s offered to every directed link when each pair (s, d) sends
    rates[s, d] payload bits/s along the SP agent's path (action table)."""
    load = np.zeros(topo.n_links)
    n = topo.n_nodes
    for s in range(n):
        for d in range(n):
            if s == d or rates[s, d] <= 0:
                continue
            u = s
            while u != d:
                l = int(topo.row_ptr[u]) + int(table[u, d])
                load[l] += rates[s, d] * WIRE_BITS_PER_PAYLOAD_BIT
                u = int(topo.link_dst[l])
    return load


def erdos_renyi_scenario(n: int = 256, p: float = 8 / 255, seed: int = 100, max_rate_bps: float = 64000.0,
                         link_cap: int = 500000, max_util: float = 1.0):
    """(adjacency, integer TM in b/s, SP table): rates U(0, max_rate_bps) per ordered
    pair (the same PCG64 stream, after the graph), scaled so that the most loaded
    link carries max_util * link_cap wire bits/s under SP routing, truncated to
    whole b/s (zero rates create no flow, sim.cc:604)."""
    adj = erdos_renyi_adjacency(n, p, seed)
    rng = np.random.default_rng([seed, 1])
    u = rng.uniform(0.0, max_rate_bps, (n, n))
    np.fill_diagonal(u, 0.0)
    unit = Topology.from_matrices(adj, np.ones((n, n), dtype=np.int64) - np.eye(n, dtype=np.int64), name="er")
    table = sp_next_hop_table(unit)
    load = sp_link_loads(unit, u, table)
    scale = max_util * link_cap / load.max()
    tm = np.floor(u * scale).astype(np.int64)
    return adj, tm, table
