"""Scenario construction vs the reference's own outputs (tests/golden, from parse_arguments + networkx)."""
import json
import os

import numpy as np
import pytest

from prisma_amd.topology import Topology, parse_data_rate, sp_next_hop_table, sp_paths, loss_penalty
from prisma_amd.config import engine_params, parse_arguments

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    with open(os.path.join(GOLD, f"reference_{name}.json")) as fh:
        return json.load(fh)


@pytest.mark.parametrize("text,expect", [
    ("0bps", 0), ("499.89bps", 499), ("6.11Kbps", 6110), ("32.66Kbps", 32659), ("8.11Kbps", 8109),
    ("500000bps", 500000), ("500Kbps", 500000), ("1.5Mbps", 1500000), ("83.85bps", 83), ("2B/s", 16),
])
def test_ns3_datarate_truncating_parse(text, expect):
    # ns-3 DataRate::DoParse: (uint64_t)(double(r) * multiplier), 1000-based units
    assert parse_data_rate(text) == expect


@pytest.mark.parametrize("name", ["abilene", "geant"])
def test_neighbour_order_matches_reference(name):
    g = gold(name)
    t = Topology.example(name)
    assert t.n_nodes == g["numNodes"]
    for u in range(t.n_nodes):
        assert t.neighbors(u) == g["neighbors"][str(u)]


def test_abilene_known_neighbours():
    # SURVEY Appendix A item 7
    t = Topology.example("abilene")
    expect = {0: [1, 2, 3], 1: [0, 4, 5], 2: [0, 4, 6], 3: [0, 7], 4: [1, 2, 8], 5: [1, 9], 6: [2, 7],
              7: [3, 6], 8: [4, 9, 10], 9: [5, 8, 10], 10: [8, 9]}
    assert {u: t.neighbors(u) for u in range(11)} == expect
    assert t.n_links == 28 and t.max_deg == 3 and t.obs_width == 4


@pytest.mark.parametrize("name", ["abilene", "geant"])
def test_loss_penalty_matches_reference(name):
    g = gold(name)
    t = Topology.example(name)
    assert loss_penalty(16260, 512, 500000, t.n_nodes) == g["loss_penalty"]
    assert engine_params(t)["loss_penalty"] == g["loss_penalty"]


@pytest.mark.parametrize("name", ["abilene", "geant"])
def test_sp_table_matches_networkx(name):
    g = gold(name)
    t = Topology.example(name)
    table = sp_next_hop_table(t)
    paths = sp_paths(t)
    for key, path in g["sp_paths"].items():
        u, d = map(int, key.split(","))
        assert paths[(u, d)] == path, key
        assert t.neighbors(u)[table[u, d]] == path[1]


def test_sp_tie_pairs_exist():
    # a plain BFS tie-break would not match: SURVEY Appendix B counts 15 / 154 tie pairs
    import itertools
    for name, want in (("abilene", 15), ("geant", 154)):
        t = Topology.example(name)
        n = t.n_nodes
        dist = np.full((n, n), 10 ** 6)
        for s in range(n):
            dist[s, s] = 0
            frontier = [s]
            while frontier:
                nxt = []
                for v in frontier:
                    for w in t.neighbors(v):
                        if dist[s, w] > dist[s, v] + 1:
                            dist[s, w] = dist[s, v] + 1
                            nxt.append(w)
                frontier = nxt
        ties = sum(1 for u, d in itertools.permutations(range(n), 2)
                   if sum(1 for w in t.neighbors(u) if dist[w, d] == dist[u, d] - 1) > 1)
        assert ties == want


@pytest.mark.parametrize("name", ["abilene", "geant"])
def test_flow_rates_match_fixture(name):
    g = gold(name)
    for k in range(4):
        t = Topology.example(name, k, 1.0)
        rates = g["tm_rates_bps"][str(k)]
        expect = [(i, j, rates[i][j]) for i in range(t.n_nodes) for j in range(t.n_nodes)
                  if i != j and rates[i][j] > 0]
        got = list(zip(t.flow_src.tolist(), t.flow_dst.tolist(), t.flow_rate_bps.tolist()))
        assert got == expect


def test_load_factor_ceil():
    t1 = Topology.example("abilene", 0, 1.0)
    t2 = Topology.example("abilene", 0, 1.5)
    assert np.array_equal(t2.flow_rate_bps, np.ceil(t1.flow_base_bps.astype(np.float64) * 1.5).astype(np.uint64))


def test_reference_defaults():
    g = gold("abilene")["defaults"]
    p = parse_arguments([])
    for k, v in g.items():
        assert p[k] == v, k


def test_bad_inputs_fail_loudly():
    with pytest.raises(ValueError):
        Topology.from_matrices(np.ones((3, 3)), [["0bps"] * 3] * 3)      # self loops
    with pytest.raises(ValueError):
        Topology.from_matrices(np.array([[0, 1], [0, 0]]), [["0bps"] * 2] * 2)  # asymmetric
    with pytest.raises(ValueError):
        Topology.from_matrices(np.array([[0, 1], [1, 0]]), [["0bps"] * 3] * 3)  # TM shape (sim.cc:310)
    with pytest.raises(ValueError):
        # the shipped overlay example has an 11x11 TM 1 for a 6-node underlay: NS_FATAL_ERROR (sim.cc:310-313)
        Topology.example("overlay_full_mesh_3n_abilene", 1)


def test_overlay_example_tunnels_known_answer():
    """overlay_full_mesh_3n_abilene (prisma/examples/...): 6-node underlay, overlay nodes
    0,2,4,5 (map 0 -1 1 -1 2 3), full mesh.  Paths checked by hand against the ns-3 global
    routing rule (lowest-id neighbour on a shortest path; topology.py docstring):
    2->4 and 4->2 tie between 1 and 3 and take 1; 0<->5 cross overlay node 2."""
    t = Topology.example("overlay_full_mesh_3n_abilene")
    assert t.n_nodes == 6 and t.n_overlay == 4 and not t.identity
    assert list(t.overlay_nodes) == [0, 2, 4, 5] and list(t.overlay_index) == [0, -1, 1, -1, 2, 3]
    assert {u: t.neighbors(u) for u in (0, 2, 4, 5)} == {0: [2, 4, 5], 2: [0, 4, 5], 4: [0, 2, 5], 5: [0, 2, 4]}
    paths = {(int(t.tun_src[k]), int(t.tun_dst[k])): t.tunnel_path(k) for k in range(t.n_tunnels)}
    assert paths == {(0, 2): [0, 2], (0, 4): [0, 1, 4], (0, 5): [0, 2, 5], (2, 0): [2, 0], (2, 4): [2, 1, 4],
                     (2, 5): [2, 5], (4, 0): [4, 1, 0], (4, 2): [4, 1, 2], (4, 5): [4, 3, 5], (5, 0): [5, 2, 0],
                     (5, 2): [5, 2], (5, 4): [5, 3, 4]}
    assert list(t.tun_len) == [len(paths[(int(a), int(b))]) - 1 for a, b in zip(t.tun_src, t.tun_dst)]
    # flows only between overlay pairs, underlay (i, j) order (sim.cc:494-514, 599-631)
    assert list(zip(t.flow_src.tolist(), t.flow_dst.tolist())) == [
        (0, 2), (0, 4), (0, 5), (2, 0), (2, 4), (2, 5), (4, 0), (4, 2), (4, 5), (5, 0), (5, 2), (5, 4)]
    assert int(t.flow_rate_bps[7]) == 83                    # "83.85bps" truncates
    # loss penalty counts overlay nodes (argument_parser.py:127-128,163)
    assert engine_params(t)["loss_penalty"] == loss_penalty(16260, 512, 500000, 4)
    # SP agent on the overlay graph (forwarder.py:190-191): full mesh -> direct tunnel
    table = sp_next_hop_table(t)
    for u in (0, 2, 4, 5):
        for d in (0, 2, 4, 5):
            if u != d:
                assert t.neighbors(u)[table[u, d]] == d


def test_er256_config5_files():
    """BASELINE config 5 data (scripts/make_er256.py): G(256, 8/255) seed 100, connected,
    identity overlay; the TM loads the busiest SP link to 1.0 of capacity (wire bits,
    within the truncation to whole b/s); the shipped SP table is the agent's."""
    from prisma_amd.topology import DATA_DIR, erdos_renyi_adjacency, sp_link_loads
    topo = Topology.example("er256")
    assert topo.n_nodes == 256 and topo.identity
    assert np.array_equal(topo.adjacency, erdos_renyi_adjacency(256, 8 / 255, 100))
    assert topo.n_links == 2008 and topo.max_deg == 19 and topo.phys_degrees.min() == 1
    assert topo.n_flows == 65251 and topo.obs_width == 20
    table = np.load(f"{DATA_DIR}/er256/sp_next_hop_table.npy")
    rates = np.zeros((256, 256))
    rates[topo.flow_src, topo.flow_dst] = topo.flow_rate_bps.astype(np.float64)
    util = sp_link_loads(topo, rates, table) / 500000.0
    assert 0.999 < util.max() <= 1.0
    # every table entry is a valid action; following it reaches the destination
    deg = topo.degrees
    assert np.all(table < deg[:, None])
