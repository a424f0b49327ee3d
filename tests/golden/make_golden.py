"""Generate the committed golden fixtures (run in the build container only).

Sources (nothing from the reference is copied; only its outputs are kept):
  * the reference's own ``source.argument_parser.parse_arguments`` imported
    from /root/reference (with ``nx.from_numpy_matrix`` shimmed to
    ``from_numpy_array``: networkx 3.x here, the reference pins 2.8.7):
    numNodes, neighbour lists (= the agents' action order) and loss_penalty;
  * ``networkx.shortest_path(G, u, d)`` on the reference's DiGraph ``G`` —
    the SP agent's decision rule (forwarder.py:190-191) — for every pair;
  * Philox4x32-10 known-answer vectors published with Random123
    (Salmon et al., SC'11; kat_vectors) for the RNG the engine uses;
  * the ns-3 DataRate truncating parse of every traffic-matrix entry,
    computed with the C++-equivalent double arithmetic (checked by the
    hand-computed examples in tests/test_topology.py).

Usage: python tests/golden/make_golden.py   (writes tests/golden/*.json)
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/prisma"


def reference_params(topology: str) -> dict:
    import networkx as nx
    nx.from_numpy_matrix = nx.from_numpy_array
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from source.argument_parser import parse_arguments  # the reference's own code
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "examples", topology), exist_ok=True)
        os.chdir(tmp)
        try:
            ex = f"{REF}/examples/{topology}"
            sys.argv = ["main.py", f"--topology_name={topology}",
                        f"--physical_adjacency_matrix_path={ex}/topology_files/physical_adjacency_matrix.txt",
                        f"--overlay_adjacency_matrix_path={ex}/topology_files/overlay_adjacency_matrix.txt",
                        f"--map_overlay_path={ex}/topology_files/map_overlay.txt",
                        f"--traffic_matrix_root_path={ex}/traffic_matrices/",
                        f"--logs_parent_folder={tmp}/logs"]
            p = parse_arguments()
        finally:
            os.chdir(cwd)
    G = p["G"]
    sp = {}
    for u in G.nodes:
        for d in G.nodes:
            if u != d:
                sp[f"{u},{d}"] = [int(x) for x in nx.shortest_path(G, u, d)]
    return {
        "numNodes": int(p["numNodes"]),
        "loss_penalty": p["loss_penalty"],
        "neighbors": {str(u): [int(x) for x in G.neighbors(u)] for u in G.nodes},
        "defaults": {k: p[k] for k in ("simTime", "seed", "load_factor", "max_out_buffer_size", "link_delay",
                                       "packet_size", "link_cap", "pingAsObs", "pingPacketIntervalTime",
                                       "movingAverageObsSize", "train", "agent_type", "signaling_type")},
        "sp_paths": sp,
        "networkx_version": nx.__version__,
    }


# Random123 kat_vectors, philox4x32 10 rounds: (ctr[4], key[2]) -> out[4]
PHILOX_KAT = [
    ([0x00000000, 0x00000000, 0x00000000, 0x00000000], [0x00000000, 0x00000000],
     [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff], [0xffffffff, 0xffffffff],
     [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


def tm_rates(topology: str) -> dict:
    sys.path.insert(0, REPO)
    from prisma_amd.topology import read_square, parse_data_rate
    out = {}
    for k in range(4):
        tm = read_square(f"{REPO}/prisma_amd/data/{topology}/traffic_matrices/node_intensity_normalized_{k}.txt",
                         kind=str)
        out[str(k)] = [[parse_data_rate(str(x)) for x in row] for row in tm]
    return out


def main():
    for topo in ("abilene", "geant"):
        data = reference_params(topo)
        data["tm_rates_bps"] = tm_rates(topo)
        with open(os.path.join(HERE, f"reference_{topo}.json"), "w") as fh:
            json.dump(data, fh, indent=1, sort_keys=True)
    with open(os.path.join(HERE, "philox_kat.json"), "w") as fh:
        json.dump([{"ctr": c, "key": k, "out": o} for c, k, o in PHILOX_KAT], fh, indent=1)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
