"""Generate BASELINE config 5's scenario files: Erdos-Renyi G(256, 8/255),
seed 100, connected; uniform TM scaled to a maximum SP link utilisation of 1.0.

Writes prisma_amd/data/er256/{topology_files,traffic_matrices} in the reference's
example format (identity overlay) and the SP agent's next-hop table
(sp_next_hop_table.npy, the networkx tie-break) so runs need
not recompute its 65 280 bidirectional BFS paths.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from prisma_amd.topology import DATA_DIR, erdos_renyi_scenario  # noqa: E402


def write_matrix(path, m):
    with open(path, "w") as fh:                       # no trailing newline (Appendix E)
        fh.write("\n".join(" ".join(str(int(x)) for x in row) for row in m))


def main():
    adj, tm, table = erdos_renyi_scenario()
    n = adj.shape[0]
    root = os.path.join(DATA_DIR, "er256")
    os.makedirs(os.path.join(root, "topology_files"), exist_ok=True)
    os.makedirs(os.path.join(root, "traffic_matrices"), exist_ok=True)
    write_matrix(os.path.join(root, "topology_files", "physical_adjacency_matrix.txt"), adj)
    write_matrix(os.path.join(root, "topology_files", "overlay_adjacency_matrix.txt"), adj)
    with open(os.path.join(root, "topology_files", "map_overlay.txt"), "w") as fh:
        fh.write("\n".join(str(i) for i in range(n)))
    write_matrix(os.path.join(root, "traffic_matrices", "node_intensity_normalized_0.txt"), tm)
    np.save(os.path.join(root, "sp_next_hop_table.npy"), table)
    deg = adj.sum(axis=1)
    print(f"ER-256: {int(adj.sum())} directed links, degree {deg.min()}..{deg.max()} (mean {deg.mean():.2f}), "
          f"{int((tm > 0).sum())} flows, {tm.sum() / 1e6:.2f} Mb/s offered")


if __name__ == "__main__":
    main()
