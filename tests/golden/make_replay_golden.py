"""Generate tests/golden/replay_buffer.json from the reference's own ReplayBuffer
(/root/reference/prisma/source/replay_buffer.py:12-37, imported here, run in the build
container only; nothing of it is copied, only the states it reaches are kept).

One ReplayBuffer per node (forwarder.py keeps one per agent, sized replay_buffer_max_size),
fed a fixed seeded sequence of transition batches in the order the Forwarders would add
them; after every batch the fixture records, per node: len(storage), _next_idx,
total_samples and the tag (obs_t[0]) of every stored transition in storage order, plus the
full stored tuples of the final state.

Usage: python tests/golden/make_replay_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/prisma"

N, SIZE, W = 5, 7, 4
BATCHES = (3, 20, 1, 40, 0, 9, 7, 14)       # includes batches that overflow a ring


def sequence():
    """The transition batches: (node, obs_t, action, reward, obs_tp1, done) lists."""
    rng = np.random.default_rng(20261016)
    uid = 0
    out = []
    for b in BATCHES:
        node = rng.integers(0, N, b)
        obs = np.zeros((b, W), dtype=np.int64)
        obs[:, 0] = np.arange(uid, uid + b)
        obs[:, 1:] = rng.integers(0, 16260, (b, W - 1))
        nxt = obs.copy()
        nxt[:, 1:] = rng.integers(0, 16260, (b, W - 1))
        action = rng.integers(0, 3, b)
        reward = np.round(rng.random(b) * 0.05, 6)
        done = rng.random(b) < 0.3
        out.append({"node": node.tolist(), "obs": obs.tolist(), "next_obs": nxt.tolist(),
                    "action": action.tolist(), "reward": reward.tolist(), "done": done.tolist()})
        uid += b
    return out


def main():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from source.replay_buffer import ReplayBuffer      # the reference's own class
    bufs = [ReplayBuffer(SIZE) for _ in range(N)]
    batches = sequence()
    states = []
    for bt in batches:
        for i, u in enumerate(bt["node"]):
            bufs[u].add(bt["obs"][i], bt["action"][i], bt["reward"][i], bt["next_obs"][i], bt["done"][i])
        states.append([{"len": len(b), "next_idx": b._next_idx, "total_samples": b.total_samples,
                        "tags": [int(d[0][0]) for d in b._storage]} for b in bufs])
    final = [[{"obs": list(map(int, d[0])), "action": int(d[1]), "reward": float(d[2]),
               "next_obs": list(map(int, d[3])), "done": bool(d[4])} for d in b._storage] for b in bufs]
    fx = {"source": "reference source/replay_buffer.py ReplayBuffer.add (imported), one buffer per node",
          "n_nodes": N, "size": SIZE, "obs_width": W, "batches": batches, "states": states, "final": final}
    with open(os.path.join(HERE, "replay_buffer.json"), "w") as fh:
        json.dump(fx, fh, indent=0)
    print("wrote", os.path.join(HERE, "replay_buffer.json"))


if __name__ == "__main__":
    main()
