"""Generate tests/golden/prio_replay_buffer.json from the reference's own
PrioritizedReplayBuffer (/root/reference/prisma/source/replay_buffer.py:393-534, imported here,
run in the build container only; nothing of it is copied, only the states it reaches are kept).

One buffer per node, as agent.py:66-67 builds them (alpha 1, one priority class per neighbour),
driven by a fixed seeded script of the three operations the Forwarder performs on it:
  * add(obs, action, reward, next_obs, done, prio)      forwarder.py:227-233, 495-501
  * a newer gradient step for an action: latest_gradient_step[action] = step and
    update_priorities(neighbors_idx[action], action)     forwarder.py:502-505
  * sample(batch_size)                                   trainer.py:51
After every operation the fixture keeps the node's priorities of the stored slots (the sum
tree's leaves), its tree total, max priority, latest gradient steps, neighbors_idx lists and
storage tags; a sample keeps the indices Python's `random` drew (seeded) and the importance
weights, so the restatement can be fed the same indices.

Usage: python tests/golden/make_prio_replay_golden.py
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/prisma"

DEGREES = (2, 3, 1)
SIZE, W = 6, 4                # capacity rounds up to 8 leaves: the unused leaves stay 0


def script():
    rng = np.random.default_rng(20261017)
    ops = []
    uid = 0
    latest = [[1] * d for d in DEGREES]
    for k in range(90):
        u = int(rng.integers(0, len(DEGREES)))
        x = rng.random()
        if x < 0.6:
            a = int(rng.integers(0, DEGREES[u]))
            obs = [uid] + rng.integers(0, 16260, W - 1).tolist()
            nxt = [uid] + rng.integers(0, 16260, W - 1).tolist()
            # the gradient step the transition's target came from: at most the latest one known
            prio = int(rng.integers(1, latest[u][a] + 3))
            ops.append({"op": "add", "node": u, "obs": obs, "action": a, "reward": round(float(rng.random()) * 0.05, 6),
                        "next_obs": nxt, "done": bool(rng.random() < 0.3), "prio": prio})
            uid += 1
        elif x < 0.8:
            a = int(rng.integers(0, DEGREES[u]))
            step = latest[u][a] + int(rng.integers(0, 4))
            latest[u][a] = max(latest[u][a], step)
            ops.append({"op": "grad", "node": u, "action": a, "step": step})
        else:
            ops.append({"op": "sample", "node": u, "batch": int(rng.integers(1, 6))})
    return ops


def state(b):
    n = len(b._storage)
    return {"len": n, "next_idx": b._next_idx, "total_samples": b.total_samples,
            "tags": [int(d[0][0]) for d in b._storage],
            "prio": [float(b._it_sum[i]) for i in range(n)], "prio_min": [float(b._it_min[i]) for i in range(n)],
            "tree_sum": float(b._it_sum.sum()), "max_priority": float(b._max_priority),
            "latest_gradient_step": [int(x) for x in b.latest_gradient_step],
            "neighbors_idx": [[int(i) for i in l] for l in b.neighbors_idx]}


def main():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from source.replay_buffer import PrioritizedReplayBuffer      # the reference's own class
    random.seed(1234)
    bufs = [PrioritizedReplayBuffer(SIZE, 1, d, u) for u, d in enumerate(DEGREES)]
    ops = script()
    trace = []
    for op in ops:
        b = bufs[op["node"]]
        rec = {}
        if op["op"] == "add":
            # ndarrays (a 0-d one for the action): the reference's _encode_sample calls
            # np.array(x, copy=False), which numpy 2 refuses for Python lists and scalars
            b.add(np.array(op["obs"]), np.array(op["action"]), op["reward"], np.array(op["next_obs"]), op["done"],
                  op["prio"])
        elif op["op"] == "grad":
            a = op["action"]
            if op["step"] > b.latest_gradient_step[a]:
                b.latest_gradient_step[a] = op["step"]
                if len(b.neighbors_idx[a]):
                    b.update_priorities(b.neighbors_idx[a], a)
        else:
            if len(b) == 0:
                rec["skipped"] = True
            else:
                st = random.getstate()
                out = b.sample(op["batch"])
                random.setstate(st)
                idx = [random.randint(0, len(b._storage) - 1) for _ in range(op["batch"])]
                rec["idx"] = idx
                rec["weights"] = [float(w) for w in out[5]]
                rec["tags"] = [int(o[0]) for o in out[0]]
        rec["state"] = state(b)
        trace.append(rec)
    fx = {"source": "reference source/replay_buffer.py PrioritizedReplayBuffer (imported), one buffer per node, "
                    "alpha 1 (agent.py:66-67)",
          "degrees": list(DEGREES), "size": SIZE, "obs_width": W, "alpha": 1.0, "ops": ops, "trace": trace}
    with open(os.path.join(HERE, "prio_replay_buffer.json"), "w") as fh:
        json.dump(fx, fh, indent=0)
    print("wrote", os.path.join(HERE, "prio_replay_buffer.json"))


if __name__ == "__main__":
    main()
