"""numpy views of the C-ABI record and counter layouts (include/prisma.h)."""
from __future__ import annotations

import numpy as np

ST_PENDING, ST_ENQUEUED, ST_DROPPED, ST_DESTINATION, ST_DISCARDED = 0, 1, 2, 3, 4

EBIT_RING, EBIT_WIRE, EBIT_ACKORDER, EBIT_TIME, EBIT_LOGWRAP, EBIT_PINGIDX = 1, 2, 4, 8, 16, 32


def record_dtype(obs_width: int) -> np.dtype:
    """prisma_record_t with obs_width observation words (32 + 4*W bytes)."""
    if obs_width % 4:
        raise ValueError("obs_width must be a multiple of 4")
    return np.dtype([
        ("t_ns", "<i8"), ("uid", "<u4"), ("prev", "<i4"), ("reward", "<f8"),
        ("node", "u1"), ("dst", "u1"), ("start_s", "<u2"), ("action", "i1"), ("status", "u1"),
        ("ttl", "u1"), ("episode", "u1"), ("obs", "<u4", (obs_width,)),
    ])


COUNTERS_DTYPE = np.dtype([
    ("events", "<u8"), ("hops", "<u8"), ("decisions", "<u8"), ("hop_deg_sum", "<u8"),
    ("now_ns", "<i8"), ("reward_sum", "<f8"),
    ("ov_injected", "<i4"), ("ov_arrived", "<i4"), ("ov_lost", "<i4"),
    ("un_injected", "<i4"), ("un_arrived", "<i4"), ("un_lost", "<i4"),
    ("bytes_data", "<i4"), ("bytes_signaling", "<i4"),
    ("cost_sum", "<f4"), ("e2e_sum", "<f4"), ("cost_n", "<i4"), ("e2e_n", "<i4"),
    ("episode", "<u4"), ("ping_rounds", "<u4"), ("seq", "<u4"), ("uid", "<u4"),
    ("dec_count", "<u4"), ("ctrl_dropped", "<u4"), ("error", "<u4"), ("episode_over", "<u4"),
    ("hops_total", "<u8"), ("events_total", "<u8"),
    ("un_cost_sum", "<f4"), ("un_cost_n", "<i4"),
])
assert COUNTERS_DTYPE.itemsize == 152


def transitions(records: np.ndarray, loss_penalty: float):
    """Join decision records into replay transitions (forwarder.py:352-379, 214-244).

    Returns a dict of arrays (obs, action, reward, next_obs, done, node) for
    every decision whose outcome is known: forwarded hops completed by a later
    record (prev == d) and dropped hops (loss transition with the fixed
    penalty and next_obs = [dst, 0, ...]).  ``records`` must be the contiguous
    log of one replica starting at decision index ``records_base`` = index of
    records[0] (taken from the uid order: records are in decision order).
    """
    n = records.shape[0]
    W = records["obs"].shape[1]
    obs, act, rew, nxt, done, node = [], [], [], [], [], []
    base = 0
    for k in range(n):
        r = records[k]
        p = int(r["prev"])
        if p >= base and p - base < n:
            q = records[p - base]
            obs.append(q["obs"]); act.append(int(q["action"])); rew.append(float(r["reward"]))
            nxt.append(r["obs"]); done.append(int(r["status"]) == ST_DESTINATION); node.append(int(q["node"]))
        if int(r["status"]) == ST_DROPPED:
            o = np.zeros(W, dtype=np.uint32)
            o[0] = r["obs"][0]
            obs.append(r["obs"]); act.append(int(r["action"])); rew.append(float(loss_penalty))
            nxt.append(o); done.append(True); node.append(int(r["node"]))
    return {
        "obs": np.array(obs, dtype=np.uint32).reshape(-1, W), "action": np.array(act, dtype=np.int64),
        "reward": np.array(rew, dtype=np.float64), "next_obs": np.array(nxt, dtype=np.uint32).reshape(-1, W),
        "done": np.array(done, dtype=bool), "node": np.array(node, dtype=np.int64),
    }
