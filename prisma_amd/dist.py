"""Multi-GPU = replica sharding: no exchange while stepping.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm,
"gloo" for the CPU tests).  Rank k owns the contiguous replica ids
[base_k, base_k + R_k); its Philox key words are those global ids, so any
sharding reproduces the single-GPU replicas bit for bit.  The only
collective is one all-gather of per-replica episode statistics (returns,
delivered/lost/injected counters) at the end of a run: at most
16384 x 8 x 8 B = 1 MB, latency-bound on xGMI.
"""
from __future__ import annotations

import numpy as np

STAT_FIELDS = ("reward_sum", "episode", "hops_total", "ov_injected", "ov_arrived", "ov_lost",
               "cost_sum", "cost_n", "now_ns")


def shard(total: int, rank: int, world: int):
    """(replica_base, n_replicas) of `rank` for `total` replicas over `world` ranks."""
    if not (0 <= rank < world) or total < world:
        raise ValueError("need 0 <= rank < world <= total")
    per, extra = divmod(total, world)
    base = rank * per + min(rank, extra)
    return base, per + (1 if rank < extra else 0)


def replica_stats(counters: np.ndarray) -> np.ndarray:
    """[R, len(STAT_FIELDS)] float64 per-replica episode statistics."""
    return np.stack([counters[f].astype(np.float64) for f in STAT_FIELDS], axis=1)


def gather_replica_stats(counters: np.ndarray, world: int, device=None) -> dict:
    """All-gather every rank's per-replica statistics and summarise.

    Ranks may hold different replica counts (shard() of a total that world does not divide):
    the counts are all-gathered first, every rank pads its block to the largest, and the
    padding is cut out again, so the result is always [total, F] in global replica order.
    Returns {"stats": [total, F] ndarray, "episodes_completed": int, "mean_return": float,
    "delivered": int, "lost": int}.
    """
    import torch
    import torch.distributed as dist
    local = torch.from_numpy(replica_stats(counters))
    # the collective runs whenever a process group is up (also a 1-rank group: bench.py --force-dist)
    if world > 1 or (dist.is_available() and dist.is_initialized()):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" \
                else torch.device("cpu")
        n = torch.tensor([local.shape[0]], dtype=torch.int64, device=device)
        sizes = torch.empty(world, dtype=torch.int64, device=device)
        dist.all_gather_into_tensor(sizes, n)
        sizes = [int(x) for x in sizes.cpu().tolist()]
        width = max(sizes)
        block = torch.zeros((width, local.shape[1]), dtype=local.dtype, device=device)
        block[:local.shape[0]] = local.to(device)
        out = torch.empty((world * width, local.shape[1]), dtype=local.dtype, device=device)
        dist.all_gather_into_tensor(out, block)
        out = out.cpu().numpy()
        allst = np.concatenate([out[r * width: r * width + sizes[r]] for r in range(world)])
    else:
        allst = local.numpy()
    ep = allst[:, STAT_FIELDS.index("episode")]
    return {
        "stats": allst,
        "episodes_completed": int(ep.sum()),
        "mean_return": float(allst[:, STAT_FIELDS.index("reward_sum")].mean()),
        "delivered": int(allst[:, STAT_FIELDS.index("ov_arrived")].sum()),
        "lost": int(allst[:, STAT_FIELDS.index("ov_lost")].sum()),
    }
