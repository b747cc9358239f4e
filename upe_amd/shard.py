"""Static sharding of the hot path over GPUs.

Each packet's verdict depends only on its bytes and the read-only tables, except for the one-entry
L1 neighbour caches, which belong to a worker exactly as in the reference (one `worker_t` per
thread, `include/worker.h:50-58`).  So a batch splits into contiguous static shards, one per GPU,
with the tables replicated and no data-path collective; counters and rule_stats are summed the
way the reference's stats thread sums its workers (`src/main.c:293-315`).  torch.distributed is
used only for the barrier around a timed region and the max / sum of the per-rank results.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from .layout import desc_offsets


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous static range [rank * n / world, (rank + 1) * n / world)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return n * rank // world, n * (rank + 1) // world


def shard_workload(wl, rank: int, world: int):
    """This rank's contiguous shard of a synth.Workload: its own packed frames buffer (offsets
    rebased to the shard's first frame) and descriptors; tables replicated; a calloc'd L1 state,
    as a freshly started worker has."""
    from .layout import l1_zero

    s, e = shard_range(wl.n, rank, world)
    desc = wl.desc[s:e]
    if desc.size == 0:
        return dataclasses.replace(wl, frames=np.zeros(256, np.uint8), desc=desc.copy(),
                                   arp=wl.arp.copy(), ndp=wl.ndp.copy(), l1=l1_zero())
    offs = desc_offsets(desc)
    lo = int(offs.min())
    hi = min(int(offs.max()) + 2048 + 128, wl.frames.shape[0])
    frames = wl.frames[lo:hi].copy()
    rebased = (desc - np.uint64(lo << 16)).astype(np.uint64)
    return dataclasses.replace(wl, frames=frames, desc=rebased, arp=wl.arp.copy(),
                               ndp=wl.ndp.copy(), l1=l1_zero())


def max_over_ranks(value: float, dist, device="cpu") -> float:
    """The slowest rank's time (the job ends when the last shard does)."""
    if dist is None:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, dist, device="cpu") -> np.ndarray:
    """Element-wise sum of per-rank integer arrays (counters, rule_stats) across ranks."""
    a = np.ascontiguousarray(np.asarray(values, dtype=np.int64))
    if dist is None:
        return a
    import torch

    t = torch.from_numpy(a.copy()).to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()
