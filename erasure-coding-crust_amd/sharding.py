"""Payload sharding across ranks (one process per GPU) — SURVEY.md §8e.

Payloads are independent, so the multi-GPU path is a partition of the payload
set with no data-path collective; RCCL (or gloo in the CPU tests) carries only
the barrier and the max-over-ranks timing.

* weak scaling (bench.py): every rank owns `per_rank` payloads whose synthetic
  seeds are global payload indices, so the data a payload gets does not depend
  on the world size;
* a fixed stream of mixed-size payloads (BASELINE config 5): a byte-balanced
  greedy partition (largest first onto the least-loaded rank), deterministic
  so every rank computes the same assignment without communicating.
"""
from __future__ import annotations

import heapq


def rank_seeds(rank: int, per_rank: int) -> list[int]:
    """Global payload indices owned by `rank` under weak scaling."""
    return list(range(rank * per_rank, (rank + 1) * per_rank))


def contiguous_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """(start, count) of `rank`'s block when `total` payloads are split evenly."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def balanced_partition(sizes: list[int], world: int) -> list[list[int]]:
    """Indices of `sizes` per rank, greedy longest-processing-time by bytes.

    Ties are broken by rank then index, so the result is a pure function of
    (sizes, world): ranks agree without exchanging anything."""
    order = sorted(range(len(sizes)), key=lambda i: (-sizes[i], i))
    heap = [(0, r) for r in range(world)]
    parts: list[list[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        parts[r].append(i)
        heapq.heappush(heap, (load + sizes[i], r))
    for p in parts:
        p.sort()
    return parts


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """Max of a per-rank scalar (the step time) over the process group."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
