"""Payload sharding across ranks (one process per GPU) — SURVEY.md §8e.

Payloads are independent, so the multi-GPU path is a partition of the payload
set with no data-path collective; RCCL (or gloo in the CPU tests) carries the
barrier and the max-over-ranks timing, and -- only when a batch starts or ends
on one GPU -- the trivial scatter / gather below (grouped point-to-point sends
and receives: ncclGroupStart; ncclSend / ncclRecv; ncclGroupEnd under RCCL,
each rank's slice on its own xGMI link from the root).

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


def rank_table(info: dict, dist=None) -> list[dict]:
    """Every rank's `info` (its device, PCI bus id, own step time ...), in rank
    order, on every rank: the evidence that a multi-GPU line ran on N distinct
    devices and how far the slowest rank is from the others (VERDICT r04
    item 7).  One process: [info]."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [dict(info)]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, dict(info))
    return out


def scatter_from_root(dist, src, dst, rank: int, world: int, root: int = 0) -> None:
    """Root sends slice r of `src` ([world][...]; only read on the root) to rank
    r; every rank (root included) receives its slice into `dst`.  One grouped
    batch of point-to-point ops, so the root's sends run concurrently."""
    if world == 1:
        dst.copy_(src[0])
        return
    ops = []
    if rank == root:
        for r in range(world):
            if r != root:
                ops.append(dist.P2POp(dist.isend, src[r], r))
    else:
        ops.append(dist.P2POp(dist.irecv, dst, root))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    if rank == root and dst.data_ptr() != src[root].data_ptr():
        dst.copy_(src[root])


def gather_to_root(dist, src, dst, rank: int, world: int, root: int = 0) -> None:
    """Inverse of scatter_from_root: rank r's `src` lands in dst[r] on the root
    (`dst` [world][...] is only written on the root)."""
    if world == 1:
        dst[0].copy_(src)
        return
    ops = []
    if rank == root:
        for r in range(world):
            if r != root:
                ops.append(dist.P2POp(dist.irecv, dst[r], r))
    else:
        ops.append(dist.P2POp(dist.isend, src, root))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    if rank == root and dst[root].data_ptr() != src.data_ptr():
        dst[root].copy_(src)

