"""Multi-rank path on CPU (gloo, world_size 2): the payload sharding bench.py
uses is disjoint and complete, ranks agree on the mixed-size partition without
communicating, the max-over-ranks timing is the max, and encoding each rank's
shard of payloads (oracle, CPU) gives exactly the single-process result —
i.e. sharding by payload needs no data-path collective."""
import hashlib
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "erasure-coding-crust_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import sharding  # noqa: E402
import synth  # noqa: E402

NV, PLEN, PER_RANK = 16, 3001, 3
MIXED = [15, 300, 5000, 100000, 1000, 7, 4096, 65536, 300, 15]


def _digest(oracle, seeds):
    h = hashlib.sha256()
    for s in seeds:
        for shard in oracle.encode(NV, synth.payload(s, PLEN).tobytes()):
            h.update(shard)
    return h.hexdigest()


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import oracle as orc
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seeds = sharding.rank_seeds(rank, PER_RANK)
        all_seeds = [None] * world
        dist.all_gather_object(all_seeds, seeds)
        parts = sharding.balanced_partition(MIXED, world)
        all_parts = [None] * world
        dist.all_gather_object(all_parts, parts)
        mx = sharding.max_over_ranks(10.0 + rank, dist)
        digests = [None] * world
        dist.all_gather_object(digests, _digest(orc.Oracle(), seeds))
        if rank == 0:
            q.put((all_seeds, all_parts, mx, digests))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_sharding(oracle):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        all_seeds, all_parts, mx, digests = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    # weak-scaling ownership: disjoint, complete, independent of world size
    flat = [s for r in all_seeds for s in r]
    assert sorted(flat) == list(range(world * PER_RANK))
    # every rank computed the same byte-balanced partition of the mixed stream
    assert all(p == all_parts[0] for p in all_parts)
    parts = all_parts[0]
    assert sorted(i for p in parts for i in p) == list(range(len(MIXED)))
    loads = [sum(MIXED[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(MIXED)
    assert mx == 11.0
    # sharded encode == single-process encode of the same payloads
    single = [_digest(oracle, sharding.rank_seeds(r, PER_RANK)) for r in range(world)]
    assert digests == single


@pytest.mark.parametrize("total,world", [(10, 3), (8, 8), (3, 4), (4096, 8)])
def test_contiguous_range(total, world):
    covered = []
    for r in range(world):
        s, c = sharding.contiguous_range(r, world, total)
        covered += list(range(s, s + c))
    assert covered == list(range(total))


def test_balanced_partition_deterministic():
    a = sharding.balanced_partition(MIXED, 4)
    assert a == sharding.balanced_partition(list(MIXED), 4)
    assert sorted(i for p in a for i in p) == list(range(len(MIXED)))


def _sg_worker(rank, world, port, q):
    """gloo rehearsal of bench.py's scatter / gather (the RCCL path runs the
    same calls on GPU tensors): the root holds every rank's payloads, scatters
    them, each rank encodes + reconstructs its slice on the CPU oracle, and the
    decoded payloads are gathered back to the root."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import oracle as orc
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        per, plen, nv = 2, 777, 6
        o = orc.Oracle()
        n, k = o.params(nv)
        sl = o.shard_len(k, plen)
        whole = None
        if rank == 0:
            seeds = [s for r in range(world) for s in sharding.rank_seeds(r, per)]
            whole = torch.from_numpy(np.stack([synth.payload(s, plen) for s in seeds])).view(world, per, plen)
        mine = torch.empty((per, plen), dtype=torch.uint8)
        sharding.scatter_from_root(dist, whole, mine, rank, world)
        want = np.stack([synth.payload(s, plen) for s in sharding.rank_seeds(rank, per)])
        ok_scatter = bool((mine.numpy() == want).all())
        dec = []
        for b in range(per):
            sh = o.encode(nv, mine[b].numpy().tobytes())
            keep = [sh[i] if i % 2 == 0 else None for i in range(nv)]
            dec.append(np.frombuffer(o.reconstruct(nv, keep), np.uint8))
        dec = torch.from_numpy(np.stack(dec))
        assert dec.shape == (per, sl * k)
        gathered = torch.zeros((world, per, sl * k), dtype=torch.uint8) if rank == 0 else None
        sharding.gather_to_root(dist, dec, gathered, rank, world)
        oks = [None] * world
        dist.all_gather_object(oks, ok_scatter)
        if rank == 0:
            ok_gather = bool((gathered[:, :, :plen].reshape(world * per, plen) ==
                              whole.reshape(world * per, plen)).all())
            q.put((oks, ok_gather))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_scatter_gather_rehearsal(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        oks, ok_gather = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(oks) and ok_gather


def _bench_sg_worker(rank, world, port, q):
    """bench.py's scatter_gather() itself, on gloo with CPU tensors (the box
    runs it on RCCL with device tensors): payloads scattered from the root,
    outputs gathered back, checked, timed."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B, plen, ob = 3, 1001, 1024
        dev = torch.device("cpu")
        d_pay = synth.payloads_torch(sharding.rank_seeds(rank, B), plen, device=dev).contiguous()
        d_out = torch.zeros((B, ob), dtype=torch.uint8)
        d_out[:, :plen] = d_pay  # a correct reconstruction
        r = bench.scatter_gather(dist, rank, world, dev, B, plen, d_pay, d_out, 1e-3, 120.0)
        if rank == 0:
            q.put(r)
    finally:
        dist.destroy_process_group()


def test_bench_scatter_gather_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_bench_sg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        r = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert r["ok"] and r["scatter_bytes"] == 3 * 1001 and r["gather_bytes"] == 3 * 1024



def _bench_sg_hang_worker(rank, world, port):
    """rank 0 enters bench.scatter_gather, rank 1 never joins the collective:
    the watchdog must end rank 0 with the timeout status (bench.EXIT_SG_TIMEOUT),
    not 0, after printing the marked line."""
    import time
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if rank == 1:
        time.sleep(20)
        os._exit(0)
    B, plen = 2, 101
    dev = torch.device("cpu")
    d_pay = torch.zeros((B, plen), dtype=torch.uint8)
    bench.scatter_gather(dist, rank, world, dev, B, plen, d_pay, d_pay.clone(), 1e-3, 3.0,
                         lambda: print('{"marked": true}', flush=True))
    os._exit(0)  # not reached: the watchdog exits first


def test_bench_scatter_gather_timeout_exits_nonzero():
    import torch.multiprocessing as mp
    sys.path.insert(0, ROOT)
    import bench
    ctx = mp.get_context("spawn")
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_bench_sg_hang_worker, args=(r, world, port)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert procs[0].exitcode == bench.EXIT_SG_TIMEOUT == 3


def _rank_table_worker(rank, world, port, q):
    """bench.py's per-rank evidence on gloo: every rank's
    device_info + own step time, all-gathered in rank order."""
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        info = dict(bench.device_info(rank), rank=rank, step_ms=1.0 + rank)
        table = sharding.rank_table(info, dist)
        mx = sharding.max_over_ranks(1.0 + rank, dist)
        if rank == 0:
            q.put((table, mx))
    finally:
        dist.destroy_process_group()


def test_rank_table_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_rank_table_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        table, mx = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert [t["rank"] for t in table] == [0, 1] and [t["device"] for t in table] == [0, 1]
    assert all(set(t) >= {"rank", "device", "name", "pci_bus_id", "step_ms"} for t in table), table
    assert mx == max(t["step_ms"] for t in table) == 2.0
    assert sharding.rank_table({"rank": 0}) == [{"rank": 0}]  # one process: no group needed
