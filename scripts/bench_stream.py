#!/usr/bin/env python3
"""BASELINE config 5 driver: a mixed-size payload stream (the README sizes
15 B .. 10 MB, round-robin), end-to-end from host memory (pinned H2D, encode,
D2H of every shard; then H2D of threshold-many compacted shards, error
locator + reconstruct, D2H of the payload), sharded over the GPUs of one node.

One process per GPU under torchrun (RCCL for the barrier / max timing only):
the stream is split by `sharding.balanced_partition` (byte-balanced, the same
on every rank without communicating); each rank pushes its payloads through
the host-batch pipeline, one batch per size class (ECCR_AMD_*_host_batch,
chunk = 0).  Whole-job rate = stream bytes / max-over-ranks time.

  python scripts/bench_stream.py                      # 1 GPU
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
      scripts/bench_stream.py                         # 8 GPUs
ECCR_BENCH_BACKEND=gloo (rehearsal only, as bench.py): ranks may share a GPU,
the barrier / max timing run on CPU tensors over gloo.
Prints one JSON line on rank 0; exit status 1 if a round trip failed.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "erasure-coding-crust_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ecc_amd as E  # noqa: E402
import sharding  # noqa: E402
import synth  # noqa: E402

README_SIZES = [15, 300, 5000, 100_000, 1_000_000, 10_000_000]  # README.md:50-84


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nv", type=int, default=1024)
    ap.add_argument("--per-size", type=int, default=48, help="payloads of each size in the stream")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("ECCR_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # collective tensors
    assert E.lib().ECCR_AMD_init_device().tag == 0, E.last_error()
    nv = a.nv
    n, k, thr = E.code_params(nv)

    sizes = [README_SIZES[i % len(README_SIZES)] for i in range(a.per_size * len(README_SIZES))]
    mine = sharding.balanced_partition(sizes, world)[rank]
    classes = {}
    for i in mine:
        classes.setdefault(sizes[i], []).append(i)

    # untimed setup: pinned payloads, shard buffers, compacted reconstruct inputs
    work = []
    for plen, ids in sorted(classes.items()):
        B, sl = len(ids), E.shard_len(nv, plen)
        pay = torch.empty((B, plen), dtype=torch.uint8, pin_memory=True)
        for c0 in range(0, B, 16):
            pay[c0:c0 + 16] = synth.payloads_torch(ids[c0:c0 + 16], plen, device=dev).cpu()
        sh = torch.empty((B, nv, sl), dtype=torch.uint8, pin_memory=True)
        E.encode_host_batch(nv, pay, plen, plen, B, sh, sl, 0)
        idx = np.stack([synth.present_set(10**6 + i, nv, thr) for i in ids]).astype(np.uint16)
        comp = torch.empty((B, thr, sl), dtype=torch.uint8, pin_memory=True)
        shn = sh.numpy()
        for b in range(B):
            comp[b] = torch.from_numpy(shn[b][idx[b]])
        idx_t = torch.from_numpy(idx.view(np.int16)).pin_memory()
        out = torch.empty((B, sl * k), dtype=torch.uint8, pin_memory=True)
        work.append((plen, B, sl, pay, sh, comp, idx_t, out))

    def one_pass():
        for plen, B, sl, pay, sh, comp, idx_t, out in work:
            E.encode_host_batch(nv, pay, plen, plen, B, sh, sl, 0)
        for plen, B, sl, pay, sh, comp, idx_t, out in work:
            E.reconstruct_host_batch(nv, comp, sl, sl, idx_t, thr, B, out, sl * k, 0)

    one_pass()  # warm-up (pipeline buffers)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        one_pass()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    el = sharding.max_over_ranks(t1 - t0, dist, cdev)
    ok = all(torch.equal(out[:, :plen], pay) for plen, B, sl, pay, sh, comp, idx_t, out in work)
    if dist:
        f = torch.tensor([int(ok)], dtype=torch.int32, device=cdev)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = bool(f.item())
    total = sum(sizes) * a.reps
    line = {"metric": "config5 mixed-size stream, end-to-end host->device->host encode + reconstruct",
            "value": round(total / el / 2**30, 3), "unit": "GiB/s",
            "n_gpus": world if backend == "nccl" else min(world, max(torch.cuda.device_count(), 1)),
            "n_validators": nv, "stream_payloads": len(sizes), "stream_bytes": sum(sizes),
            "sizes": README_SIZES, "reps": a.reps, "seconds": round(el, 4),
            "present_shards": thr, "my_payloads": len(mine), "roundtrip_ok": ok,
            "partition": "sharding.balanced_partition (bytes, greedy LPT)"}
    if backend != "nccl":
        line["rehearsal"] = f"{world} ranks on {line['n_gpus']} GPU(s), {backend}"
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
