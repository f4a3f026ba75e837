#!/usr/bin/env python3
"""Host-resident (PCIe-inclusive) rates for DESIGN.md §6.1 — north_star: "this
path starts and ends in host memory ... the rate including the H2D/D2H copies
must also be measured".  Not the bench.py `value` (that one is device-resident).

  host-batch encode      : pinned payloads -> H2D -> encode -> D2H all shards
  host-batch reconstruct : pinned compacted present shards (threshold of them)
                           -> H2D -> scatter + locator + reconstruct -> D2H payload
  C ABI per call         : ECCR_obtain_chunks / ECCR_reconstruct (pageable
                           buffers, per-shard malloc, as a reference caller)
  mixed stream           : README sizes {15 B .. 10 MB} through the host-batch
                           API, one batch per size class, automatic chunking
                           (config 5 shape, 1 GPU)
Prints one JSON object.
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
import synth  # noqa: E402


def pinned(shape, dtype=torch.uint8):
    return torch.empty(shape, dtype=dtype, pin_memory=True)


def timeit(fn, reps):
    fn()  # warm (allocations, first-touch)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def host_batch(nv, plen, batch, chunk, reps):
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    pay = pinned((batch, plen))
    for c0 in range(0, batch, 64):
        pay[c0:c0 + 64] = synth.payloads_torch(list(range(c0, min(batch, c0 + 64))), plen,
                                               device="cuda").cpu()
    sh = pinned((batch, nv, sl))
    t_enc = timeit(lambda: E.encode_host_batch(nv, pay, plen, plen, batch, sh, sl, chunk), reps)
    idx = np.stack([np.sort(synth.present_set(10**6 + b, nv, thr)) for b in range(batch)])
    idx_t = torch.from_numpy(idx.astype(np.uint16).view(np.int16)).pin_memory()
    comp = pinned((batch, thr, sl))
    shn = sh.numpy()
    for b in range(batch):
        comp[b] = torch.from_numpy(shn[b][idx[b]])
    out = pinned((batch, sl * k))
    t_rec = timeit(lambda: E.reconstruct_host_batch(nv, comp, sl, sl, idx_t, thr, batch, out,
                                                    sl * k, chunk), reps)
    ok = bool(torch.equal(out[:, :plen], pay))
    gib = batch * plen / 2**30
    return {"payload_bytes": plen, "batch": batch, "chunk": chunk,
            "encode_GiBps": round(gib / t_enc, 3), "reconstruct_GiBps": round(gib / t_rec, 3),
            "encode_pcie_GBps": round(batch * (plen + nv * sl) / t_enc / 1e9, 2),
            "reconstruct_pcie_GBps": round(batch * (thr * sl + k * sl) / t_rec / 1e9, 2),
            "roundtrip_GiBps": round(gib / (t_enc + t_rec), 3), "roundtrip_ok": ok,
            "encode_s": t_enc, "reconstruct_s": t_rec}


def capi_per_call(nv, plen, reps):
    p = synth.payload(7, plen).tobytes()
    n, k, thr = E.code_params(nv)
    keep = set(int(x) for x in synth.present_set(11, nv, thr))
    sh = E.obtain_chunks(nv, p)
    t_enc = timeit(lambda: E.obtain_chunks(nv, p), reps)
    chunks = [(i, sh[i]) for i in range(nv) if i in keep]
    t_rec = timeit(lambda: E.reconstruct(nv, chunks), reps)
    assert E.reconstruct(nv, chunks)[:plen] == p
    return {"payload_bytes": plen, "obtain_chunks_ms": round(t_enc * 1e3, 3),
            "reconstruct_ms": round(t_rec * 1e3, 3),
            "roundtrip_GiBps": round(plen / (t_enc + t_rec) / 2**30, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nv", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--chunk", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    assert E.lib().ECCR_AMD_init_device().tag == 0, E.last_error()
    res = {"what": "host-resident (PCIe-inclusive) rates, 1 GPU", "n_validators": a.nv,
           "host_batch_1MB": host_batch(a.nv, 1_000_000, a.batch, a.chunk, a.reps),
           "capi_per_call_1MB": capi_per_call(a.nv, 1_000_000, a.reps)}
    mixed = []
    for plen, batch in ((15, 4096), (300, 4096), (5000, 2048), (100000, 512), (1_000_000, 128),
                        (10_000_000, 16)):
        mixed.append(host_batch(a.nv, plen, batch, 0, 2))  # chunk 0: library sizes the steps
    res["mixed_stream"] = mixed
    tot_b = sum(m["payload_bytes"] * m["batch"] for m in mixed)
    tot_t = sum(m["encode_s"] + m["reconstruct_s"] for m in mixed)
    res["mixed_stream_roundtrip_GiBps"] = round(tot_b / 2**30 / tot_t, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
