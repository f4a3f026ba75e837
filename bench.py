#!/usr/bin/env python3
"""Device-resident encode+reconstruct throughput (BASELINE.json metric).

One step = for a batch of independent payloads already resident in HBM:
  ECCR_AMD_encode_batch   (payload -> n_validators shards, ec-cpp encode)
  ECCR_AMD_error_locator  (per-payload erasure pattern -> log multipliers)
  ECCR_AMD_reconstruct_batch (random `threshold`-of-n shards -> payload)
value = total payload bytes of all ranks / max-over-ranks step time, GiB/s.

Multi-GPU: one process per GPU, payloads sharded by rank with no data-path
collective (weak scaling); RCCL only for the barrier / max-timing (and the
separately timed scatter / gather of a GPU0-resident batch).  Under torchrun
(WORLD_SIZE set) this process is one rank and WORLD_SIZE must equal --gpus;
run directly with --gpus N > 1 it starts N fresh rank processes itself (before
any GPU call), relays rank 0's JSON line and exits with the worst rank status.

Prints ONE JSON line on rank 0 (contract in the task statement), with a
`roofline` object for the dominant kernel (HIP events on the launch stream)
and a `cpu_baseline` timed on this host (the reference ec-cpp built in
oracle/_ref if present, else the C restatement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "erasure-coding-crust_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ecc_amd as E  # noqa: E402
import sharding  # noqa: E402
import synth  # noqa: E402

METRIC = "device-resident encode+reconstruct GiB/s (and % HBM roofline), n_val=1024"
HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md)
# exit status: 0 ok; 1 a round trip / scatter-gather check failed; 3 the RCCL
# scatter / gather hung (watchdog); 4 it raised.  The JSON line is printed first
# in every case, so the measurement is kept and marked.
EXIT_CHECK, EXIT_USAGE, EXIT_SG_TIMEOUT, EXIT_SG_ERROR = 1, 2, 3, 4


def pmc_traffic(kernel, nv, plen, cnt, batch):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (scripts/pmc_traffic.sh + scripts/pmc_summary.py, newest profiles/rNN),
    when it was measured on this workload shape; scaled linearly in batch."""
    import glob
    # (profiles/rNN/pmc_traffic.json: the default workload; c4_pmc_traffic.json
    # and the like: other shapes, picked by the workload check below)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "*pmc_traffic.json")),
                       reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
            w = d["workload"]
            if (w["n_validators"], w["payload_bytes"], w["present"]) != (nv, plen, cnt):
                continue
            return d["kernels"][kernel]["hbm_bytes_per_payload"] * batch, os.path.relpath(path, ROOT)
        except (OSError, KeyError, ValueError):
            continue
    return None, None


# waves per SIMD of the dominant kernels (launch shapes in csrc/): the SQ
# counters' per-wave VALU instruction rate summed over a SIMD's waves (the
# VALU instructions one SIMD issued per quad-cycle), and the per-wave wait
# fractions beside it.
_WAVES_PER_SIMD = {"reconstruct": (("reconstruct_n1024x", 3), ("reconstruct_n1024<false>", 2), ("reconstruct_n1024", 2)),
                   "encode": (("encode_k256w", 4), ("encode_k256<1024, 0>", 4), ("encode_k256<1024>", 4))}


def sq_issue(kernel, nv):
    """SQ issue counters of `kernel` from the committed SQ counter summary
    (scripts/prof_r5.sh + scripts/sq_summary.py, newest profiles/rNN), measured
    on the default workload shape (nv = 1024): the kernels are bounded by
    instruction issue, not HBM."""
    import glob
    names = _WAVES_PER_SIMD.get(kernel)
    if names is None or nv != 1024:
        return None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "sq_counters.json")),
                       reverse=True):
        try:
            with open(path) as f:
                ks = json.load(f)["kernels"]
            name, waves = next((n, w) for n, w in names if n in ks)  # (kernel names by round)
            k = ks[name]
            # SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU: it counts instructions
            # (per quad-cycle of SQ_WAVE_CYCLES), not VALU busy time; the
            # busy fraction needs per-opcode prices (profiles/r05/*_account.md)
            per_quad = k["frac_active_valu"] * waves
            return {"kernel": name, "waves_per_simd": waves,
                    "valu_insts_per_simd_quad_cycle": round(per_quad, 3),
                    "cycles_per_valu_inst": round(4.0 / per_quad, 2) if per_quad else None,
                    "wave_wait_any_frac": round(k["frac_wait_any"], 3),
                    "wave_wait_inst_any_frac": round(k["frac_wait_inst_any"], 3),
                    "measured_in_this_run": False,
                    "source": os.path.relpath(path, ROOT) + " (stored SQ counter profile)",
                    "account": "profiles/r05/enc_valu_account.md, profiles/r05/rec_account.md"}
        except (OSError, KeyError, ValueError, StopIteration):
            continue
    return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(nv, plen, cnt, seconds, threads_all=None):
    """The reference ec-cpp (oracle/_ref, -O3) on this host's cores, on a
    bounded sample of the same workload: 1 thread, then `threads` threads with
    one payload per thread.  `threads` is the GPU box's CPU
    share per GPU (16: the pool's rule for worker pools on a one-GPU lease),
    or `threads_all` (--cpu-threads) when the whole host may be used; the
    usable-CPU count and the 16-thread rate scaled to it are reported beside
    (labelled as an extrapolation, not a measurement).  The C restatement
    (1 thread) stands in if the reference build is absent."""
    import oracle as orc
    kind = "reference" if orc.RefEC.available() else "port"
    impl = orc.RefEC() if kind == "reference" else orc.Oracle()
    p = synth.payload(424242, plen).tobytes()
    present = synth.present_mask(10**6, nv, cnt)
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = max(1, threads_all or min(usable, 16))
    res = {"unit": "GiB/s", "kind": kind, "cpu_model": cpu_model(), "host_cpus_usable": usable}
    if kind == "reference":
        d1, w1, e1, r1 = impl.time_mt(nv, p, present, 1, seconds)
        dn, wn, en, rn = impl.time_mt(nv, p, present, threads, seconds)
        rate = dn * plen / wn / 2**30
        res.update({
            "value": round(rate, 6), "cores": threads,
            "single_thread_GiBps": round(d1 * plen / w1 / 2**30, 6),
            "single_thread_encode_GiBps": round(d1 * plen / e1 / 2**30, 6),
            "single_thread_reconstruct_GiBps": round(d1 * plen / r1 / 2**30, 6),
            f"threads{threads}_GiBps": round(rate, 6),
            "all_usable_cpus_GiBps_extrapolated": (None if threads >= usable else
                                                   round(rate * usable / threads, 6)),
            "sample": f"ec-cpp -O3 (oracle/_ref): {plen} B payload encode + reconstruct from {cnt} of "
                      f"{nv} shards, repeated for ~{seconds:.0f} s on 1 thread ({d1} payloads) and on "
                      f"{threads} threads, one payload per thread ({dn} payloads)"
                      + ("" if threads >= usable else
                         f"; {threads} = the box's CPU share per GPU of {usable} usable CPUs "
                         "(--cpu-threads to use more)")})
        return res
    t_enc = t_dec = 0.0
    reps = 0
    t_start = time.perf_counter()
    while reps < 1 or time.perf_counter() - t_start < seconds:
        t0 = time.perf_counter()
        sh = impl.encode(nv, p)
        t1 = time.perf_counter()
        impl.reconstruct(nv, [sh[i] if present[i] else None for i in range(nv)])
        t_enc += t1 - t0
        t_dec += time.perf_counter() - t1
        reps += 1
    res.update({"value": round(reps * plen / (t_enc + t_dec) / 2**30, 6), "cores": 1,
                "sample": f"{reps} x ({plen} B payload encode + reconstruct from {cnt} of {nv} "
                          "shards), 1 thread, oracle/ec_oracle.c"})
    return res


# the reference's own benchmark sizes (benchmark/benchmark.cpp:36-45,
# README.md:50-84) and the per-GPU batch each is measured on
BENCH_SIZES = (15, 300, 5000, 100_000, 1_000_000, 10_000_000)
SWEEP_BATCH = {15: 4096, 300: 4096, 5000: 4096, 100_000: 1024, 1_000_000: 4096, 10_000_000: 400}


def cpu_size_rate(nv, plen, cnt, seconds, threads):
    """ec-cpp (oracle/_ref) encode + reconstruct rate at one payload size on
    this host: 1 thread and `threads` threads (one payload per thread)."""
    import oracle as orc
    if not orc.RefEC.available():
        return None
    ref = orc.RefEC()
    p = synth.payload(424242 + plen, plen).tobytes()
    present = synth.present_mask(10**6 + plen, nv, cnt)
    d1, w1, _, _ = ref.time_mt(nv, p, present, 1, seconds)
    dn, wn, _, _ = ref.time_mt(nv, p, present, threads, seconds)
    return {"GiBps_1thread": round(d1 * plen / w1 / 2**30, 6),
            f"GiBps_{threads}threads": round(dn * plen / wn / 2**30, 6)}


def device_info(local):
    """This rank's device: index, name and PCI location (a multi-GPU line must
    show N distinct bus ids).  Works without a GPU (CPU tests): nulls."""
    info = {"device": local, "name": None, "pci_bus_id": None}
    try:
        if torch.cuda.is_available():
            p = torch.cuda.get_device_properties(local)
            info["name"] = p.name
            bus = getattr(p, "pci_bus_id", None)
            if bus is not None:
                info["pci_bus_id"] = "%04x:%02x:%02x" % (getattr(p, "pci_domain_id", 0), bus,
                                                        getattr(p, "pci_device_id", 0))
    except Exception as exc:  # noqa: BLE001 (reported, never fatal)
        info["error"] = f"{type(exc).__name__}: {exc}"[:120]
    return info


def device_bandwidth(dev, nbytes=1 << 30, reps=5):
    """Measured device bandwidth on this box (the roofline also
    against a measured copy): a 1 GiB device-to-device copy (read + write
    bytes) and a 1 GiB fill (write bytes), HIP events on the current stream."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)
    b.copy_(a)
    out = {}
    for name, fn, moved in (("copy_GBps", lambda: b.copy_(a), 2 * nbytes),
                            ("fill_GBps", lambda: b.fill_(7), nbytes)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize(dev)
        out[name] = round(moved * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    del a, b
    torch.cuda.empty_cache()
    return out


def gf_mul_counts(nv, n, k, cnt):
    """GF(2^16) multiplies the reference algorithm executes (SURVEY.md §8d
    secondary ceiling; additive_fft.hpp:99-141 skips the 0xFFFF skews, one
    block per stage at index 0): encode per 2k-byte piece = inverse_afft(k) at
    0 + (n/k - 1) afft(k) at the cosets (poly_encoder.hpp:217-240); reconstruct
    per shard column = c locator products + inverse_afft(n) + afft(n) at 0 +
    the erased outputs y < k (poly_encoder.hpp:164-189; k - present data rows
    on average k (1 - c/nv))."""
    lk, ln = k.bit_length() - 1, n.bit_length() - 1
    ifft_k = k // 2 * lk - (k - 1)
    enc = ifft_k + (n // k - 1) * (k // 2 * lk)
    fft_n = n // 2 * ln - (n - 1)
    rec = cnt + 2 * fft_n + k * (1 - cnt / nv)
    return enc, rec


def size_sweep(args, nv, cnt_key, dev, stream, dist, world, rank, backend, headline):
    """Device-resident encode + locator + reconstruct at each benchmark/ size
    (north_star): the same step as the headline on synthetic payloads of that
    size, tight payload pitch (the packed kernels take small payloads), shard
    rows padded to 64 B; per size the whole-job GiB/s (max-over-ranks time),
    the dominant kernel's HBM roofline fraction, and ec-cpp on this host's
    cores beside it (rank 0).  Shard rows shorter than 64 B are tight (the
    reference's own shard buffers are exactly shard_len long).  The 1 MB row is
    the headline measurement."""
    n, k, thr = E.code_params(nv)
    cnt = {"threshold": thr, "k": k}.get(cnt_key) or int(cnt_key)
    threads = max(1, min(len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 1, 16))
    rows = []
    for plen in args.sweep_sizes:
        if plen == args.payload and args.batch == SWEEP_BATCH.get(plen) and headline is not None:
            row = dict(headline)
        else:
            B = SWEEP_BATCH.get(plen, max(1, min(4096, (4 << 30) // max(plen, 1))))
            sl = E.shard_len(nv, plen)
            # shard rows padded to 64 B (aligned vector stores), except rows
            # shorter than that, which stay tight: a 2-byte shard in a 64-byte
            # slot would make every shard write its own HBM burst (32x the bytes)
            ss = (sl + 63) // 64 * 64 if sl >= 64 else sl
            seeds = sharding.rank_seeds(rank, B)
            d_pay = torch.empty((B, plen), dtype=torch.uint8, device=dev)
            for c0 in range(0, B, 256):
                d_pay[c0:c0 + 256] = synth.payloads_torch(seeds[c0:c0 + 256], plen, device=dev)
            d_pres = torch.from_numpy(synth.present_masks([10**6 + s for s in seeds], nv, cnt, n)).to(dev)
            d_sh = torch.empty((B, nv, ss), dtype=torch.uint8, device=dev)
            d_el = torch.empty((B, n), dtype=torch.int16, device=dev)
            d_out = torch.empty((B, sl * k), dtype=torch.uint8, device=dev)
            ev = []

            def step(record):
                if record:
                    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                    e[0].record(stream)
                E.encode_batch(nv, d_pay, plen, plen, B, d_sh, ss, stream)
                if record:
                    e[1].record(stream)
                E.error_locator(nv, d_pres, B, d_el, stream)
                if record:
                    e[2].record(stream)
                E.reconstruct_batch(nv, d_sh, sl, ss, d_pres, d_el, B, d_out, sl * k, stream)
                if record:
                    e[3].record(stream)
                    ev.append(e)

            # sub-millisecond steps: more of them (launch latency and clock ramp
            # dominate a handful), as many on every rank
            steps = args.steps if plen >= args.payload else max(args.steps, 50)
            for _ in range(args.warmup if plen >= args.payload else max(args.warmup, 5)):
                step(False)
            torch.cuda.synchronize(dev)
            if dist:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                step(True)
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            if dist:
                dist.barrier()
            el = sharding.max_over_ranks(t1 - t0, dist, dev if backend == "nccl" else None)
            ok = bool(torch.equal(d_out[:, :plen], d_pay))
            ms = lambda a, b: float(np.mean([x[a].elapsed_time(x[b]) for x in ev]))  # noqa: E731
            t_enc, t_loc, t_rec = ms(0, 1), ms(1, 2), ms(2, 3)
            kern = {"encode": (t_enc, B * (plen + nv * sl)),
                    "reconstruct": (t_rec, B * (cnt + k) * sl + B * n * 2)}
            dom = max(kern, key=lambda x: kern[x][0])
            achieved = kern[dom][1] / (kern[dom][0] * 1e-3)
            row = {"payload_bytes": plen, "batch_per_gpu": B,
                   "steps": steps,
                   "ms_per_step": round(el / steps * 1e3, 4),
                   "GiBps": round(world * B * plen * steps / el / 2**30, 3),
                   "kernels_ms": {"encode": round(t_enc, 4), "error_locator": round(t_loc, 4),
                                  "reconstruct": round(t_rec, 4)},
                   "roofline": {"kernel": dom, "achieved_GBps": round(achieved / 1e9, 2),
                                "frac": round(achieved / HBM_PEAK, 5)},
                   "roundtrip_ok": ok}
            del d_pay, d_pres, d_sh, d_el, d_out
            torch.cuda.empty_cache()
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            row["cpu_ec_cpp"] = cpu_size_rate(nv, plen, cnt, args.sweep_cpu_seconds, threads)
        rows.append(row)
    return rows


def pcie_bandwidth(dev, nbytes=256 << 20, reps=4):
    """Measured pinned-host <-> device copy rates on this box (the PCIe bound of
    the host-resident path): H2D alone, D2H alone, and both at once on two
    streams (aggregate bytes / time), GB/s."""
    h_in = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).fill_(1)
    h_out = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_b = torch.ones(nbytes, dtype=torch.uint8, device=dev)
    s_h2d, s_d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps

    def duplex():
        with torch.cuda.stream(s_h2d):
            d_a.copy_(h_in, non_blocking=True)
        with torch.cuda.stream(s_d2h):
            h_out.copy_(d_b, non_blocking=True)

    t_h2d = timed(lambda: d_a.copy_(h_in, non_blocking=True))
    t_d2h = timed(lambda: h_out.copy_(d_b, non_blocking=True))
    t_dup = timed(duplex)
    del h_in, h_out, d_a, d_b
    torch.cuda.empty_cache()
    return {"h2d_GBps": round(nbytes / t_h2d / 1e9, 2), "d2h_GBps": round(nbytes / t_d2h / 1e9, 2),
            "duplex_GBps": round(2 * nbytes / t_dup / 1e9, 2), "bytes_per_copy": nbytes}


def _pcie_bound_s(pcie, h2d, d2h):
    """Least time the copies of a host-resident call can take on this box: PCIe
    is full duplex, so each direction at its own measured rate, at the same
    time.  (`duplex_GBps`, two torch copies on two streams, is reported beside
    it: on these boxes it has read as one direction's rate, i.e. those copies
    did not overlap, while the library's pipeline does overlap them.)"""
    return max(h2d / (pcie["h2d_GBps"] * 1e9), d2h / (pcie["d2h_GBps"] * 1e9))


def _host_class(nv, plen, ids, dev):
    """Pinned inputs of one payload-size class for the host-batch calls: the
    payloads, their shard buffer, the compacted threshold-many present shards
    (and their indices) of each, and the output buffer."""
    n, k, thr = E.code_params(nv)
    B, sl = len(ids), E.shard_len(nv, plen)
    pay = torch.empty((B, plen), dtype=torch.uint8, pin_memory=True)
    for c0 in range(0, B, 64):
        pay[c0:c0 + 64] = synth.payloads_torch(ids[c0:c0 + 64], plen, device=dev).cpu()
    sh = torch.empty((B, nv, sl), dtype=torch.uint8, pin_memory=True)
    E.encode_host_batch(nv, pay, plen, plen, B, sh, sl, 0)
    idx = np.stack([synth.present_set(10**6 + i, nv, thr) for i in ids]).astype(np.uint16)
    comp = torch.empty((B, thr, sl), dtype=torch.uint8, pin_memory=True)
    shn = sh.numpy()
    for b in range(B):
        comp[b] = torch.from_numpy(shn[b][idx[b].astype(np.int64)])
    idx_t = torch.from_numpy(idx.view(np.int16)).pin_memory()
    out = torch.empty((B, sl * k), dtype=torch.uint8, pin_memory=True)
    return {"plen": plen, "B": B, "sl": sl, "pay": pay, "sh": sh, "comp": comp, "idx": idx_t,
            "out": out}


def e2e(args, nv, dev, dist, world, rank, cdev):
    """north_star: "this path starts and ends in host memory ... the rate
    including the H2D/D2H copies must also be measured".  Through the
    host-batch pipeline (ECCR_AMD_encode_host_batch / _reconstruct_host_batch,
    csrc/host_pipeline.hip; reference: erasure_coding.rs:246-264,404-406 take
    and return host buffers), on every rank at once, max-over-ranks time:
      config 2 shape: B x 1 MB pinned payloads -> H2D -> encode -> D2H of every
        shard; then H2D of threshold-many compacted shards per payload ->
        locator + reconstruct -> D2H of the payload;
      config 5: the README size mix (15 B .. 10 MB, `--e2e-per-size` of each,
        byte-balanced over the ranks), the same two calls per size class.
    Each next to the PCIe bound from this box's measured pinned copy rates
    (H2D and D2H at their own rates, at once).
    Never the bench `value` (that one is device-resident)."""
    n, k, thr = E.code_params(nv)
    pcie = pcie_bandwidth(dev)

    def timed(fn, reps):
        fn()  # warm: pipeline slots, first touch
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        el = time.perf_counter() - t0
        if dist:
            dist.barrier()
        return sharding.max_over_ranks(el / reps, dist, cdev)

    def enc(c):
        E.encode_host_batch(nv, c["pay"], c["plen"], c["plen"], c["B"], c["sh"], c["sl"], 0)

    def rec(c):
        E.reconstruct_host_batch(nv, c["comp"], c["sl"], c["sl"], c["idx"], thr, c["B"], c["out"],
                                 c["sl"] * k, 0)

    def moved(c):  # PCIe bytes of the encode and of the reconstruct call
        B, plen, sl = c["B"], c["plen"], c["sl"]
        return (B * plen, B * nv * sl), (B * thr * (sl + 2), B * sl * k)

    # config 2 shape, a bounded batch per rank
    c2 = _host_class(nv, args.payload, sharding.rank_seeds(rank, args.e2e_batch), dev)
    t_e = timed(lambda: enc(c2), args.e2e_reps)
    t_r = timed(lambda: rec(c2), args.e2e_reps)
    (eh, ed), (rh, rd) = moved(c2)
    be, br = _pcie_bound_s(pcie, eh, ed), _pcie_bound_s(pcie, rh, rd)
    ok = bool(torch.equal(c2["out"][:, :args.payload], c2["pay"]))
    gib = world * c2["B"] * args.payload / 2**30
    cfg2 = {"payload_bytes": args.payload, "batch_per_gpu": c2["B"], "reps": args.e2e_reps,
            "encode_GiBps": round(gib / t_e, 3), "reconstruct_GiBps": round(gib / t_r, 3),
            "roundtrip_GiBps": round(gib / (t_e + t_r), 3),
            "pcie_bound_roundtrip_GiBps": round(gib / (be + br), 3),
            "frac_of_pcie_bound": round((be + br) / (t_e + t_r), 4),
            "encode_frac_of_pcie_bound": round(be / t_e, 4),
            "reconstruct_frac_of_pcie_bound": round(br / t_r, 4),
            "pcie_bytes_per_gpu": {"encode_h2d": eh, "encode_d2h": ed, "reconstruct_h2d": rh,
                                   "reconstruct_d2h": rd},
            "roundtrip_ok": ok}
    del c2
    # config 5: the README size mix
    sizes = [BENCH_SIZES[i % len(BENCH_SIZES)] for i in range(args.e2e_per_size * len(BENCH_SIZES))]
    mine = sharding.balanced_partition(sizes, world)[rank]
    by = {}
    for i in mine:
        by.setdefault(sizes[i], []).append(i)
    work = [_host_class(nv, plen, ids, dev) for plen, ids in sorted(by.items())]

    def one_pass():
        for c in work:
            enc(c)
        for c in work:
            rec(c)

    t_m = timed(one_pass, args.e2e_reps)
    bound = 0.0
    for c in work:
        (eh, ed), (rh, rd) = moved(c)
        bound += _pcie_bound_s(pcie, eh, ed) + _pcie_bound_s(pcie, rh, rd)
    bound = sharding.max_over_ranks(bound, dist, cdev)
    ok5 = all(torch.equal(c["out"][:, :c["plen"]], c["pay"]) for c in work)
    del work
    total = sum(sizes)
    cfg5 = {"sizes": list(BENCH_SIZES), "payloads": len(sizes), "stream_bytes": total,
            "reps": args.e2e_reps, "roundtrip_GiBps": round(total / t_m / 2**30, 3),
            "pcie_bound_roundtrip_GiBps": round(total / bound / 2**30, 3),
            "frac_of_pcie_bound": round(bound / t_m, 4),
            "partition": "sharding.balanced_partition (bytes, greedy LPT)", "roundtrip_ok": ok5}
    if dist:
        f = torch.tensor([int(ok and ok5)], dtype=torch.int32, device=cdev)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = ok5 = bool(f.item())
    return {"what": "host-resident path: pinned host -> H2D -> kernels -> D2H -> pinned host, "
                    "whole job over all ranks, max-over-ranks time (not the bench value)",
            "n_validators": nv, "present_shards": thr, "pcie_measured": pcie,
            "config2": cfg2, "config5_mixed": cfg5}, ok and ok5


def scatter_gather(dist, rank, world, dev, B, plen, d_pay, d_out, step_s, timeout_s,
                   on_timeout=None):
    """SURVEY.md §8e / north_star: the batch starts on GPU0 and the decoded
    payloads end there.  Rank 0 holds every rank's payloads, scatters them over
    RCCL (one grouped batch of ncclSend / ncclRecv: each rank's slice on its own
    xGMI link), and the reconstructed payloads are gathered back.  Timed apart
    from the device-resident step (barrier + synchronize around each phase, max
    over ranks) and checked: the scattered slices equal each rank's own
    payloads, the gathered outputs equal the root's copy of every payload."""
    import threading
    done = threading.Event()

    def watchdog():  # a hung collective must not cost the main measurement
        if not done.wait(timeout_s):
            print(json.dumps({"scatter_gather_timeout_s": timeout_s}), file=sys.stderr, flush=True)
            if on_timeout:
                on_timeout()  # rank 0: the measurement line, marked
            # non-zero: a hung collective is a failure of a north_star component
            os._exit(EXIT_SG_TIMEOUT)

    threading.Thread(target=watchdog, daemon=True).start()
    try:
        return _scatter_gather(dist, rank, world, dev, B, plen, d_pay, d_out, step_s)
    finally:
        done.set()


def _scatter_gather(dist, rank, world, dev, B, plen, d_pay, d_out, step_s):
    whole = None
    if rank == 0:
        whole = torch.empty((world, B, plen), dtype=torch.uint8, device=dev)
        for r in range(world):
            seeds = sharding.rank_seeds(r, B)
            for c0 in range(0, B, 256):
                whole[r, c0:c0 + 256] = synth.payloads_torch(seeds[c0:c0 + 256], plen, device=dev)
    recv = torch.empty((B, plen), dtype=torch.uint8, device=dev)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def timed(fn):
        sync()
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        fn()
        sync()
        t1 = time.perf_counter()
        dist.barrier()
        return sharding.max_over_ranks(t1 - t0, dist, dev)

    t_sc = timed(lambda: sharding.scatter_from_root(dist, whole, recv, rank, world))
    ok = int(torch.equal(recv, d_pay))
    del recv
    ob = d_out.shape[1]
    gath = torch.empty((world, B, ob), dtype=torch.uint8, device=dev) if rank == 0 else None
    t_ga = timed(lambda: sharding.gather_to_root(dist, d_out, gath, rank, world))
    if rank == 0:
        for r in range(world):
            ok &= int(torch.equal(gath[r, :, :plen], whole[r]))
        del gath, whole
    flag = torch.tensor([ok], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    sc_bytes = (world - 1) * B * plen
    ga_bytes = (world - 1) * B * ob
    return {"scatter_ms": round(t_sc * 1e3, 3), "scatter_bytes": sc_bytes,
            "scatter_GBps": round(sc_bytes / t_sc / 1e9, 2),
            "gather_ms": round(t_ga * 1e3, 3), "gather_bytes": ga_bytes,
            "gather_GBps": round(ga_bytes / t_ga / 1e9, 2),
            "rate_incl_scatter_gather_GiBps": round(world * B * plen / (t_sc + step_s + t_ga) / 2**30, 3),
            "collective": "RCCL grouped ncclSend/ncclRecv (torch.distributed batch_isend_irecv)",
            "ok": bool(flag.item())}


def launch_ranks(n, backend, grace_s=60.0):
    """`python bench.py --gpus N` without a launcher: start N rank processes of
    this script (fresh interpreters, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    in their environment, one per GPU: LOCAL_RANK = RANK), before this process
    makes any GPU call (it never makes one).  Their output is inherited, so
    rank 0's JSON line is the line printed.  Returns the worst exit status: the
    largest non-zero one, a signal as 128 + signo; once a rank has failed the
    others get `grace_s` to finish before they are terminated (a rank blocked
    in a collective with a dead peer would otherwise hang)."""
    import signal
    import socket
    import subprocess
    if backend == "nccl":
        have = torch.cuda.device_count()  # (counting does not initialise the GPU)
        if have < n:
            print(json.dumps({"error": f"--gpus {n} needs {n} visible GPUs, {have} found"}),
                  file=sys.stderr, flush=True)
            return EXIT_USAGE
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []

    def forward(signo, _frame):  # the parent killed alone must not leave ranks holding GPUs
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        deadline = time.monotonic() + 15
        for p in procs:
            try:
                p.wait(max(deadline - time.monotonic(), 0.1))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        os._exit(128 + signo)

    for signo in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(signo, forward)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    status = {}
    failed_at = None
    while len(status) < n:
        for r, p in enumerate(procs):
            if r not in status and p.poll() is not None:
                status[r] = p.returncode
                if p.returncode != 0 and failed_at is None:
                    failed_at = time.monotonic()
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for r, p in enumerate(procs):
                if r not in status:
                    p.send_signal(signal.SIGTERM)
            for r, p in enumerate(procs):
                if r not in status:
                    try:
                        status[r] = p.wait(15)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        status[r] = p.wait()
        time.sleep(0.05)
    codes = [c if c >= 0 else 128 - c for c in status.values()]
    return max(codes)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="payloads per GPU")
    ap.add_argument("--payload", type=int, default=1_000_000)
    ap.add_argument("--nv", type=int, default=1024)
    ap.add_argument("--present", default="threshold", help="'threshold', 'k' or a count")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="CPU baseline sample per leg (1 thread, all cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the multi-thread CPU baseline leg (default: min(usable, 16), "
                         "the GPU box's CPU share per GPU)")
    ap.add_argument("--no-scatter", action="store_true",
                    help="skip the RCCL scatter / gather phase (N > 1)")
    ap.add_argument("--scatter-timeout", type=float, default=180.0)
    ap.add_argument("--sweep", default="bench",
                    help="'bench': also measure the benchmark/ payload sizes (15 B .. 10 MB) at "
                         "n_validators=nv and report them in `sizes`; 'none': skip; or a comma list")
    ap.add_argument("--sweep-cpu-seconds", type=float, default=0.5,
                    help="ec-cpp sample per size and thread count in the sweep")
    ap.add_argument("--row-stride", type=int, default=0,
                    help="device shard row stride in bytes (0: shard_len rounded up to --row-align)")
    ap.add_argument("--row-align", type=int, default=64,
                    help="device shard row stride = shard_len rounded up to this many bytes")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the host-resident (PCIe-inclusive) `e2e` block")
    ap.add_argument("--e2e-batch", type=int, default=256,
                    help="1 MB-class payloads per GPU in the e2e config-2 leg")
    ap.add_argument("--e2e-per-size", type=int, default=16,
                    help="payloads of each README size in the e2e config-5 stream (whole job)")
    ap.add_argument("--e2e-reps", type=int, default=3)
    ap.add_argument("--graph", action="store_true",
                    help="time K replays of one captured hipGraph step (ECCR_AMD_*_ws calls on "
                         "caller-owned scratch) instead of K eager steps")
    args = ap.parse_args()
    args.sweep_sizes = (() if args.sweep == "none" else BENCH_SIZES if args.sweep == "bench"
                        else tuple(int(x) for x in args.sweep.split(",")))

    # ECCR_BENCH_BACKEND=gloo (rehearsal only): ranks may share a GPU, the
    # barrier / max-timing run on CPU tensors.  Default: one rank per GPU, RCCL.
    backend = os.environ.get("ECCR_BENCH_BACKEND", "nccl")
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, backend))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(json.dumps({"error": f"--gpus {args.gpus} but WORLD_SIZE={world}: the launcher's "
                                   "rank count must equal --gpus"}), file=sys.stderr, flush=True)
        sys.exit(EXIT_USAGE)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend != "nccl":
        local %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    assert E.lib().ECCR_AMD_init_device().tag == 0, E.last_error()

    nv, plen, B = args.nv, args.payload, args.batch
    n, k, thr = E.code_params(nv)
    cnt = {"threshold": thr, "k": k}.get(args.present) or int(args.present)
    sl = E.shard_len(nv, plen)
    ss = (sl + args.row_align - 1) // args.row_align * args.row_align  # device shard row stride
    if args.row_stride:
        if args.row_stride < sl or args.row_stride % 16:
            ap.error(f"--row-stride must be >= shard_len ({sl}) and a multiple of 16")
        ss = args.row_stride
    dev = torch.device("cuda", local)

    # synthetic inputs, resident before timing; seeds are global payload indices
    seeds = sharding.rank_seeds(rank, B)
    d_pay = torch.empty((B, plen), dtype=torch.uint8, device=dev)
    for c0 in range(0, B, 256):
        d_pay[c0:c0 + 256] = synth.payloads_torch(seeds[c0:c0 + 256], plen, device=dev)
    d_pres = torch.from_numpy(synth.present_masks([10**6 + s for s in seeds], nv, cnt, n)).to(dev)
    d_sh = torch.empty((B, nv, ss), dtype=torch.uint8, device=dev)
    d_el = torch.empty((B, n), dtype=torch.int16, device=dev)
    d_out = torch.empty((B, sl * k), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    ev = []
    # --graph: the *_ws calls on one caller-owned workspace (stream-ordered)
    ws = (torch.empty(max(max(E.workspace_bytes(nv, plen, B)), 1), dtype=torch.uint8, device=dev)
          if args.graph else None)

    def step(record, st=None):
        st = st or stream
        if record:
            e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            e[0].record(st)
        if ws is None:
            E.encode_batch(nv, d_pay, plen, plen, B, d_sh, ss, st)
        else:
            E.encode_batch_ws(nv, d_pay, plen, plen, B, d_sh, ss, ws, st)
        if record:
            e[1].record(st)
        if ws is None:
            E.error_locator(nv, d_pres, B, d_el, st)
        else:
            E.error_locator_ws(nv, d_pres, B, d_el, ws, st)
        if record:
            e[2].record(st)
        if ws is None:
            E.reconstruct_batch(nv, d_sh, sl, ss, d_pres, d_el, B, d_out, sl * k, st)
        else:
            E.reconstruct_batch_ws(nv, d_sh, sl, ss, d_pres, d_el, B, d_out, sl * k, ws, stream=st)
        if record:
            e[3].record(st)
            ev.append(e)

    for _ in range(args.warmup):
        step(False)
    graph = None
    if args.graph:  # one step captured after the warm-up (kernel attributes, tables set)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step(False, torch.cuda.current_stream(dev))
        graph.replay()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if graph is None:
            step(True)
        else:
            graph.replay()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if graph is not None:  # per-kernel times from eager steps after the timed region
        for _ in range(3):
            step(True)
        torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = sharding.max_over_ranks(t1 - t0, dist, dev if backend == "nccl" else None)
    ranks_detail = sharding.rank_table(dict(device_info(local), rank=rank,
                                            step_ms=round((t1 - t0) / args.steps * 1e3, 3)), dist)

    # sanity: the last step's reconstruction equals the payloads (round trip)
    ok = bool(torch.equal(d_out[:, :plen], d_pay))

    ms = lambda a, b: np.mean([x[a].elapsed_time(x[b]) for x in ev])  # noqa: E731
    t_enc, t_loc, t_rec = ms(0, 1), ms(1, 2), ms(2, 3)
    enc_bytes = B * (plen + nv * sl)           # SURVEY.md §8d algorithmic bytes
    rec_bytes = B * (cnt + k) * sl + B * n * 2  # + error-locator multipliers read
    kern = {"encode": (t_enc, enc_bytes), "reconstruct": (t_rec, rec_bytes)}
    dom = max(kern, key=lambda x: kern[x][0])
    t_dom, b_dom = kern[dom]
    achieved = b_dom / (t_dom * 1e-3)

    traffic, traffic_src = pmc_traffic(dom, nv, plen, cnt, B)
    bw = device_bandwidth(dev)
    mul_enc, mul_rec = gf_mul_counts(nv, n, k, cnt)
    pieces, cols = -(-plen // (2 * k)), sl // 2
    total_bytes = world * B * plen * args.steps
    value = total_bytes / elapsed / 2**30
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s",
        # ranks share GPUs only in the gloo rehearsal mode (ECCR_BENCH_BACKEND)
        "n_gpus": world if backend == "nccl" else min(world, max(torch.cuda.device_count(), 1)),
        "ranks": world,
        "world_size": dist.get_world_size() if dist else 1,
        # per rank: its device and PCI bus id and its own step time (the value
        # uses the slowest, ms_per_step); distinct bus ids = distinct GPUs
        "ranks_detail": ranks_detail,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u16",
        "data": "synthetic: splitmix64 payloads (seed = payload index), per-payload random "
                f"{cnt}-of-{nv} present shards",
        "config": {"workload": f"{'config2: ' if (nv, plen, cnt) == (1024, 1_000_000, 342) else ''}{plen} B payloads, n_validators={nv}, batch={B}/GPU, "
                               f"encode + reconstruct from {cnt} random shards",
                   "n_validators": nv, "payload_bytes": plen, "batch_per_gpu": B,
                   "present_shards": cnt, "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved / 1e9, 2),
                     "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "bytes_per_launch": b_dom, "avg_launch_ms": round(t_dom, 4),
                     "issue": sq_issue(dom, nv),
                     "measured": dict(bw, frac_of_copy=round(achieved / (bw["copy_GBps"] * 1e9), 4))},
        # secondary figure: the REFERENCE algorithm's GF(2^16)
        # multiplies (additive_fft.hpp:99-141) per second of our kernel time.
        # Not a ceiling: the kernels run fewer multiplies than the reference
        # (restricted FFT, zero skews) and most in cheaper subfield / F9 forms,
        # so no single multiply rate bounds it; the bound is
        # SIMD instruction issue, reported under roofline.issue
        "gf_mul": {"encode_per_s": round(B * pieces * mul_enc / (t_enc * 1e-3), -9),
                   "reconstruct_per_s": round(B * cols * mul_rec / (t_rec * 1e-3), -9),
                   "per_piece_encode": mul_enc, "per_column_reconstruct": round(mul_rec, 1),
                   "counts": "reference algorithm (ec-cpp), not the multiplies executed"},
        "kernels_ms": {"encode": round(t_enc, 4), "error_locator": round(t_loc, 4),
                       "reconstruct": round(t_rec, 4)},
        "encode_GiBps": round(world * B * plen / (t_enc * 1e-3) / 2**30, 3),
        "reconstruct_GiBps": round(world * B * plen / ((t_loc + t_rec) * 1e-3) / 2**30, 3),
        "roundtrip_ok": ok,
    }
    if graph is not None:
        line["graph"] = "timed steps are hipGraph replays of one captured step; kernels_ms from eager steps"
    if args.sweep_sizes:
        headline = {"payload_bytes": plen, "batch_per_gpu": B, "ms_per_step": line["ms_per_step"],
                    "GiBps": line["value"], "kernels_ms": line["kernels_ms"],
                    "roofline": {"kernel": dom, "achieved_GBps": line["roofline"]["achieved"],
                                 "frac": line["roofline"]["frac"]},
                    "roundtrip_ok": ok, "note": "the headline measurement above"}
        line["sizes"] = size_sweep(args, nv, args.present, dev, stream, dist, world, rank, backend,
                                   headline)
        ok = ok and all(r["roundtrip_ok"] for r in line["sizes"])
    if not args.no_e2e:
        del d_sh, d_el  # the host-batch pipeline allocates its own device slots
        torch.cuda.empty_cache()
        line["e2e"], ok_e2e = e2e(args, nv, dev, dist, world, rank,
                                  dev if backend == "nccl" else torch.device("cpu"))
        ok = ok and ok_e2e
    if backend != "nccl":
        line["rehearsal"] = f"{world} ranks on {line['n_gpus']} GPU(s), gloo"
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # (contract: rank 0 at N = 1)
        line["cpu_baseline"] = cpu_baseline(nv, plen, cnt, args.cpu_seconds,
                                           args.cpu_threads or None)
    sg_failed = False
    sg_bad = False
    if dist and backend == "nccl" and not args.no_scatter:
        # the device-resident line above is the measurement; the scatter /
        # gather is reported beside it and can neither hang nor fail it
        def on_timeout():
            if rank == 0:
                line["scatter_gather"] = {"timeout_s": args.scatter_timeout}
                print(json.dumps(line), flush=True)
        try:
            line["scatter_gather"] = scatter_gather(dist, rank, world, dev, B, plen, d_pay, d_out,
                                                    elapsed / args.steps, args.scatter_timeout,
                                                    on_timeout)
            sg_bad = not line["scatter_gather"]["ok"]
        except Exception as exc:  # noqa: BLE001 (reported in the line, then exit 4)
            sg_failed = True
            line["scatter_gather"] = {"error": f"{type(exc).__name__}: {exc}"[:300]}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist and not sg_failed:
        dist.destroy_process_group()
    if sg_failed:
        sys.exit(EXIT_SG_ERROR)
    if not ok or sg_bad:
        sys.exit(EXIT_CHECK)


if __name__ == "__main__":
    main()
