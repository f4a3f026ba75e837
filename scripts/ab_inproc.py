#!/usr/bin/env python3
"""In-process A/B of library variants: every variant (lib/<name>.so, `main` =
the default build) is loaded into THIS process (its own ctypes handle, its
own device tables) and the variants take turns on the same resident buffers,
round by round, so box-to-box and minute-to-minute clock drift falls on all
of them alike.  Per round and variant: `--steps` encode + locator +
reconstruct steps timed by HIP events; prints per variant the median and
the per-round kernel times, and whether its round trip held.

  ab_inproc.py [--batch B] [--nv N] [--rounds R] [--steps K] main var1 var2 ...
Variants whose name starts with `diag` may fail the round trip."""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "erasure-coding-crust_amd"))

import torch  # noqa: E402

import ecc_amd as E  # noqa: E402
import synth  # noqa: E402


def load(name):
    path = E.LIB_PATH if name == "main" else os.path.join(os.path.dirname(E.LIB_PATH), name + ".so")
    L = C.CDLL(path, mode=C.RTLD_LOCAL)
    ul, vp = C.c_ulong, C.c_void_p
    L.ECCR_AMD_init_device.restype = E.NPRSResult
    for f, args in (("ECCR_AMD_encode_batch", [ul, vp, ul, ul, ul, vp, ul, vp]),
                    ("ECCR_AMD_error_locator", [ul, vp, ul, vp, vp]),
                    ("ECCR_AMD_reconstruct_batch", [ul, vp, ul, ul, vp, vp, ul, vp, ul, vp])):
        getattr(L, f).restype = E.NPRSResult
        getattr(L, f).argtypes = args
    assert L.ECCR_AMD_init_device().tag == 0, name
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--payload", type=int, default=1_000_000)
    ap.add_argument("--nv", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="synchronise and idle this long between the locator and the reconstruct")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    libs = {v: load(v) for v in a.variants}
    nv, plen, B = a.nv, a.payload, a.batch
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    ss = (sl + 63) // 64 * 64
    dev = torch.device("cuda", 0)
    d_pay = torch.empty((B, plen), dtype=torch.uint8, device=dev)
    for c0 in range(0, B, 256):
        d_pay[c0:c0 + 256] = synth.payloads_torch(list(range(c0, min(B, c0 + 256))), plen, device=dev)
    d_pres = torch.from_numpy(synth.present_masks([10**6 + s for s in range(B)], nv, thr, n)).to(dev)
    d_sh = torch.empty((B, nv, ss), dtype=torch.uint8, device=dev)
    d_el = torch.empty((B, n), dtype=torch.int16, device=dev)
    d_out = torch.empty((B, sl * k), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731

    def step(L, ev):
        ev[0].record(st)
        assert L.ECCR_AMD_encode_batch(nv, P(d_pay), plen, plen, B, P(d_sh), ss, sp).tag == 0
        ev[1].record(st)
        assert L.ECCR_AMD_error_locator(nv, P(d_pres), B, P(d_el), sp).tag == 0
        if a.gap_ms > 0:
            torch.cuda.synchronize()
            time.sleep(a.gap_ms / 1000)
        ev[2].record(st)
        assert L.ECCR_AMD_reconstruct_batch(nv, P(d_sh), sl, ss, P(d_pres), P(d_el), B, P(d_out),
                                            sl * k, sp).tag == 0
        ev[3].record(st)

    res = {v: {"encode": [], "reconstruct": [], "ok": True} for v in a.variants}
    for v, L in libs.items():  # warm-up: every variant once
        step(L, [torch.cuda.Event(enable_timing=True) for _ in range(4)])
    torch.cuda.synchronize()
    for r in range(a.rounds):
        order = a.variants[r % len(a.variants):] + a.variants[:r % len(a.variants)]
        for v in order:
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(a.steps)]
            d_out.zero_()
            d_sh.zero_()  # a variant that does not write its shards fails the round trip
            for ev in evs:
                step(libs[v], ev)
            torch.cuda.synchronize()
            res[v]["encode"].append(statistics.mean(e[0].elapsed_time(e[1]) for e in evs))
            res[v]["reconstruct"].append(statistics.mean(e[2].elapsed_time(e[3]) for e in evs))
            res[v]["ok"] &= bool(torch.equal(d_out[:, :plen], d_pay))
    out = {}
    for v in a.variants:
        d = res[v]
        out[v] = {"encode_med": round(statistics.median(d["encode"]), 4),
                  "reconstruct_med": round(statistics.median(d["reconstruct"]), 4),
                  "encode": [round(x, 4) for x in d["encode"]],
                  "reconstruct": [round(x, 4) for x in d["reconstruct"]], "ok": d["ok"]}
        print(f"{v:14s} enc {out[v]['encode_med']:.4f} rec {out[v]['reconstruct_med']:.4f} ok={d['ok']} "
              f"enc/round {out[v]['encode']}", flush=True)
    print(json.dumps({"workload": {"batch": B, "payload": plen, "nv": nv, "rounds": a.rounds,
                                   "steps": a.steps}, "variants": out}))
    bad = [v for v in a.variants if not res[v]["ok"] and not v.startswith("diag")]
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
