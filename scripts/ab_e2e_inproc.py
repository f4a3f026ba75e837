#!/usr/bin/env python3
"""In-process A/B of the host-batch pipeline (ECCR_AMD_*_host_batch) across
library variants (lib/<name>.so, `main` = the default build), as
scripts/ab_inproc.py does for the device kernels: the variants take turns on
the same pinned buffers, round by round.  Config-2 shape by default (256 x
1 MB, n_validators 1024, threshold-many compacted present shards).

  ab_e2e_inproc.py [--batch B] [--rounds R] main var1 ..."""
import argparse
import ctypes as C
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "erasure-coding-crust_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import ecc_amd as E  # noqa: E402


def load(name):
    path = E.LIB_PATH if name == "main" else os.path.join(os.path.dirname(E.LIB_PATH), name + ".so")
    L = C.CDLL(path, mode=C.RTLD_LOCAL)
    ul, vp = C.c_ulong, C.c_void_p
    L.ECCR_AMD_init_device.restype = E.NPRSResult
    L.ECCR_AMD_encode_host_batch.restype = E.NPRSResult
    L.ECCR_AMD_encode_host_batch.argtypes = [ul, vp, ul, ul, ul, vp, ul, ul]
    L.ECCR_AMD_reconstruct_host_batch.restype = E.NPRSResult
    L.ECCR_AMD_reconstruct_host_batch.argtypes = [ul, vp, ul, ul, vp, ul, ul, vp, ul, ul]
    assert L.ECCR_AMD_init_device().tag == 0, name
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--payload", type=int, default=1_000_000)
    ap.add_argument("--nv", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    assert E.lib().ECCR_AMD_init_device().tag == 0
    libs = {v: load(v) for v in a.variants}
    nv = a.nv
    n, k, thr = E.code_params(nv)
    dev = torch.device("cuda", 0)
    c = bench._host_class(nv, a.payload, list(range(a.batch)), dev)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    res = {v: {"enc": [], "rec": [], "ok": True} for v in a.variants}

    def enc(L):
        assert L.ECCR_AMD_encode_host_batch(nv, P(c["pay"]), c["plen"], c["plen"], c["B"], P(c["sh"]),
                                            c["sl"], 0).tag == 0

    def rec(L):
        assert L.ECCR_AMD_reconstruct_host_batch(nv, P(c["comp"]), c["sl"], c["sl"], P(c["idx"]), thr,
                                                 c["B"], P(c["out"]), c["sl"] * k, 0).tag == 0

    for L in libs.values():  # warm: every variant's pipeline slots
        enc(L)
        rec(L)
    ref_sh = c["sh"].clone()  # the shards every variant must write (zeroed before each encode)
    gib = c["B"] * a.payload / 2**30
    for r in range(a.rounds):
        order = a.variants[r % len(a.variants):] + a.variants[:r % len(a.variants)]
        for v in order:
            L = libs[v]
            c["sh"].zero_()
            t0 = time.perf_counter()
            enc(L)
            t1 = time.perf_counter()
            c["out"].zero_()
            t2 = time.perf_counter()
            rec(L)
            t3 = time.perf_counter()
            res[v]["enc"].append(gib / (t1 - t0))
            res[v]["rec"].append(gib / (t3 - t2))
            res[v]["ok"] &= bool(torch.equal(c["out"][:, :a.payload], c["pay"]))
            res[v]["ok"] &= bool(torch.equal(c["sh"], ref_sh))
    for v in a.variants:
        d = res[v]
        print(f"{v:10s} encode {statistics.median(d['enc']):.3f} reconstruct {statistics.median(d['rec']):.3f} "
              f"GiB/s ok={d['ok']}  enc {[round(x, 2) for x in d['enc']]}  rec {[round(x, 2) for x in d['rec']]}",
              flush=True)
    sys.exit(0 if all(res[v]["ok"] for v in a.variants) else 1)


if __name__ == "__main__":
    main()
