#!/usr/bin/env python3
"""Run the default bench kernels a few times on a stamp variant (ECC_AMD_LIB)
and print each phase's share of the summed wave cycles.
usage: ECC_AMD_LIB=... stamp_run.py enc|dec NAMES [B]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "erasure-coding-crust_amd"))
import torch  # noqa: E402
import ecc_amd as E  # noqa: E402
import synth  # noqa: E402

kind, names = sys.argv[1], sys.argv[2].split(",")
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
nv, plen = int(os.environ.get("NV", "1024")), 1_000_000
n, k, thr = E.code_params(nv)
sl = E.shard_len(nv, plen)
ss = (sl + 63) // 64 * 64
d_pay = torch.empty((B, plen), dtype=torch.uint8, device="cuda")
for c0 in range(0, B, 256):
    d_pay[c0:c0 + 256] = synth.payloads_torch(list(range(c0, min(c0 + 256, B))), plen)
d_pr = torch.from_numpy(synth.present_masks([10**6 + s for s in range(B)], nv, thr, n)).cuda()
d_sh = torch.empty((B, nv, ss), dtype=torch.uint8, device="cuda")
d_el = torch.empty((B, n), dtype=torch.int16, device="cuda")
d_out = torch.empty((B, sl * k), dtype=torch.uint8, device="cuda")
L = E.lib()
L.ECCR_DIAG_stamps.restype = C.c_int
L.ECCR_DIAG_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()


def step():
    E.encode_batch(nv, d_pay, plen, plen, B, d_sh, ss)
    E.error_locator(nv, d_pr, B, d_el)
    E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, B, d_out, sl * k)


step()
torch.cuda.synchronize()
L.ECCR_DIAG_stamps(buf, 16, 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(3):
    step()
e1.record()
torch.cuda.synchronize()
L.ECCR_DIAG_stamps(buf, 16, 0)
tot = sum(buf[i] for i in range(len(names)))
print(kind, f"B={B}", f"step {e0.elapsed_time(e1) / 3:.3f} ms", "ok" if torch.equal(d_out[:, :plen], d_pay) else "MISMATCH")
for i, nm in enumerate(names):
    print(f"  {nm:10s} {100.0 * buf[i] / tot:5.1f}%")
