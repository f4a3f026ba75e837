#!/usr/bin/env python3
"""Shader clock under load of an enc_diag.py 'clk' / 'dclk' variant
(ECC_AMD_LIB): runs the probed kernel ITERS times at B payloads of 1 MB
(nv = 1024) and prints the summed s_memtime / s_memrealtime ratio of the
workgroups' wave 0 (GHz), the mean kernel time (HIP events), and for one more
launch the spread of the workgroups' start and end times.
usage: ECC_AMD_LIB=... clk_run.py [enc|dec|step] [B] [ITERS]  (step: encode + locator +
reconstruct per iteration, the reconstruct probed: a dclk variant)"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "erasure-coding-crust_amd"))
import torch  # noqa: E402
import ecc_amd as E  # noqa: E402
import synth  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "enc"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
nv, plen = int(os.environ.get("NV", "1024")), 1_000_000
n, k, thr = E.code_params(nv)
sl = E.shard_len(nv, plen)
ss = (sl + 63) // 64 * 64
d_pay = torch.empty((B, plen), dtype=torch.uint8, device="cuda")
for c0 in range(0, B, 256):
    d_pay[c0:c0 + 256] = synth.payloads_torch(list(range(c0, min(c0 + 256, B))), plen)
d_sh = torch.empty((B, nv, ss), dtype=torch.uint8, device="cuda")
d_pr = torch.from_numpy(synth.present_masks([10**6 + s for s in range(B)], nv, thr, n)).cuda()
d_el = torch.empty((B, n), dtype=torch.int16, device="cuda")
d_out = torch.empty((B, sl * k), dtype=torch.uint8, device="cuda")
L = E.lib()
L.ECCR_DIAG_stamps.restype = C.c_int
L.ECCR_DIAG_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()


def run():
    if kind in ("enc", "step"):
        E.encode_batch(nv, d_pay, plen, plen, B, d_sh, ss)
    if kind == "step":  # the bench step: the probed reconstruct right after an encode
        E.error_locator(nv, d_pr, B, d_el)
    if kind in ("dec", "step"):
        E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, B, d_out, sl * k)


E.encode_batch(nv, d_pay, plen, plen, B, d_sh, ss)
E.error_locator(nv, d_pr, B, d_el)
run()
torch.cuda.synchronize()
L.ECCR_DIAG_stamps(buf, 16, 1)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    run()
e1.record()
torch.cuda.synchronize()
L.ECCR_DIAG_stamps(buf, 16, 0)
ok = kind == "enc" or torch.equal(d_out[:, :plen], d_pay)
ghz = buf[0] / buf[1] * 0.1 if buf[1] else float("nan")
print(f"{os.path.basename(os.environ.get('ECC_AMD_LIB', 'main'))} {kind} nv={nv} B={B} {e0.elapsed_time(e1) / iters:.3f} ms"
      f"  shader clock {ghz:.3f} GHz  (memtime {buf[0]}, realtime {buf[1]}, wgs {buf[6]})"
      f"{'' if ok else '  MISMATCH'}")
# one more launch alone: the spread of workgroup start / end times (realtime ticks, 10 ns)
L.ECCR_DIAG_stamps(buf, 16, 1)
torch.cuda.synchronize()
e0.record()
run()
e1.record()
torch.cuda.synchronize()
L.ECCR_DIAG_stamps(buf, 16, 0)
if buf[6]:
    t0 = buf[2]
    print(f"  one launch ({e0.elapsed_time(e1):.3f} ms), {buf[6]} workgroups: starts 0..{(buf[3] - t0) / 100:.1f} us,"
          f" ends {(buf[4] - t0) / 100:.1f}..{(buf[5] - t0) / 100:.1f} us, mean life {buf[1] / buf[6] / 100:.1f} us")
