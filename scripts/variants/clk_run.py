#!/usr/bin/env python3
"""Shader clock under load of an enc_diag.py 'clk' variant (ECC_AMD_LIB): runs
the encode ITERS times at B payloads of 1 MB (nv = 1024) and prints the
summed s_memtime / s_memrealtime ratio of the workgroups' wave 0 (GHz) and
the mean kernel time.   usage: ECC_AMD_LIB=... clk_run.py [B] [ITERS]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "erasure-coding-crust_amd"))
import torch  # noqa: E402
import ecc_amd as E  # noqa: E402
import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nv, plen = 1024, 1_000_000
sl = E.shard_len(nv, plen)
ss = (sl + 63) // 64 * 64
d_pay = torch.empty((B, plen), dtype=torch.uint8, device="cuda")
for c0 in range(0, B, 256):
    d_pay[c0:c0 + 256] = synth.payloads_torch(list(range(c0, min(c0 + 256, B))), plen)
d_sh = torch.empty((B, nv, ss), dtype=torch.uint8, device="cuda")
L = E.lib()
L.ECCR_DIAG_stamps.restype = C.c_int
L.ECCR_DIAG_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
buf = (C.c_ulonglong * 16)()
E.encode_batch(nv, d_pay, plen, plen, B, d_sh, ss)
torch.cuda.synchronize()
L.ECCR_DIAG_stamps(buf, 16, 1)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    E.encode_batch(nv, d_pay, plen, plen, B, d_sh, ss)
e1.record()
torch.cuda.synchronize()
L.ECCR_DIAG_stamps(buf, 16, 0)
ghz = buf[0] / buf[1] * 0.1 if buf[1] else float("nan")
# one more launch alone: the spread of workgroup start / end times (realtime ticks, 10 ns)
buf2 = (C.c_ulonglong * 16)()
L.ECCR_DIAG_stamps(buf2, 16, 1)
E.encode_batch(nv, d_pay, plen, plen, B, d_sh, ss)
torch.cuda.synchronize()
L.ECCR_DIAG_stamps(buf2, 16, 0)
if buf2[6]:
    t0 = buf2[2]
    print(f"  one launch, {buf2[6]} workgroups: starts {0:.0f}..{(buf2[3] - t0) / 100:.1f} us, "
          f"ends {(buf2[4] - t0) / 100:.1f}..{(buf2[5] - t0) / 100:.1f} us")
print(f"{os.path.basename(os.environ.get('ECC_AMD_LIB', 'main'))} B={B} encode {e0.elapsed_time(e1) / iters:.3f} ms"
      f"  shader clock {ghz:.3f} GHz  (memtime {buf[0]}, realtime {buf[1]})")
