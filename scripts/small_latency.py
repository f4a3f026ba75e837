#!/usr/bin/env python3
"""Kernel times (HIP events) of the encode / locator / reconstruct step at
small payload sizes for batch sizes 1 .. 4096 (n_validators = 1024, tight
payload pitch, shard rows tight below 64 B): latency vs throughput of the
packed kernels."""
import sys, time
sys.path[:0] = ["erasure-coding-crust_amd"]
import numpy as np, torch
import ecc_amd as E, synth
E.lib().ECCR_AMD_init_device()
nv = 1024
n, k, thr = E.code_params(nv)
for plen in (15, 5000):
  for B in (1, 8, 64, 512, 4096):
    sl = E.shard_len(nv, plen); ss = sl if sl < 64 else (sl + 63) // 64 * 64
    d_pay = synth.payloads_torch(list(range(B)), plen, device="cuda").contiguous()
    d_pr = torch.from_numpy(synth.present_masks([10**6 + s for s in range(B)], nv, thr, n)).cuda()
    d_sh = torch.empty((B, nv, ss), dtype=torch.uint8, device="cuda")
    d_el = torch.empty((B, n), dtype=torch.int16, device="cuda")
    d_out = torch.empty((B, sl * k), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    res = []
    for rep in range(6):
      e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
      e[0].record(st); E.encode_batch(nv, d_pay, plen, plen, B, d_sh, ss, st); e[1].record(st)
      E.error_locator(nv, d_pr, B, d_el, st); e[2].record(st)
      E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, B, d_out, sl * k, st); e[3].record(st)
      torch.cuda.synchronize()
      if rep >= 2: res.append([e[i].elapsed_time(e[i + 1]) * 1e3 for i in range(3)])
    r = np.median(np.array(res), axis=0)
    print(f"plen {plen} B {B:5d}  encode {r[0]:7.1f} us  locator {r[1]:6.1f} us  reconstruct {r[2]:7.1f} us  ok {bool(torch.equal(d_out[:, :plen], d_pay))}")
