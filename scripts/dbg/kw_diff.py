#!/usr/bin/env python3
"""Debug helper: encode one batch through the C ABI and report where the
shards differ from the reference encoder (rows, piece ranges)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "erasure-coding-crust_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import ecc_amd as E  # noqa: E402
import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main(nv, plen, batch, pad):
    n, k, _ = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    ss = (sl + pad - 1) // pad * pad
    pays = [synth.payload(nv * 5 + b, plen) for b in range(batch)]
    d_pay = torch.from_numpy(np.stack(pays)).cuda()
    d_sh = torch.full((batch, nv, ss), 0x5C, dtype=torch.uint8, device="cuda")
    E.encode_batch(nv, d_pay, plen, plen, batch, d_sh, ss)
    torch.cuda.synchronize()
    got = d_sh.cpu().numpy()
    chk = O.Checker.default()
    for b in range(batch):
        want = chk.encode(nv, pays[b].tobytes())
        bad_rows = []
        for i in range(nv):
            g = got[b, i, :sl]
            w = np.frombuffer(want[i], dtype=np.uint8)
            if not np.array_equal(g, w):
                d = np.nonzero(g != w)[0]
                bad_rows.append((i, int(d[0]) // 2, int(d[-1]) // 2, len(d)))
        print(f"payload {b}: {len(bad_rows)} bad rows of {nv}")
        for r in bad_rows[:12]:
            print("  row", r[0], "pieces", r[1], "..", r[2], "bytes", r[3])
        if bad_rows:
            rows = [r[0] for r in bad_rows]
            print("  row range", min(rows), max(rows), "pieces", min(r[1] for r in bad_rows), max(r[2] for r in bad_rows))


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:5]])
