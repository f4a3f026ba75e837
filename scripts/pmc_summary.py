#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (scripts/pmc_traffic.sh)
into per-launch HBM bytes for the codec kernels of the default bench workload.

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section, and our own
calibration scripts/micro/fetchcal.hip, profiles/r01/fetchcal.txt): the counters
are in KiB summed over the TCC instances.  FETCH_SIZE reports half the bytes of
16-B-per-lane and 8-B-per-lane coalesced reads (x2), and 1.043x the bytes of the
reconstruct kernel's 64-B-per-lane row reads (/1.043).  WRITE_SIZE is exact for
the 16-B-per-lane stores.
  encode:       fetch = raw x 2 (payload reads are 16 B per lane)
  reconstruct:  fetch = raw / 1.043 (reconstruct_n1024 and _n4096 alike: both
                read 64 B of a row per lane in the gather).  reconstruct_n1024x
                (round 5) reads 96 B of a row per lane: raw / 1.0017
                (profiles/r05/fetchcal.txt, k96), and re-reads its present data
                rows y < k in phase 5 (8 B per lane; L2 hits, see below: no
                term added).  Since r04
                reconstruct_n4096 also reads the received output rows y < k
                (16 B per lane, LDS-DMA) and the 80 KB per-payload output image
                per tile; those reads count at half weight and are added back as
                p16 = B x (c k / nv) x shard_len (the rows, expected count) +
                B x 80 KB (the image: one L2 miss per payload, its tiles
                sharing one XCD under xcd_span).  (Until r02 the kernel re-read the
                present data rows y < k in phase 5, 8 B per lane, and this
                added them back as p5 = B x (present rows < k) x shard_len at
                half weight.  Since r02 those rows are staged in LDS; the raw
                count did not move when the re-read went away (7.01 vs 7.00
                GB), i.e. the re-reads had been L2 hits, not HBM traffic.)
usage: pmc_summary.py SRC DST B NV PAYLOAD PRESENT
"""
import csv
import collections
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
B, NV, P, CNT = (int(x) for x in sys.argv[3:7])
N = 1 << (NV - 1).bit_length()
thr = (NV - 1) // 3 + 1
K = 1 << (thr.bit_length() - 1)
SL = ((P + 2 * K - 1) // (2 * K)) * 2
KERNELS = {"encode_k256": "encode", "encode_k256w": "encode", "reconstruct_n1024": "reconstruct",
           "reconstruct_n1024x": "reconstruct",
           "encode_k1024_fused": "encode", "reconstruct_n4096": "reconstruct",
           "encode_gen": "encode", "reconstruct_gen": "reconstruct",
           "encode_g": "encode", "reconstruct_g": "reconstruct", "error_locator_g": "error_locator"}


def per_launch(path, counter):
    val = collections.defaultdict(float)
    name = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        val[r["Dispatch_Id"]] += float(r["Counter_Value"])
        name[r["Dispatch_Id"]] = r["Kernel_Name"]
    out = collections.defaultdict(list)
    for d, v in val.items():
        for k, short in KERNELS.items():
            if k + "(" in name[d] or k + "<" in name[d]:
                # the 96-B-per-lane gather's FETCH_SIZE is exact to 0.2%:
                # rescaled here to the 64-B-per-lane units corrected below
                scale = 1.043 / 1.0017 if (counter == "FETCH_SIZE" and k == "reconstruct_n1024x") else 1.0
                out[short].append(v * 1024.0 * scale)
    return {k: sum(v) / len(v) for k, v in out.items()}


fetch = per_launch(f"{src}/FETCH_SIZE/run_counter_collection.csv", "FETCH_SIZE")
write = per_launch(f"{src}/WRITE_SIZE/run_counter_collection.csv", "WRITE_SIZE")
p5 = 0  # phase-5 re-reads: none since r02 (LDS staging)
# reconstruct_n4096 (n > 1024) 16-B-per-lane reads since r04 (see above); the
# image term assumes one L2 miss per payload (xcd_span)
p16 = 0
if N > 1024:
    p16 = B * (CNT * K / NV) * SL + B * 81920
res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, kernel-trace only",
       "workload": {"batch": B, "n_validators": NV, "payload_bytes": P, "present": CNT,
                    "shard_len": SL},
       "corrections": __doc__.split("usage:")[0].strip(), "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    f, w = fetch.get(k, 0.0), write.get(k, 0.0)
    if k == "reconstruct":
        fc = (f - p5 / 2 - p16 / 2) / 1.043 + p5 + p16
    else:
        fc = 2 * f
    res["kernels"][k] = {"fetch_raw_bytes": round(f), "fetch_bytes": round(fc),
                         "write_bytes": round(w), "hbm_bytes": round(fc + w),
                         "hbm_bytes_per_payload": round((fc + w) / B)}
json.dump(res, open(dst, "w"), indent=1)
print(json.dumps(res["kernels"], indent=1))
