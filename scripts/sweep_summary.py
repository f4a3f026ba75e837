#!/usr/bin/env python3
"""Print the headline and the benchmark/ size sweep of a bench.py JSON line."""
import json
import sys

d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value", d["value"], d["kernels_ms"], "roundtrip_ok", d["roundtrip_ok"])
for r in d.get("sizes", []):
    print(r["payload_bytes"], r["batch_per_gpu"], r["ms_per_step"], r["GiBps"], r["kernels_ms"],
          r["roofline"]["frac"], r.get("cpu_ec_cpp"))
