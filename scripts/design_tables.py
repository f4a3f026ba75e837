#!/usr/bin/env python3
"""Rewrite DESIGN.md's measured tables (benchmark/ sizes, BASELINE configs,
n_validators sweep) from profiles/r03/{final,configs,nv_sweep} (the output of
scripts/gpu_final_r3.sh).  Round-2 values in the r02 -> r03 columns are kept
from the current tables."""
import glob
import json
import re

D = "DESIGN.md"


def last_json(path):
    return json.loads([l for l in open(path) if l.startswith("{")][-1])


def replace_rows(s, header_start, rows):
    i = s.index(header_start)
    j = s.index("|---", i)
    j = s.index("\n", j) + 1
    k = s.index("\n\n", j)
    return s[:j] + "\n".join(rows) + s[k:]


s = open(D).read()
b = last_json("profiles/r03/final/bench.json")
rows = []
for r in b["sizes"]:
    k, c = r["kernels_ms"], r["cpu_ec_cpp"]
    c16 = [v for kk, v in c.items() if kk != "GiBps_1thread"][0]
    rows.append(f"| {r['payload_bytes']:,} B | {r['batch_per_gpu']} | {r['ms_per_step']} | **{r['GiBps']}** | "
                f"{k['encode']*1e3:.0f} / {k['error_locator']*1e3:.0f} / {k['reconstruct']*1e3:.0f} | "
                f"{r['roofline']['kernel']} {r['roofline']['frac']*100:.2f}% | {c['GiBps_1thread']} / {c16} |")
s = replace_rows(s, "| payload | batch | ms per step | GiB/s | encode / locator", rows)

# configs: keep the r02 figure of each row
hdr = "| config | encode | reconstruct | step GiB/s (r02 → r03) |"
i = s.index(hdr)
old = s[i:s.index("\n\n", i)].splitlines()[2:]
r02 = [re.search(r"\| ([\d.]+) → [\d.]+ \|$", l).group(1) for l in old]
names = ["c3_10MB_thr", "c3_10MB_k", "c2_k", "c4_nv4096"]
rows = []
for l, nm, o in zip(old, names, r02):
    x = last_json(f"profiles/r03/configs/{nm}.json")
    label = l.split("|")[1].strip()
    k = x["kernels_ms"]
    rows.append(f"| {label} | {k['encode']:.2f} ms | {k['reconstruct']:.2f} ms | {o} → {x['value']:.1f} |")
s = replace_rows(s, hdr, rows)

hdr = "| nv | (n, k) | encode ms | encode GB/s (alg.) |"
i = s.index(hdr)
old = {int(l.split("|")[1]): re.search(r"\| ([\d.–]+) → [\d.]+ \|$", l).group(1)
       for l in s[i:s.index("\n\n", i)].splitlines()[2:]}
rows = []
for f in glob.glob("profiles/r03/nv_sweep/nv*.json"):
    d = last_json(f)
    c = d["config"]
    nv, P, B, cnt = c["n_validators"], c["payload_bytes"], c["batch_per_gpu"], c["present_shards"]
    n = 1 << (nv - 1).bit_length()
    thr = (nv - 1) // 3 + 1
    k = 1 << (thr.bit_length() - 1)
    sl = ((P + 2 * k - 1) // (2 * k)) * 2
    te, tr = d["kernels_ms"]["encode"], d["kernels_ms"]["reconstruct"]
    enc = B * (P + nv * sl) / (te * 1e-3) / 1e9
    rec = (B * (cnt + k) * sl + B * n * 2) / (tr * 1e-3) / 1e9
    rows.append((nv, f"| {nv} | ({n}, {k}) | {te:.2f} | {enc:,.0f} | {tr:.2f} | {rec:,.0f} | "
                     f"{old.get(nv, '–')} → {d['value']:.1f} |"))
s = replace_rows(s, hdr, [r for _, r in sorted(rows)])
open(D, "w").write(s)
print("tables rewritten")
