#!/usr/bin/env python3
"""Summarise scripts/pmc_sq.sh passes: per codec kernel, the SQ counters
summed over its dispatches, and derived fractions (SQ counters count
quad-cycles; WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY,
MI355X_MICROARCH.md).  usage: sq_summary.py SRC_DIR DST_JSON"""
import collections
import re
import csv
import glob
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in sorted(glob.glob(f"{src}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "ecamd::" not in name:
            continue
        short = re.search(r"(\w+(?:<[^>]*>)?)\(", name.replace("(anonymous namespace)::", "")).group(1)
        agg[short][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[short].add((path, r["Dispatch_Id"]))
out = {"source": "rocprofv3 --pmc SQ_* (3 passes, kernel-trace only), bench.py --batch 512 --steps 2 --warmup 1",
       "kernels": {}}
for k, c in agg.items():
    d = dict(c)
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        d["frac_wait_any"] = round(c.get("SQ_WAIT_ANY", 0) / wc, 4)
        d["frac_wait_inst_any"] = round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
        d["frac_active_inst_any"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
        d["frac_active_valu"] = round(c.get("SQ_ACTIVE_INST_VALU", 0) / wc, 4)
        d["frac_wait_inst_lds"] = round(c.get("SQ_WAIT_INST_LDS", 0) / wc, 4)
    if c.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
    if c.get("SQ_INSTS_VALU") and c.get("SQ_WAVES"):
        d["valu_insts_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1)
    out["kernels"][k] = d
json.dump(out, open(dst, "w"), indent=1)
for k, d in out["kernels"].items():
    print(k, {x: d[x] for x in d if x.startswith(("frac", "lds_", "valu_"))})
