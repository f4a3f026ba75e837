#!/bin/bash
# LDS bank-conflict counters of the default bench workload (small batch) for
# alternative library builds (lib/var_*.so) and the tree's, one box.
set -u
export TMPDIR=/tmp
O=gpurun_out/pmc_ab; mkdir -p $O
for v in ${VARS:-main var_diag}; do
  if [ $v = main ]; then unset ECC_AMD_LIB; else export ECC_AMD_LIB=$PWD/erasure-coding-crust_amd/lib/$v.so; fi
  timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv \
    -d $O/$v -o run -- python3 bench.py --batch 512 --steps 2 --warmup 1 --no-cpu-baseline --sweep none ${ARGS:-} > $O/$v.log 2>&1; [ -f $O/$v/run_counter_collection.csv ] || { tail -3 $O/$v.log; exit 1; }
  python3 - "$O/$v" "$v" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for p in glob.glob(sys.argv[1] + "/run_counter_collection.csv"):
    for r in csv.DictReader(open(p)):
        if "ecamd" in r["Kernel_Name"]:
            agg[r["Kernel_Name"].split("(")[0][-32:]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    if c.get("SQ_LDS_IDX_ACTIVE"):
        print(sys.argv[2], k, "bank_conflict/idx_active = %.4f" % (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]))
PY
done
