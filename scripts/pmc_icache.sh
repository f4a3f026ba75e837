#!/bin/bash
# Instruction-cache counters of the bench kernels for library variants VARS
# (rocprofv3 --pmc, kernel-trace only, small batch, one pass per variant).
set -u
export TMPDIR=/tmp
O=${OUT:-gpurun_out}/pmc_icache
mkdir -p $O
L=erasure-coding-crust_amd/lib
for v in ${VARS:-main}; do
  if [ $v = main ]; then unset ECC_AMD_LIB; else export ECC_AMD_LIB=$PWD/$L/$v.so; fi
  timeout -s KILL 240 rocprofv3 --pmc ${CTRS:-SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES} --kernel-trace --output-format csv -d $O/$v -o run -- python3 bench.py --batch 512 --steps 2 --warmup 1 --no-cpu-baseline --sweep none > $O/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  python3 - "$O/$v/run_counter_collection.csv" <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "encode_k256" in n or "reconstruct_n1024" in n:
        agg[n.split("(")[0][-40:]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items(): print(k, dict(c))
PY
done
