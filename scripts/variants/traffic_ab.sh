#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the default workload for each library in VARS
# (main = the default build, else lib/<name>.so) -> gpurun_out/tab/<var>/
set -u
export TMPDIR=/tmp
L=erasure-coding-crust_amd/lib
for v in ${VARS:-main}; do
  if [ $v = main ]; then unset ECC_AMD_LIB; else export ECC_AMD_LIB=$PWD/$L/$v.so; fi
  O=gpurun_out/tab/$v; mkdir -p $O
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/$c -o run -- python3 bench.py --steps 2 --warmup 1 --sweep none --no-cpu-baseline ${ARGS:-} > $O/$c.log 2>&1 || { tail -3 $O/$c.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $O $O/pmc_traffic.json ${PMCARGS:-4096 1024 1000000 342} | head -20
done
