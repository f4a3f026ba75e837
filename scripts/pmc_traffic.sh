#!/bin/bash
# HBM traffic of the bench kernels: separate rocprofv3 --pmc passes for
# FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md: they cannot share a pass),
# kernel-trace only, default bench workload; summarised by
# scripts/pmc_summary.py into profiles/<round>/pmc_traffic.json.
set -u
export TMPDIR=/tmp
O=${OUT:-gpurun_out}/pmc_traffic
mkdir -p $O
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/$c -o run -- python3 bench.py $ARGS > $O/$c.log 2>&1 || exit 1
done
