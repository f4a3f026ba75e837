#!/bin/bash
# Full measurement of the default bench workload (B = 4096 x 1 MB, nv = 1024):
# bench line, rocprofv3 kernel stats, PMC HBM traffic (separate FETCH_SIZE /
# WRITE_SIZE passes), SQ counter passes.  Outputs under gpurun_out/meas/.
set -u
export TMPDIR=/tmp
O=gpurun_out/meas
mkdir -p $O
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  echo "=== $n ($(date +%T))"
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "=== $n rc=$rc"; tail -3 $O/$n.log
  [ $rc -eq 0 ] || exit $rc
}
run bench 600 python bench.py
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline
run fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc/FETCH_SIZE -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1
run write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc/WRITE_SIZE -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1
OUT=$O bash scripts/pmc_sq.sh
