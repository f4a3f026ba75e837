#!/bin/bash
# One GPU session: tests -> smoke -> bench -> rocprof.  Stops at the first
# fault/abort/timeout (exit codes other than 0/1 from a test run).
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -5 "$OUT/$name.log"
  return $rc
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for s in "$@"; do
  case $s in
    test) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?; ok $rc || exit $rc ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; ok $rc || exit $rc ;;
    bench_small) step bench_small 600 python bench.py --batch 512 --steps 3 --warmup 1 --cpu-seconds 3; rc=$?; ok $rc || exit $rc ;;
    bench) step bench 900 python bench.py; rc=$?; ok $rc || exit $rc ;;
    stream) step stream 600 python scripts/bench_stream.py; rc=$?; ok $rc || exit $rc ;;
    e2e) step e2e 600 python scripts/bench_e2e.py; rc=$?; ok $rc || exit $rc ;;
    # profiles of the default bench workload (same kernels/sizes as `python bench.py`)
    prof) step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline; rc=$?; ok $rc || exit $rc ;;
    pmc_fetch) step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1; rc=$?; ok $rc || exit $rc ;;
    pmc_write) step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1; rc=$?; ok $rc || exit $rc ;;
  esac
done
