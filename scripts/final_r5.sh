#!/bin/bash
# Round-5 closing measurements on the current tree (stops at the first failure).
# PART=a: the -m gpu suite, the driver's bench command, rocprofv3 stats of the
#         same workload, smoke();
# PART=b: BASELINE configs (scripts/gpu_configs.sh), the nv sweep at 512 x 1 MB,
#         the reference benchmark binary and the per-call probes.
set -u
export TMPDIR=/tmp
O=${O:-gpurun_out/r5final}; mkdir -p $O/nv_sweep
step() { echo "== $1 ($(date +%T))"; }
if [ "${PART:-a}" = a ]; then
  step pytest
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  step "driver bench"
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
    || { tail -5 $O/bench_driver.err; exit 1; }
  step rocprof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --sweep none --no-cpu-baseline > $O/prof.log 2>&1 \
    || { tail -5 $O/prof.log; exit 1; }
  step smoke
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
    || { tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
else
  step configs
  bash scripts/gpu_configs.sh > $O/configs.log 2>&1 || { tail -5 $O/configs.log; exit 1; }
  mkdir -p $O/configs && cp gpurun_out/configs/*.json $O/configs/
  step "nv sweep"
  for nv in 600 765 1024 1025 1500 2500 3069 4096; do
    timeout -k 10 300 python3 bench.py --nv $nv --batch 512 --steps 5 --warmup 2 --sweep none --no-cpu-baseline \
      > $O/nv_sweep/nv$nv.json 2> $O/nv_sweep/nv$nv.err || { tail -5 $O/nv_sweep/nv$nv.err; exit 1; }
  done
  step "reference benchmark"
  timeout -k 10 200 oracle/_ref/benchmark > $O/reference_benchmark.txt 2>&1 || { tail -5 $O/reference_benchmark.txt; exit 1; }
  timeout -k 10 120 scripts/micro/capi_bench > $O/capi_bench.jsonl 2>&1 || exit 1
  timeout -k 10 60 scripts/micro/bin/mp_calls > $O/mp_calls.txt 2>&1 || exit 1
fi
step done
