#!/bin/bash
# Kernel, copy and HIP-API trace of the host-resident benchmark (scripts/bench_e2e.py,
# one rep) for the pipeline's overlap: gpurun_out/e2etrace/*.csv
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
  -d gpurun_out/e2etrace -o run -- python3 scripts/bench_e2e.py --reps 1 > gpurun_out/e2etrace.log 2>&1 || { tail -5 gpurun_out/e2etrace.log; exit 1; }
ls gpurun_out/e2etrace
