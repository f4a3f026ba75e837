#!/bin/bash
# Config-4 family A/B (VARS libraries vs main) at n_validators 4096 / 2500 / 1500,
# after the GPU parity tests of those shapes.
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTS:-4096 or golden or oracle or graph or workspace or quarters}" > gpurun_out/t4096.log 2>&1; tail -3 gpurun_out/t4096.log
for nv in ${NVS:-4096 2500 1500}; do
  B=$([ $nv = 4096 ] && echo 2048 || echo 1024)
  VARS="${VARS:-var_head main}" B=$B ARGS="--nv $nv --sweep none" bash scripts/ab_run.sh || exit 1
done
