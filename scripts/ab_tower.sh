#!/bin/bash
# GPU parity suite, then A/B of library variants (VARS) at n_validators 1024
# (B = 2048) and the NVS shapes (B = 1024).
set -o pipefail
bash scripts/gpu_round.sh test || exit 1
VARS="${VARS:-t1 main}" B=2048 ARGS="--sweep none" bash scripts/ab_run.sh || exit 1
for nv in ${NVS:-1500}; do
  VARS="${VARS:-t1 main}" B=1024 ARGS="--nv $nv --sweep none" bash scripts/ab_run.sh || exit 1
done
