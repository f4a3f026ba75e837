#!/bin/bash
# GPU parity suite, then A/B of VARS at n_validators 4096 (B = 2048) and the
# NVS shapes (B = 1024), default workload flags otherwise.
set -o pipefail
bash scripts/gpu_round.sh test || exit 1
for nv in ${NVS:-4096 2500 1500}; do
  B=$([ $nv = 4096 ] && echo 2048 || echo 1024)
  VARS="${VARS:-t2 main}" B=$B ARGS="--nv $nv --sweep none" bash scripts/ab_run.sh || exit 1
done
