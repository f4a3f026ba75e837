#!/bin/bash
# A/B over n_validators shapes: lib/$VARS (default var_base vs main), 512 x 1 MB
set -o pipefail
for nv in ${NVS:-4096 2500 2048 1500 600 300 100}; do
  echo "nv=$nv"
  VARS="${VARS:-var_base main}" B=512 ARGS="--nv $nv" bash scripts/ab_run.sh || exit 1
done
