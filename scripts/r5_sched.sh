#!/bin/bash
# Round 5: machine-scheduler strategy A/B (libraries from scripts/build_var.sh
# with -mllvm scheduler flags).  Headline (B = 4096, nv 1024) over VARS, then
# config 4 per GPU at B = 2048 and nv 2500 / 600 at B = 512 over VARS2.
set -o pipefail
export TMPDIR=/tmp
NOTEST=1 VARS="${VARS:-main mcl}" REPS=${REPS:-3} B=4096 bash scripts/r5_ab.sh || exit 1
for a in "--nv 4096:2048" "--nv 2500:512" "--nv 600:512"; do
  echo "== ${a%%:*}"
  NOTEST=1 VARS="${VARS2:-main mcl}" REPS=2 B=${a##*:} ARGS="${a%%:*}" bash scripts/r5_ab.sh || exit 1
done
