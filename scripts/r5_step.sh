#!/bin/bash
# Round-5 GPU step (edit per experiment): -m gpu suite, A/B.
set -o pipefail
export TMPDIR=/tmp
VARS="main prev" REPS=2 B=2048 ARGS="--nv 4096" bash scripts/r5_ab.sh || exit 1
NOTEST=1 VARS="main prev" REPS=2 B=512 ARGS="--nv 1500" bash scripts/ab_r4.sh
