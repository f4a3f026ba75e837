#!/bin/bash
# Round-5 GPU step (edit per experiment): -m gpu suite, A/B, PMC traffic.
set -o pipefail
export TMPDIR=/tmp
VARS="main base" REPS=2 B=2048 ARGS="--nv 4096" bash scripts/r5_ab.sh || exit 1
OUT=gpurun_out/c4 BENCH_ARGS="--nv 4096 --batch 2048 --steps 2 --warmup 1 --no-cpu-baseline --sweep none" bash scripts/pmc_traffic.sh || exit 1
python3 scripts/pmc_summary.py gpurun_out/c4/pmc_traffic gpurun_out/c4/pmc_traffic.json 2048 4096 1000000 1366 && cat gpurun_out/c4/pmc_traffic.json | head -40
