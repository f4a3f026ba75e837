#!/bin/bash
# parity subset on the default library, then an A/B of VARS at B and ARGS
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-batch or golden}" > gpurun_out/parity_subset.log 2>&1 || { tail -20 gpurun_out/parity_subset.log; exit 1; }
tail -2 gpurun_out/parity_subset.log
bash scripts/ab_run.sh
