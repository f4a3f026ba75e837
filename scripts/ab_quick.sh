#!/bin/bash
# quick GPU check of a kernel change: parity tests on the reconstruct shapes,
# then an A/B of the default workload against lib/var_base.so
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "${TESTK:-batch or random_vs_oracle}" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
VARS="${VARS:-var_base main}" B=${B:-2048} bash scripts/ab_run.sh
