#!/bin/bash
# Round-5 GPU step: the full -m gpu suite on the default library (unless
# NOTEST=1), then scripts/ab_r4.sh over VARS.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
bash scripts/ab_r4.sh
