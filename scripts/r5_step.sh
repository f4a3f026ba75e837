#!/bin/bash
# Round-5 GPU step (edit per experiment): -m gpu suite (writes
# gpurun_out/reference_benchmark.txt), then the reference benchmark twice more.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for i in 1 2; do timeout -k 10 120 oracle/_ref/benchmark > gpurun_out/refbench_$i.txt 2>&1 || exit 1; grep -A2 "15 bytes\|300 bytes\|5000 bytes" gpurun_out/refbench_$i.txt | grep RUST; done
