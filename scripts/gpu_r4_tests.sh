#!/bin/bash
# Round 4: the -m gpu suite on the current tree (stops at the first failure).
set -u
export TMPDIR=/tmp
O=gpurun_out/r4tests; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
grep -E "PASSED|FAILED|ERROR" $O/pytest_gpu.log | grep -E "4GiB|concurrent_default|release_stream|gpus_flag" || true
exit $rc
