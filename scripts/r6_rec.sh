#!/bin/bash
# Round-6 GPU step for the reconstruct_n1024x relayout: the full -m gpu suite,
# then an in-process A/B against the previous kernel (lib/n1024x_old.so).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6rec}; mkdir -p $O
stop_on_fault() { if [ "$1" -ge 124 ]; then echo "FAULT status $1 in $2: stopping"; exit "$1"; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest_gpu.log | head -20
stop_on_fault $rc pytest; [ $rc -ne 0 ] && exit $rc
for nv in 1024 800; do
  timeout -k 10 300 python -u scripts/ab_inproc.py --nv $nv --batch 4096 --rounds 6 --steps 3 main n1024x_old > $O/ab_nv$nv.txt 2>&1
  rc=$?; echo "== nv $nv"; grep " enc " $O/ab_nv$nv.txt; stop_on_fault $rc ab; [ $rc -ne 0 ] && exit $rc
done
exit 0
