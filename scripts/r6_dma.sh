#!/bin/bash
# Round-6 GPU step for the LDS-DMA change: the -m gpu suite on the default
# library (NOTEST=1 skips it), then in-process A/Bs of lib/old.so (the build
# before the change) against it at the shapes whose kernels use LDS-DMA
# (nv 4096: encode_k1024 / reconstruct_n4096; nv 2048, 2500, 3069: encode_gen,
# reconstruct_n4096<2048> / <4096>; nv 1024: control, no DMA).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6dma; mkdir -p $O
stop_on_fault() { if [ "$1" -ge 124 ]; then echo "FAULT status $1 in $2: stopping"; exit "$1"; fi; }
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && grep -E "^(FAILED|ERROR)|Error" $O/pytest_gpu.log | head -20
  stop_on_fault $rc pytest
  [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${CFGS:-"4096 2048" "3069 512" "2500 512" "2048 512" "1024 1024"}; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/ab_inproc.py --nv $1 --batch $2 --rounds ${ROUNDS:-4} ${VARS:-old main} > $O/ab_nv$1.txt 2>&1
  rc=$?; echo "== nv $1 B $2 (rc $rc)"; tail -${TAILN:-4} $O/ab_nv$1.txt; stop_on_fault $rc ab_nv$1
done
exit 0
