#!/bin/bash
# Round-6 in-process A/B at the headline shapes: main against the variants
# given as arguments (lib/<name>.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6ab2; mkdir -p $O
stop_on_fault() { if [ "$1" -ge 124 ]; then echo "FAULT status $1 in $2: stopping"; exit "$1"; fi; }
for nv in 1024 800; do
  timeout -k 10 300 python -u scripts/ab_inproc.py --nv $nv --batch 4096 --rounds 6 --steps 3 main "$@" > $O/ab_nv$nv.txt 2>&1
  rc=$?; echo "== nv $nv"; grep " enc " $O/ab_nv$nv.txt; stop_on_fault $rc ab; [ $rc -ne 0 ] && exit $rc
done
exit 0
