#!/bin/bash
# Round-6 in-process A/B of reconstruct_n4096's schedule knobs
# (scripts/variants/n4096_knobs.py) at the shapes above a power of two.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6n4096; mkdir -p $O
stop_on_fault() { if [ "$1" -ge 124 ]; then echo "FAULT status $1 in $2: stopping"; exit "$1"; fi; }
for cfg in "3069 main n4096_p4" "2500 main n4096_p4" "1500 main n4096_d2 n4096_np2" "2048 main n4096_d2 n4096_np2"; do
  set -- $cfg; nv=$1; shift
  timeout -k 10 300 python -u scripts/ab_inproc.py --nv $nv --batch 512 --rounds 6 "$@" > $O/ab_nv$nv.txt 2>&1
  rc=$?; echo "== nv $nv"; grep " enc " $O/ab_nv$nv.txt; stop_on_fault $rc ab; [ $rc -ne 0 ] && exit $rc
done
exit 0
