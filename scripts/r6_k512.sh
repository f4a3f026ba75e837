#!/bin/bash
# Round-6 GPU step after encode_k512w: the full -m gpu suite, an in-process
# A/B of the max-memory-clause scheduler build (lib/k512sched.so) at nv 3069 /
# 2048, then the n_validators sweep of the k = 512 shapes (bench.py, 512 x 1 MB).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6k512; mkdir -p $O
stop_on_fault() { if [ "$1" -ge 124 ]; then echo "FAULT status $1 in $2: stopping"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && grep -E "^(FAILED|ERROR)|Error" $O/pytest_gpu.log | head -20
stop_on_fault $rc pytest; [ $rc -ne 0 ] && exit $rc
for cfg in "3069 512" "2048 512"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/ab_inproc.py --nv $1 --batch $2 --rounds 4 main k512sched > $O/ab_sched_nv$1.txt 2>&1
  rc=$?; echo "== nv $1"; grep " enc " $O/ab_sched_nv$1.txt; stop_on_fault $rc ab
done
NVS="${NVS:-1534 1600 2048 2049 2500 3000 3069}" bash scripts/nvsweep_full.sh > $O/nvsweep.log 2>&1
rc=$?; stop_on_fault $rc nvsweep
for f in gpurun_out/nv_sweep/nv*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['value'], d['kernels_ms'])"; done
exit 0
