#!/bin/bash
# Round-6 measurement after the new encodes (encode_k512w, encode_kw): the
# full -m gpu suite, then the BASELINE configurations (scripts/gpu_configs.sh)
# and the n_validators sweep (scripts/nvsweep_full.sh); results copied to
# profiles/r06/final/{configs,nv_sweep}.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6sweep; mkdir -p $O
stop_on_fault() { if [ "$1" -ge 124 ]; then echo "FAULT status $1 in $2: stopping"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && grep -E "^(FAILED|ERROR)|Error" $O/pytest_gpu.log | head -20
stop_on_fault $rc pytest; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_configs.sh > $O/configs.log 2>&1; rc=$?; stop_on_fault $rc configs; [ $rc -ne 0 ] && { tail -5 $O/configs.log; exit $rc; }
bash scripts/nvsweep_full.sh > $O/nvsweep.log 2>&1; rc=$?; stop_on_fault $rc nvsweep; [ $rc -ne 0 ] && { tail -5 $O/nvsweep.log; exit $rc; }
for f in gpurun_out/configs/*.json gpurun_out/nv_sweep/nv*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['value'], d['kernels_ms'])"; done
exit 0
