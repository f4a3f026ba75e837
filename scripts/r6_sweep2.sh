#!/bin/bash
# Round-6 closing sweep on the final code: the BASELINE configurations
# (scripts/gpu_configs.sh) and the n_validators sweep (scripts/nvsweep_full.sh),
# without the test suite (run by the closing run of the same code).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6sweep2; mkdir -p $O
bash scripts/gpu_configs.sh > $O/configs.log 2>&1 || { tail -5 $O/configs.log; exit 1; }
bash scripts/nvsweep_full.sh > $O/nvsweep.log 2>&1 || { tail -5 $O/nvsweep.log; exit 1; }
for f in gpurun_out/configs/*.json gpurun_out/nv_sweep/nv*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['value'], d['kernels_ms'])"; done
