#!/bin/bash
# parity tests, then the 1 MB x 512 bench at the given n_validators (NVS)
set -o pipefail
mkdir -p gpurun_out/dg
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/dg/pytest.log 2>&1 || { tail -40 gpurun_out/dg/pytest.log; exit 1; }
tail -3 gpurun_out/dg/pytest.log
for nv in ${NVS:-46 100 300 600 765}; do timeout -k 10 120 python bench.py --nv $nv --batch 512 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/dg/nv$nv.json 2> gpurun_out/dg/nv$nv.err || { tail -5 gpurun_out/dg/nv$nv.err; exit 1; }; python3 -c "import json; d=json.load(open('gpurun_out/dg/nv$nv.json')); print($nv, d['value'], d['kernels_ms'])"; done
