#!/bin/bash
# Above-power-of-two shapes: bench lines at 512 x 1 MB
# for each nv in NVS, kernel split from rocprofv3 --stats of the same command.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/nv; mkdir -p $O
for nv in ${NVS:-2500 3069}; do
  timeout -k 10 300 python bench.py --nv $nv --batch ${B:-512} --steps 5 --warmup 2 --sweep none --no-cpu-baseline > $O/nv$nv.json 2> $O/nv$nv.err || { tail -5 $O/nv$nv.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/nv$nv.json').read().strip().splitlines()[-1]); print($nv, d['value'], d['kernels_ms'], d['roundtrip_ok'])"
  if [ -n "${PROF:-}" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$nv -o run -- python3 bench.py --nv $nv --batch ${B:-512} --steps 5 --warmup 2 --sweep none --no-cpu-baseline > $O/prof$nv.log 2>&1 || { tail -5 $O/prof$nv.log; exit 1; }
  fi
done
