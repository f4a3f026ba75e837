#!/bin/bash
# Eager steps vs hipGraph replays (bench.py --graph) over payload sizes, nv = 1024:
# gpurun_out/graph_ab/*.json
set -o pipefail
O=gpurun_out/graph_ab; mkdir -p $O
for cfg in "15 4096" "300 4096" "5000 4096" "100000 1024" "1000000 4096"; do
  set -- $cfg
  for mode in eager graph; do
    extra=""; [ $mode = graph ] && extra="--graph"
    timeout -k 10 200 python bench.py --payload $1 --batch $2 --steps 20 --warmup 3 --no-cpu-baseline $extra > $O/p$1_$mode.json 2> $O/p$1_$mode.err || { tail -5 $O/p$1_$mode.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/p$1_$mode.json')); print('$1 B x $2', '$mode', d['ms_per_step'], 'ms/step', d['value'], 'GiB/s', d['kernels_ms'], d['roundtrip_ok'])"
  done
done
