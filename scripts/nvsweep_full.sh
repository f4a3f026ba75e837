#!/bin/bash
# n_validators sweep behind DESIGN.md §6 (1 MB x 512, threshold-many random
# present shards); results into gpurun_out/nv_sweep/, copied to profiles/<round>/nv_sweep/.
set -u
O=gpurun_out/nv_sweep; mkdir -p $O
for nv in ${NVS:-46 64 65 100 129 200 300 384 600 765 1024 1025 1500 2048 2500 3069 3070 4096}; do
  timeout -k 10 200 python bench.py --nv $nv --batch 512 --steps 5 --warmup 2 --no-cpu-baseline --sweep none --no-e2e > $O/nv$nv.json 2> $O/nv$nv.err || { tail -5 $O/nv$nv.err; exit 1; }
  echo "nv=$nv done"
done
