#!/bin/bash
# BASELINE.json configs other than the headline: 10 MB payloads (config 3),
# n_validators sweep incl. 4096 (config 4 per GPU), exactly-k erasures.
set -u
O=gpurun_out/configs; mkdir -p $O
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 python bench.py --sweep none "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }; cat $O/$name.json; }
run c3_10MB_thr --payload 10000000 --batch 400 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
run c3_10MB_k --payload 10000000 --batch 400 --present k --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
run c2_k --present k --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
run c4_nv4096 --nv 4096 --batch 8192 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
run nv2048 --nv 2048 --batch 512 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
run nv512 --nv 512 --batch 512 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
run nv100 --nv 100 --batch 512 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e
