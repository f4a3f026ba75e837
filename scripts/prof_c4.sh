#!/bin/bash
# Config 4 shape (n_validators 4096, 1 MB): bench line, rocprofv3 kernel stats
# and the SQ counter passes of its kernels.
set -u
export TMPDIR=/tmp
O=${O:-gpurun_out/c4}
mkdir -p $O
timeout -k 10 300 python bench.py --nv 4096 --batch ${B:-2048} --sweep none --no-cpu-baseline > $O/bench.json 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --nv 4096 --batch ${B:-2048} --sweep none --no-cpu-baseline --steps 3 > $O/prof.log 2>&1 || exit 1
OUT=$O BENCH_ARGS="--nv 4096 --batch 256 --steps 2 --warmup 1 --sweep none --no-cpu-baseline" bash scripts/pmc_sq.sh > $O/sq.log 2>&1 || exit 1
python3 scripts/sq_summary.py $O/pmc_sq $O/sq_counters.json
python3 scripts/sweep_summary.py $O/bench.json
cut -d, -f1-4 $O/prof/run_kernel_stats.csv | head -12
