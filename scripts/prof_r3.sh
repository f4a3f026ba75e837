set -u
export TMPDIR=/tmp
export OUT=gpurun_out/r3prof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/headline -o run -- python3 bench.py --no-cpu-baseline --sweep none > $OUT/headline.log 2>&1 &&
BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --sweep none" bash scripts/pmc_traffic.sh &&
BENCH_ARGS="--batch 512 --steps 2 --warmup 1 --no-cpu-baseline --sweep none" bash scripts/pmc_sq.sh
