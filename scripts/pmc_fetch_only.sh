set -u
export TMPDIR=/tmp
O=gpurun_out/pmc_contig
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/FETCH_SIZE -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/fetch.log 2>&1
