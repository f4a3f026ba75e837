set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "host_batch" > gpurun_out/pytest_host.log 2>&1 || { tail -30 gpurun_out/pytest_host.log; exit 1; }
tail -2 gpurun_out/pytest_host.log
timeout -k 10 600 python scripts/bench_e2e.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -30 gpurun_out/e2e.err; exit 1; }
cat gpurun_out/e2e.json
bash scripts/pmc_ab.sh || exit 1
