set -o pipefail
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for nv in 600 2500 3069; do echo "nv=$nv"; NOTEST=1 VARS="main gstat" B=512 ARGS="--nv $nv" REPS=2 bash scripts/r5_ab.sh || exit 1; done
