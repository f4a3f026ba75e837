timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "4096 or golden or oracle or graph or workspace or quarters" > gpurun_out/t4096.log 2>&1; tail -3 gpurun_out/t4096.log
VARS="var_q0 main" B=2048 ARGS="--nv 4096 --sweep none" bash scripts/ab_run.sh &&
VARS="var_q0 main" B=1024 ARGS="--nv 2500 --sweep none" bash scripts/ab_run.sh &&
VARS="var_q0 main" B=1024 ARGS="--nv 1500 --sweep none" bash scripts/ab_run.sh
