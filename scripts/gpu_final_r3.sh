#!/bin/bash
# End-of-round GPU session: full -m gpu suite, default bench (headline + size
# sweep + CPU baseline), BASELINE configs, n_validators sweep, config-5 stream
# and host-resident end-to-end rates.  Stops at the first failing step.
set -u
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
echo bench done
bash scripts/gpu_configs.sh > $O/configs.log 2>&1 || { tail -5 $O/configs.log; exit 1; }
echo configs done
bash scripts/nvsweep_full.sh > $O/nvsweep.log 2>&1 || { tail -5 $O/nvsweep.log; exit 1; }
echo nvsweep done
timeout -k 10 600 python scripts/bench_stream.py > $O/stream.json 2> $O/stream.err || { tail -5 $O/stream.err; exit 1; }
timeout -k 10 600 python scripts/bench_e2e.py > $O/e2e.json 2> $O/e2e.err || { tail -5 $O/e2e.err; exit 1; }
echo all done
