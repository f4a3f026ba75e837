#!/bin/bash
# Round-4 closing run, part 2: BASELINE configs (scripts/gpu_configs.sh), the
# config-5 stream and the host-resident (PCIe-inclusive) rates.
set -u
export TMPDIR=/tmp
O=${O:-gpurun_out/r4final}; mkdir -p $O
bash scripts/gpu_configs.sh > $O/configs.log 2>&1 || { tail -5 $O/configs.log; exit 1; }
echo configs done
timeout -k 10 600 python scripts/bench_stream.py > $O/stream.json 2> $O/stream.err || { tail -5 $O/stream.err; exit 1; }
timeout -k 10 600 python scripts/bench_e2e.py > $O/e2e.json 2> $O/e2e.err || { tail -5 $O/e2e.err; exit 1; }
echo all done
