#!/bin/bash
# Round-4 closing measurements on the current tree (stops at the first failure):
#  1. the driver's bench command (CPU baseline and size sweep included)
#  2. the above-power-of-two sweep, 512 x 1 MB per shape
#  3. smoke()
set -u
export TMPDIR=/tmp
O=${O:-gpurun_out/r4final}; mkdir -p $O/nv_sweep
echo "== driver bench ($(date +%T))"
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { tail -5 $O/bench_driver.err; exit 1; }
echo "== nv sweep ($(date +%T))"
for nv in 600 765 1024 1025 1500 2500 3069 4096; do
  timeout -k 10 300 python3 bench.py --nv $nv --batch 512 --steps 5 --warmup 2 --sweep none --no-cpu-baseline \
    > $O/nv_sweep/nv$nv.json 2> $O/nv_sweep/nv$nv.err || { tail -5 $O/nv_sweep/nv$nv.err; exit 1; }
done
echo "== smoke ($(date +%T))"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "== done ($(date +%T))"
