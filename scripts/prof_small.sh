#!/bin/bash
# rocprofv3 kernel stats of the default bench step at the benchmark/ small
# payload sizes (nv = 1024, 4096 payloads, tight payload pitch).
set -u
export TMPDIR=/tmp
O=${O:-gpurun_out/small}
mkdir -p $O
for p in ${SIZES:-15 300 5000}; do
  echo "=== $p ($(date +%T))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$p -o run -- \
    python3 bench.py --payload $p --batch ${BATCH:-4096} --steps 5 --warmup 2 --no-cpu-baseline > $O/p$p.log 2>&1
  rc=$?
  tail -1 $O/p$p.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
  f=$(find $O/p$p -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && cut -d, -f1-4 "$f" | head -14
done
