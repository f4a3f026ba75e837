#!/bin/bash
# rocprofv3 kernel stats of the round-6 encodes at their shapes (512 x 1 MB):
# nv 600 (encode_kw<7>), 1500 (encode_kw<8>), 3069 (encode_k512w), 300
# (encode_kw<6>), 100 (encode_kw<5>), 64 (encode_kw<4>); summaries copied to
# profiles/r06/newkernels/.
set -u
export TMPDIR=/tmp
O=${O:-gpurun_out/newk}; mkdir -p $O
for nv in ${NVS:-600 1500 3069 300 100 64}; do
  ( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/nv$nv -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --nv $nv --batch 512 --steps 5 --warmup 2 --no-cpu-baseline --sweep none --no-e2e \
      > $GRAFT_REPO_ROOT/$O/nv$nv.json 2> $GRAFT_REPO_ROOT/$O/nv$nv.err ) || { echo "nv $nv failed"; tail -3 $O/nv$nv.err; exit 1; }
  f=$(find $O/nv$nv -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/nv${nv}_kernel_stats.csv
  echo "== nv $nv"; cut -d, -f1-4 $O/nv${nv}_kernel_stats.csv | grep -E "encode|reconstruct" | cut -c1-160
done
