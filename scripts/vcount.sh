#!/bin/bash
# SQ instruction counts per wave at one tile per workgroup (B = 8), for the
# default library and diagnostic builds (lib/diag_*.so; wrong results by design)
export TMPDIR=/tmp
O=gpurun_out/vcount; mkdir -p $O
for v in ${VARS:-main}; do
  if [ $v = main ]; then unset ECC_AMD_LIB; else export ECC_AMD_LIB=$PWD/erasure-coding-crust_amd/lib/$v.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $O/$v -o run -- python3 bench.py --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --sweep none > $O/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -le 1 ] || exit $rc
done
