#!/bin/bash
# SQ counter passes (scripts/pmc_sq.sh's three) for each library in VARS at
# a small batch; summaries in gpurun_out/sq_ab/<var>.json
set -u
export TMPDIR=/tmp
L=$PWD/erasure-coding-crust_amd/lib
for v in ${VARS:-main}; do
  unset ECCR_AMD_RECON_WAVES
  if [ $v = main ]; then unset ECC_AMD_LIB; elif [ $v = w8 ]; then unset ECC_AMD_LIB; export ECCR_AMD_RECON_WAVES=8; else export ECC_AMD_LIB=$L/$v.so; fi
  OUT=gpurun_out/sq_ab/$v BENCH_ARGS="${BARGS:---batch 512 --steps 2 --warmup 1 --sweep none --no-cpu-baseline}" bash scripts/pmc_sq.sh > gpurun_out/sq_ab/$v.log 2>&1 || { tail -5 gpurun_out/sq_ab/$v.log; exit 1; }
  python3 scripts/sq_summary.py gpurun_out/sq_ab/$v/pmc_sq gpurun_out/sq_ab/$v.json > /dev/null || exit 1
done
