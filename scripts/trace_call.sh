#!/bin/bash
# HIP-API + kernel + copy trace of single small C-ABI calls:
# scripts/micro/capi_bench at 15 B, nv = 6 and 1024, 20 calls of each kind.
export TMPDIR=/tmp
O=${O:-gpurun_out/calltrace_after}
mkdir -p $O
timeout -k 10 120 scripts/micro/capi_bench 15 200 > $O/capi_15.jsonl 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
  -d $O/trace -o run -- scripts/micro/capi_bench 15 20 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
cat $O/capi_15.jsonl
