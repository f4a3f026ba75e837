#!/bin/bash
# A/B of the host-resident (PCIe-inclusive) rates: lib/$VARS vs main, same box
set -o pipefail
mkdir -p gpurun_out/ab_e2e
L=erasure-coding-crust_amd/lib
for rep in 1 2; do
for v in ${VARS:-var_base main}; do
  if [ $v = main ]; then unset ECC_AMD_LIB; else export ECC_AMD_LIB=$PWD/$L/$v.so; fi
  timeout -k 10 300 python scripts/bench_e2e.py ${E2E_ARGS:-} > gpurun_out/ab_e2e/$v.json 2> gpurun_out/ab_e2e/$v.err || { tail -5 gpurun_out/ab_e2e/$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_e2e/$v.json')); h=d['host_batch_1MB']
print('$v', 'enc', h['encode_GiBps'], 'rec', h['reconstruct_GiBps'], 'rt', h['roundtrip_GiBps'], 'stream', d['mixed_stream_roundtrip_GiBps'], 'call', d['capi_per_call_1MB']['roundtrip_GiBps'])"
done
done
