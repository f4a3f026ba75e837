#!/bin/bash
# A/B of lib/$VARS over payload sizes (nv = ${NV:-1024}): bench.py per size
set -o pipefail
mkdir -p gpurun_out/ab_sizes
L=erasure-coding-crust_amd/lib
for cfg in ${CFGS:-"15:4096" "300:4096" "5000:4096" "100000:1024" "1000000:2048"}; do
  plen=${cfg%%:*}; B=${cfg##*:}
  for v in ${VARS:-var_base main}; do
    if [ $v = main ]; then unset ECC_AMD_LIB; else export ECC_AMD_LIB=$PWD/$L/$v.so; fi
    timeout -k 10 200 python bench.py --nv ${NV:-1024} --payload $plen --batch $B --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_sizes/$v.json 2> gpurun_out/ab_sizes/$v.err || { tail -5 gpurun_out/ab_sizes/$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_sizes/$v.json')); print('$plen x $B', '$v', d['value'], d['kernels_ms'], d['roundtrip_ok'])"
  done
done
