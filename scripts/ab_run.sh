#!/bin/bash
# A/B: bench the default workload with alternative library builds (lib/var_*.so)
set -o pipefail
mkdir -p gpurun_out/ab
L=erasure-coding-crust_amd/lib
for rep in 1 2; do
for v in ${VARS:-var_0 main var_a}; do
  if [ $v = main ]; then unset ECC_AMD_LIB; else export ECC_AMD_LIB=$PWD/$L/$v.so; fi
  timeout -k 10 200 python bench.py --batch ${B:-2048} --steps 5 --warmup 2 --no-cpu-baseline ${ARGS:-} > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || { tail -5 gpurun_out/ab/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$v.json')); print('$v', d['value'], d['kernels_ms'])"
done
done
