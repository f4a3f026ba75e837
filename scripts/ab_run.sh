#!/bin/bash
# A/B: bench the default workload with alternative library builds (lib/var_*.so).
# Variants named diag* are diagnostic builds with wrong results by design: their
# failed round trip (exit 1) is accepted, the timing line is still printed.
set -o pipefail
mkdir -p gpurun_out/ab
L=erasure-coding-crust_amd/lib
for rep in 1 2; do
for v in ${VARS:-var_0 main var_a}; do
  if [ $v = main ]; then unset ECC_AMD_LIB; else export ECC_AMD_LIB=$PWD/$L/$v.so; fi
  timeout -k 10 200 python bench.py --batch ${B:-2048} --steps 5 --warmup 2 --no-cpu-baseline ${ARGS:-} > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err
  rc=$?
  if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [ "${v#diag}" != "$v" ]; }; then tail -5 gpurun_out/ab/$v.err; exit 1; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/ab/$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['kernels_ms'])"
done
done
