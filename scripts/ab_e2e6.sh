#!/bin/bash
# Round-6 A/B of the host-batch pipeline variants (lib/<name>.so, main = the
# default build): bench.py's e2e block only matters, the device part is tiny.
set -o pipefail
O=gpurun_out/r6/e2e; mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
for v in ${VARS:-main}; do
  if [ "$v" = main ]; then unset ECC_AMD_LIB; else export ECC_AMD_LIB=$PWD/erasure-coding-crust_amd/lib/$v.so; fi
  timeout -k 10 200 python bench.py --batch 64 --steps 1 --warmup 1 --sweep none --no-cpu-baseline ${ARGS:-} > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); e=d['e2e']; c=e['config2']; m=e['config5_mixed']
print('$v', 'c2 enc %.2f rec %.2f rt %.3f (%.3f)' % (c['encode_GiBps'], c['reconstruct_GiBps'], c['roundtrip_GiBps'], c['frac_of_pcie_bound']), 'c5 %.3f (%.3f)' % (m['roundtrip_GiBps'], m['frac_of_pcie_bound']), c['roundtrip_ok'] and m['roundtrip_ok'])"
done
done
