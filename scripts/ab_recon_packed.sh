#!/bin/bash
# A/B on one box: the 1 MB reconstruct through reconstruct_n1024<false> (tiles,
# gather order, workgroup barriers) vs <true> (per-wave groups, compacted
# present rows, no barrier), ECCR_AMD_RECON_PACKED=1 forcing the latter.
set -o pipefail
O=gpurun_out/ab_recon; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python bench.py --sweep none --no-cpu-baseline --steps 5 --batch ${B:-2048} > $O/tile_$rep.json || exit 1
  ECCR_AMD_RECON_PACKED=1 timeout -k 10 300 python bench.py --sweep none --no-cpu-baseline --steps 5 --batch ${B:-2048} > $O/wave_$rep.json || exit 1
done
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['kernels_ms'], d['roundtrip_ok'])"; done
