#!/bin/bash
# A/B of the per-call C ABI latency (scripts/micro/capi_bench): the round-1
# library (scripts/micro/base_lib) vs the tree's, same box
set -o pipefail
mkdir -p gpurun_out/ab_capi
for rep in 1 2; do
  LD_LIBRARY_PATH=$PWD/scripts/micro/${BASE:-base_lib} timeout -k 10 400 scripts/micro/capi_bench > gpurun_out/ab_capi/base_$rep.jsonl || exit 1
  timeout -k 10 400 scripts/micro/capi_bench > gpurun_out/ab_capi/main_$rep.jsonl || exit 1
done
python3 - <<'PY'
import json
for rep in (1, 2):
    for v in ("base", "main"):
        rows = [json.loads(l) for l in open(f"gpurun_out/ab_capi/{v}_{rep}.jsonl")]
        print(v, rep, " ".join(f"{r['n_validators']}/{r['payload_bytes']}:{r['obtain_chunks_us']}/{r['reconstruct_threshold_us']}" for r in rows))
PY
