#!/bin/bash
# PMC collection: separate passes (one rocprofv3 run per counter group),
# kernel-trace only (no sys/runtime trace with --pmc).
set -u
OUT=${OUT:-gpurun_out}/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
ARGS="bench.py --batch 256 --steps 2 --warmup 1 --no-cpu-baseline"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "=== pass $i: $line"
  timeout -k 10 300 rocprofv3 --pmc $line --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- python3 $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD
FETCH_SIZE
WRITE_SIZE
GRBM_GUI_ACTIVE GRBM_COUNT
LIST
