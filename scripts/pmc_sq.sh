#!/bin/bash
# SQ counters (VALU / LDS / wait) of the bench kernels: one rocprofv3 --pmc
# pass per group (<= 8 SQ counters each), kernel-trace only, small batch.
# Summarised by scripts/pmc_sq_summary.py into profiles/<round>/sq_counters.json.
set -u
export TMPDIR=/tmp
O=${OUT:-gpurun_out}/pmc_sq
mkdir -p $O
ARGS=${BENCH_ARGS:-"--batch 512 --steps 2 --warmup 1 --no-cpu-baseline"}
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "=== pass $i: $line"
  timeout -s KILL 240 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $O/p$i -o run -- python3 bench.py $ARGS > $O/p$i.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_INT32 SQ_INSTS_SMEM SQ_LDS_UNALIGNED_STALL
LIST
