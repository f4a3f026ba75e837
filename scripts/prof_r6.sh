#!/bin/bash
# Round-6 profile set on the current tree (stops at the first failure):
#  1. headline bench line + rocprofv3 kernel stats of the same command
#  2. SQ counters (+ GRBM_GUI_ACTIVE for the clock) of the headline kernels, B = 512
#  3. PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of the headline workload
#  4. config 4 per GPU (nv 4096, 8192 x 1 MB): bench line + kernel stats,
#     SQ counters at B = 256, PMC traffic at B = 2048
set -u
export TMPDIR=/tmp
O=${O:-gpurun_out/r6prof}; mkdir -p $O
step() { echo "== $1 ($(date +%T))"; }
step headline
timeout -k 10 300 python bench.py --sweep none --no-cpu-baseline --no-e2e > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --sweep none --no-cpu-baseline --no-e2e > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
step sq
sq() {  # $1 dir, $2 bench args
  mkdir -p $1; local i=0
  while read -r line; do
    [ -z "$line" ] && continue; i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $1/p$i -o run -- python3 bench.py $2 > $1/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $1/p$i.log; return 1; }
  done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT
SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_INT32 SQ_INSTS_SMEM SQ_LDS_UNALIGNED_STALL
LIST
}
sq $O/sq "--batch 512 --steps 2 --warmup 1 --sweep none --no-cpu-baseline --no-e2e" || exit 1
python3 scripts/sq_summary.py $O/sq $O/sq_counters.json > /dev/null || exit 1
step traffic
traffic() {  # $1 dir, $2 bench args
  mkdir -p $1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $1/$c -o run -- python3 bench.py $2 > $1/$c.log 2>&1 || { tail -3 $1/$c.log; return 1; }
  done
}
traffic $O/traffic "--steps 2 --warmup 1 --sweep none --no-cpu-baseline --no-e2e" || exit 1
python3 scripts/pmc_summary.py $O/traffic $O/pmc_traffic.json 4096 1024 1000000 342 > /dev/null || exit 1
step c4
timeout -k 10 400 python bench.py --nv 4096 --batch 8192 --sweep none --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/c4_bench.json 2> $O/c4_bench.err || { tail -5 $O/c4_bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4prof -o run -- \
  python3 bench.py --nv 4096 --batch 8192 --sweep none --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/c4prof.log 2>&1 || { tail -5 $O/c4prof.log; exit 1; }
sq $O/c4sq "--nv 4096 --batch 256 --steps 2 --warmup 1 --sweep none --no-cpu-baseline --no-e2e" || exit 1
python3 scripts/sq_summary.py $O/c4sq $O/c4_sq_counters.json > /dev/null || exit 1
traffic $O/c4traffic "--nv 4096 --batch 2048 --steps 2 --warmup 1 --sweep none --no-cpu-baseline --no-e2e" || exit 1
python3 scripts/pmc_summary.py $O/c4traffic $O/c4_pmc_traffic.json 2048 4096 1000000 1366 > /dev/null || exit 1
step done
