#!/bin/bash
# VALU-issue counters for the encode kernel vs the pure-ALU microbenchmarks.
set -u
export TMPDIR=/tmp
O=gpurun_out/pmcv; mkdir -p $O
timeout -k 10 60 scripts/micro/oprate > $O/oprate.txt 2>&1 || exit 1
timeout -k 10 60 scripts/micro/mulrate > $O/mulrate.txt 2>&1 || exit 1
P="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_CYCLES"
for b in ${BINS:-enc_pipe mulrate}; do
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/$b -o run -- scripts/micro/$b > $O/$b.log 2>&1 || exit 1
done
