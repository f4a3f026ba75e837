#!/bin/bash
# Ablation timings + SQ counter passes for the specialised encode/decode
# kernels (binaries built by scripts/micro/build_ablate.sh on the CPU host).
set -u
export TMPDIR=/tmp
O=gpurun_out/abl
mkdir -p $O
for m in 0 1 2 4 8 16; do timeout -k 10 60 scripts/micro/enc_abl_$m >> $O/times.txt 2>&1 || exit 1; done
for m in 0 1 2 4 8 16 32; do timeout -k 10 60 scripts/micro/dec_abl_$m >> $O/times.txt 2>&1 || exit 1; done
cat $O/times.txt
P1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_IDX_ACTIVE"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
for k in enc dec; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/${k}_p$i -o run -- scripts/micro/${k}_abl_0 > $O/${k}_p$i.log 2>&1 || exit 1
  done
done
