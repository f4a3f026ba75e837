set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcab
for m in head 0; do
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/pmcab/$m -o run -- scripts/micro/enc_abl_$m > gpurun_out/pmcab/$m.log 2>&1 || exit 1
done
