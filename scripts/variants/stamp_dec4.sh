set -u
export TMPDIR=/tmp
L=$PWD/erasure-coding-crust_amd/lib
mkdir -p gpurun_out/stamps
NV=4096 ECC_AMD_LIB=$L/diag_dec4_stamp.so timeout -k 10 300 python scripts/variants/stamp_run.py dec gather,wait_tab_bar,ifft,bar_dma,accum,deriv_fft,outtab,output 1024 > gpurun_out/stamps/dec4.txt 2>&1 || { tail -5 gpurun_out/stamps/dec4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps/dec4.txt
