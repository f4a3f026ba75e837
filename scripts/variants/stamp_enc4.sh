set -u
export TMPDIR=/tmp
L=$PWD/erasure-coding-crust_amd/lib
mkdir -p gpurun_out/stamps
NV=4096 ECC_AMD_LIB=$L/diag_enc4_stamp.so timeout -k 10 300 python scripts/variants/stamp_run.py enc load,sys_stores,vmcnt0_barrier,ifft,coef,fft,-,barriers,stage,dma,stores 1024 > gpurun_out/stamps/enc4.txt 2>&1 || { tail -5 gpurun_out/stamps/enc4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps/enc4.txt
