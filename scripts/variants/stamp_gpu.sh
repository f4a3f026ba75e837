set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/stamps
L=$PWD/erasure-coding-crust_amd/lib
ECC_AMD_LIB=$L/diag_enc_stamp.so timeout -k 10 200 python scripts/variants/stamp_run.py enc load,barrier,stores,compute 1024 > gpurun_out/stamps/enc.txt 2>&1 || { tail -5 gpurun_out/stamps/enc.txt; exit 1; }
cat gpurun_out/stamps/enc.txt
ECC_AMD_LIB=$L/diag_dec_stamp.so timeout -k 10 200 python scripts/variants/stamp_run.py dec gather,barriers,ifft,deriv+fft,output 1024 > gpurun_out/stamps/dec.txt 2>&1 || { tail -5 gpurun_out/stamps/dec.txt; exit 1; }
cat gpurun_out/stamps/dec.txt
