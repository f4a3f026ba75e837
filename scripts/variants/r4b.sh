set -u
export TMPDIR=/tmp
VARS="var_oldrec var_rec8 main" REPS=2 bash scripts/ab_r4.sh || exit 1
L=$PWD/erasure-coding-crust_amd/lib
mkdir -p gpurun_out/stamps
ECC_AMD_LIB=$L/diag_decw_stamp.so timeout -k 10 200 python scripts/variants/stamp_run.py dec gather,barriers,ifft,deriv+fft,output 1024 > gpurun_out/stamps/decw.txt 2>&1 || { tail -5 gpurun_out/stamps/decw.txt; exit 1; }
cat gpurun_out/stamps/decw.txt
ECC_AMD_LIB=$L/diag_encw_stamp.so timeout -k 10 200 python scripts/variants/stamp_run.py enc load,barrier,stores,compute 1024 > gpurun_out/stamps/encw.txt 2>&1 || { tail -5 gpurun_out/stamps/encw.txt; exit 1; }
cat gpurun_out/stamps/encw.txt
