set -u
export TMPDIR=/tmp
L=$PWD/erasure-coding-crust_amd/lib
mkdir -p gpurun_out/stamps
for v in ${VARS:-diag_dec_stamp}; do
  ECC_AMD_LIB=$L/$v.so timeout -k 10 200 python scripts/variants/stamp_run.py dec gather,barriers,ifft,deriv+fft,output 1024 > gpurun_out/stamps/$v.txt 2>&1 || { tail -5 gpurun_out/stamps/$v.txt; exit 1; }
  echo "== $v"; cat gpurun_out/stamps/$v.txt | grep -v amdgpu.ids
done
