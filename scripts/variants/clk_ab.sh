set -o pipefail
export TMPDIR=/tmp
L=$PWD/erasure-coding-crust_amd/lib
for v in ${CLKV:-diag_clk diag_clk_nostg}; do
  ECC_AMD_LIB=$L/$v.so timeout -k 10 200 python scripts/variants/clk_run.py 4096 5 2>&1 | grep -v amdgpu.ids || exit 1
done
