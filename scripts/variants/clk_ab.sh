#!/bin/bash
# Shader clock under load: clk_run.py over the clock-probe variants
# (scripts/variants/enc_diag.py clk / dclk, built into lib/diag_*.so).
set -o pipefail
export TMPDIR=/tmp
L=$PWD/erasure-coding-crust_amd/lib
for v in ${CLKV:-diag_clk:enc diag_clk_nostg:enc diag_dclk:dec}; do
  ECC_AMD_LIB=$L/${v%%:*}.so timeout -k 10 200 python scripts/variants/clk_run.py ${v##*:} ${B:-4096} 5 2>&1 | grep -v amdgpu.ids || exit 1
done
