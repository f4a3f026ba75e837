#!/bin/bash
# Builds the encode/decode ablation timers (CPU host, gfx950 cross-compile).
cd "$(dirname "$0")"
C=../../erasure-coding-crust_amd/csrc
for m in ${ENC_MASKS:-0 1 2 4 8 16}; do
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -DENC_ABL=$m -I$C enc_ablate.cpp $C/gf_field.cpp $C/ec_runtime.cpp -o enc_abl_$m 2>&1 | grep -i ' error'
done
for m in ${DEC_MASKS:-0 1 2 4 8 16 32}; do
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -DDEC_ABL=$m -I$C dec_ablate.cpp $C/gf_field.cpp $C/ec_runtime.cpp -o dec_abl_$m 2>&1 | grep -i ' error'
done
exit 0
