#!/bin/bash
# Builds the encode/decode kernel timers (CPU host, gfx950 cross-compile): the
# kernel file compiled inside the timer (EXTRA=-DDEC_STAMP: phase split),
# linked with the product objects of every other source (make first).
cd "$(dirname "$0")"
C=../../erasure-coding-crust_amd/csrc
O=../../erasure-coding-crust_amd/build/obj
others() { for o in ec_kernels enc_k256 enc_k1024 enc_gen dec_n1024 dec_n4096 dec_gen host_pipeline capi ec_runtime gf_field; do
  case $o in "$1") ;; *) [ -f $O/$o.hip.o ] && echo $O/$o.hip.o || echo $O/$o.cpp.o ;; esac; done; }
for m in ${ENC_MASKS:-0}; do
  hipcc -O3 -std=c++17 --offload-arch=gfx950 $EXTRA -I$C -x hip enc_ablate.cpp -x none $(others enc_k256) -o enc_abl_$m 2>&1 | grep -i ' error' | head -5
done
for m in ${DEC_MASKS:-0}; do
  hipcc -O3 -std=c++17 --offload-arch=gfx950 $EXTRA -I$C -x hip dec_ablate.cpp -x none $(others dec_n1024) -o dec_abl_$m 2>&1 | grep -i ' error' | head -5
done
exit 0
