#!/bin/bash
# Build an A/B variant of the library: build_var.sh NAME [EXTRA_FLAGS] [SRC=FILE ...]
# copies erasure-coding-crust_amd/ to a scratch dir, substitutes the given
# csrc sources, builds with the extra flags (and one make variable MAKEVARS, e.g.
# "SCHED_enc_k256w.hip=") and installs lib/NAME.so.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; EXTRA=${2:-}; shift $(( $# >= 2 ? 2 : 1 ))
W=$(mktemp -d /tmp/var_XXXX)
cp -r "$ROOT/erasure-coding-crust_amd" "$ROOT/include" "$W/"
rm -rf "$W/erasure-coding-crust_amd/build" "$W/erasure-coding-crust_amd/lib"
for sub in "$@"; do cp "${sub#*=}" "$W/erasure-coding-crust_amd/csrc/${sub%%=*}"; done
make -C "$W/erasure-coding-crust_amd" -j8 ${MAKEVARS:+"$MAKEVARS"} FLAGS="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter --offload-arch=gfx950 $EXTRA" > "$W/build.log" 2>&1 || { tail -20 "$W/build.log"; exit 1; }
cp "$W/erasure-coding-crust_amd/lib/liberasure_coding_crust.so" "$ROOT/erasure-coding-crust_amd/lib/$NAME.so"
rm -rf "$W"
echo "built lib/$NAME.so"
