#!/bin/bash
# Round 5: max-memory-clause per source for the other shapes' kernels
# (k256mcl: enc_k256.hip, genmcl: enc_gen.hip, d4mcl: dec_n4096.hip).
set -o pipefail
export TMPDIR=/tmp
for a in "--nv 1500:512:main k256mcl d4mcl" "--nv 2048:512:main k256mcl d4mcl" "--nv 600:512:main genmcl" "--nv 2500:512:main genmcl d4mcl"; do
  IFS=: read -r args b vars <<< "$a"
  echo "== $args"
  NOTEST=1 VARS="$vars" REPS=3 B=$b ARGS="$args" bash scripts/r5_ab.sh || exit 1
done
