#!/bin/bash
# Round-4 A/B: parity subset on the default library (-k $TESTK), then the
# bench workload (B, ARGS) on each library in VARS (main = the default build,
# else lib/<name>.so), REPS rounds alternating.  Variants named diag* may fail
# their round trip (exit 1), the others may not.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
if [ -n "${TESTK:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTK" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
  tail -1 $O/parity.log
fi
L=erasure-coding-crust_amd/lib
for rep in $(seq 1 ${REPS:-2}); do
for v in ${VARS:-main}; do
  unset ECCR_AMD_RECON_WAVES ECCR_AMD_RECON_PACKED
  # w8: the default library with the 8-wave n = 1024 reconstruct; w8p: its packed form
  case $v in
    main) unset ECC_AMD_LIB ;;
    w8) unset ECC_AMD_LIB; export ECCR_AMD_RECON_WAVES=8 ;;
    w8p) unset ECC_AMD_LIB; export ECCR_AMD_RECON_WAVES=8 ECCR_AMD_RECON_PACKED=1 ;;
    *) export ECC_AMD_LIB=$PWD/$L/$v.so ;;
  esac
  timeout -k 10 300 python bench.py --batch ${B:-4096} --steps ${STEPS:-5} --warmup 2 --sweep none --no-cpu-baseline ${ARGS:-} > $O/$v.json 2> $O/$v.err
  rc=$?
  if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [ "${v#diag}" != "$v" ]; }; then tail -5 $O/$v.err; exit 1; fi
  python3 -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['kernels_ms'], d['roundtrip_ok'])"
done
done
