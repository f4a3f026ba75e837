#!/bin/bash
# Round-6 GPU step: (unless NOTEST=1) the -m gpu suite on the default library
# (-k $PYK to narrow), (if BENCH=1) one default bench.py line, then
# scripts/ab_r4.sh over VARS.  A failing test does not stop the A/B; a
# timeout, abort or crash (status >= 124) stops everything after it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
stop_on_fault() { if [ "$1" -ge 124 ]; then echo "FAULT status $1 in $2: stopping"; exit "$1"; fi; }
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && grep -E "^(FAILED|ERROR)|Error" $O/pytest_gpu.log | head -20
  stop_on_fault $rc pytest
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 300 python bench.py ${BENCHARGS:-} > $O/bench_default.json 2> $O/bench_default.err
  rc=$?; stop_on_fault $rc bench
  python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['kernels_ms'], d['roundtrip_ok'])
e=d.get('e2e')
if e: print('e2e', e['pcie_measured'], {k: (e[k]['roundtrip_GiBps'], e[k]['frac_of_pcie_bound']) for k in ('config2','config5_mixed')})
" || tail -5 $O/bench_default.err
fi
[ -n "${VARS:-}" ] && bash scripts/ab_r4.sh
exit 0
