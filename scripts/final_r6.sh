#!/bin/bash
# Round-6 closing run: the -m gpu suite, smoke(), and the driver's bench
# command (python3 bench.py --gpus 1 --steps 20 --warmup 5).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6final; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ge 124 ] && exit $rc; [ $rc -ne 0 ] && grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_line.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_line.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['kernels_ms'], d['roofline']['frac'], d['roundtrip_ok'])
e=d['e2e']; print('e2e', e['config2']['roundtrip_GiBps'], e['config2']['frac_of_pcie_bound'], e['config5_mixed']['roundtrip_GiBps'], e['config5_mixed']['frac_of_pcie_bound'])"
