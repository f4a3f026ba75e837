set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/stride
for rep in 1 2; do
for st in ${STRIDES:-1024 1088}; do
  timeout -k 10 300 python bench.py --nv ${NV:-4096} --batch ${B:-2048} --steps 3 --warmup 1 --sweep none --no-cpu-baseline --row-stride $st > gpurun_out/stride/s$st.json 2> gpurun_out/stride/s$st.err || { tail -5 gpurun_out/stride/s$st.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/stride/s$st.json').read().strip().splitlines()[-1]); print('stride $st', d['value'], d['kernels_ms'], d['roundtrip_ok'])"
done
done
