set -u
for nv in 4096 2048 512 100; do
  timeout -k 10 300 python bench.py --nv $nv --batch 64 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/nv_$nv.json 2> gpurun_out/nv_$nv.err || { tail -5 gpurun_out/nv_$nv.err; exit 1; }
done
