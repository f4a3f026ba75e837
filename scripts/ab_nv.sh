set -o pipefail
for nv in 4096 2500 2048 1500; do
  echo "nv=$nv"
  VARS="main var_e" B=512 ARGS="--nv $nv" bash scripts/ab_run.sh || exit 1
done
