set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -k "graph_capture_ws or empty_quarters or nv4096 or past_4GiB" --timeout 120 --timeout-method thread 2>&1 | tail -3
