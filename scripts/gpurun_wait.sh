#!/bin/bash
# gpurun, re-queued while the pool has no free box (exit 3 / "transient":
# nothing ran, nothing charged); any other outcome is returned as is.
# usage: gpurun_wait.sh TIMEOUT_S 'command'
T=$1; shift
for i in $(seq 1 40); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "status=transient"; then sleep 60; continue; fi
  echo "$out"; exit $rc
done
echo "$out"; exit $rc
