#!/bin/bash
# gpurun with waits while the pool has no free box (status=transient: nothing ran, nothing charged).
# usage: tools/gpu_retry.sh TIMEOUT 'command'
t=$1; shift
for i in $(seq 1 20); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "status=transient"; then sleep 150; continue; fi
  echo "$out" | tail -40; exit $rc
done
echo "no box after 20 tries"; exit 3
