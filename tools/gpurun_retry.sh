#!/bin/bash
# Submits one gpurun call, resubmitting it (up to 20 times, 2 min apart) only while the pool has
# no free box (nothing ran, nothing charged).  Any other outcome ends it.
# usage: tools/gpurun_retry.sh <out file> <timeout s> <command>
out=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient" "$out"; then sleep 90; continue; fi
  echo "rc=$rc" >> "$out"; exit $rc
done
