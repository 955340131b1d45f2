#!/bin/bash
# queue a gpurun call: retry only while the pool has no free box (status=transient, nothing ran, nothing charged)
# usage: gpuq.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; shift 2
for i in $(seq 1 30); do
  timeout $((lim + 900)) /usr/local/graft/bin/gpurun --timeout $lim -- "$@" > "$out" 2>&1
  if grep -q "status=transient" "$out" && grep -qE "no free box|backing off|stopped responding|slot\(s\) on this pod are busy" "$out"; then sleep 90; continue; fi
  break
done
