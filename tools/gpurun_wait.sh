#!/bin/bash
# Host-side: submit a gpurun call, re-submitting only while the pool answers "transient" (no box / slot free,
# nothing charged).  Usage: tools/gpurun_wait.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$out" 2>&1
  if grep -q "status=transient" "$out"; then sleep 150; continue; fi
  break
done
