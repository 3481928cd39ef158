#!/bin/bash
# Client-side helper: run one gpurun call; when the infrastructure reports a
# transient failure (box not prepared / pool busy, nothing charged) wait and
# submit the same call again (RETRIES attempts, default 8).  GPU-side failures
# are never retried.
T=${GPU_TIMEOUT:-900}
N=${RETRIES:-8}
for a in $(seq 1 $N); do
  out=$(/usr/local/graft/bin/gpurun --timeout $T -- "$@" 2>&1)
  echo "$out" | grep -v "^$" | tail -5
  if echo "$out" | grep -q "status=transient"; then sleep 90; continue; fi
  break
done
