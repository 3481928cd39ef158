#!/bin/bash
# Client-side helper: run one gpurun call; when the infrastructure reports a
# transient failure (box not prepared, nothing charged) wait and submit the
# same call again, at most 3 attempts.  GPU-side failures are never retried.
T=${GPU_TIMEOUT:-900}
for a in 1 2 3; do
  out=$(/usr/local/graft/bin/gpurun --timeout $T -- "$@" 2>&1)
  echo "$out" | grep -v "^$" | tail -5
  if echo "$out" | grep -q "status=transient"; then sleep 60; continue; fi
  break
done
