#!/bin/bash
# Run one gpurun call; retry ONLY when gpurun reports an infrastructure-side transient
# (no box / slot busy / box taken away: nothing ran, nothing charged).  Never retries a
# command that ran and failed.   usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  out=$(timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  echo "$out" | tail -12
  if echo "$out" | grep -q "status=transient"; then
    echo "[retry $i: transient, sleeping 90s]"; sleep 90; continue
  fi
  break
done
