#!/bin/bash
# gpurun with retries when no box/slot was available (nothing charged, nothing ran): exit code 3,
# or a box that stopped responding while being prepared.  usage: tools/gpurun_retry.sh TIMEOUT cmd...
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if [ $rc -eq 3 ] || echo "$out" | grep -q "busy\|while being prepared\|status=transient"; then
    echo "[retry $i: no box]"; sleep 150; continue
  fi
  exit $rc
done
exit 3
