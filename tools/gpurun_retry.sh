#!/bin/bash
# gpurun with retries when no box/slot was available (nothing charged, nothing ran): exit code 3,
# a busy pool, a box that stopped responding while being prepared, or an infrastructure back-off
# (its "retry in Ns" is honoured).  usage: tools/gpurun_retry.sh TIMEOUT cmd...
T=$1; shift
for i in $(seq 1 12); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if [ $rc -eq 3 ] || echo "$out" | grep -q "busy\|while being prepared\|status=transient\|backing off\|taken away"; then
    wait_s=$(echo "$out" | grep -o "retry in [0-9]*s" | tail -1 | grep -o "[0-9]*")
    wait_s=${wait_s:-150}
    [ "$wait_s" -lt 60 ] && wait_s=60
    echo "[retry $i: no box; sleeping ${wait_s}s]"; sleep $((wait_s + 10)); continue
  fi
  exit $rc
done
exit 3
