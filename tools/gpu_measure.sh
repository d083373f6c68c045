#!/bin/bash
# GPU box: one bench line per workload variant (C2, C3, C5, C2 without each memoisation
# shortcut), each time-limited, then a kernel trace of C5.  Stops at the first fatal step.
# usage: tools/gpu_measure.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-m}
OUT=$R/gpurun_out/measure_$TAG; mkdir -p "$OUT"
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 240 python3 -u "$R/bench.py" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc" >> "$OUT/status.txt"
  grep '^{' "$OUT/$name.log" > "$OUT/$name.json" || true
  return $rc
}
run c2 --steps 10 --warmup 2 &&
run c3 --steps 10 --warmup 2 --presplit host --no-cpu-baseline --e2e-steps 0 &&
run c5 --steps 10 --warmup 2 --config c5 &&
run c2_nodedupe --steps 5 --warmup 1 --no-dedupe --no-cpu-baseline --e2e-steps 0 &&
run c2_nochunktable --steps 5 --warmup 1 --no-chunk-table --no-cpu-baseline --e2e-steps 0 &&
run c2_none --steps 5 --warmup 1 --no-chunk-table --no-dedupe --no-cpu-baseline --e2e-steps 0 || exit $?
echo all-done >> "$OUT/status.txt"
