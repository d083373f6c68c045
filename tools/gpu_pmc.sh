#!/bin/bash
# GPU box: one rocprofv3 --pmc pass per counter group over a short bench (no trace domains).
# usage: tools/gpu_pmc.sh tag "GROUP1 COUNTERS" "GROUP2 COUNTERS" ...   (env BENCH_ARGS, KREGEX)
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp ${KREGEX:+--kernel-include-regex "$KREGEX"} -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "p$i ($grp) rc=$rc" >> "$OUT/status.txt"
  case $rc in 124|134|137|139) exit $rc;; esac
done
