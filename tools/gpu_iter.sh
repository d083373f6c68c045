#!/bin/bash
# one iteration on the GPU box: gpu tests, bench (chunk table on/off), kernel-trace stats
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-it}
OUT=$R/gpurun_out/iter_$TAG; mkdir -p "$OUT"
timeout -k 10 500 python3 -m pytest "$R/tests" -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; case $rc in 124|134|137|139) exit $rc;; esac
for ct in 1 0 d; do
  extra=""; [ $ct = 0 ] && extra="--no-chunk-table"; [ $ct = d ] && extra="--no-dedupe"
  timeout -k 10 300 python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline $extra > "$OUT/bench_ct$ct.json" 2> "$OUT/bench_ct$ct.err"
  rc=$?; echo "bench ct=$ct rc=$rc" >> "$OUT/status.txt"; case $rc in 124|134|137|139) exit $rc;; esac
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/trace.log" 2>&1
echo "trace rc=$?" >> "$OUT/status.txt"
