#!/bin/bash
# GPU box: gpu tests (default lib), then per library variant a bench line and a kernel trace.
# usage: tools/gpu_cmp.sh tag [--no-tests] lib1.so lib2.so ...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cmp_$TAG; mkdir -p "$OUT"
if [ "${1:-}" = "--no-tests" ]; then shift; else
  timeout -k 10 500 python3 -m pytest "$R/tests" -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; case $rc in 124|134|137|139) exit $rc;; esac
fi
export TMPDIR=/tmp
for lib in "$@"; do
  export SHREDWORD_HIP_LIB=$R/shredword_amd/$lib
  timeout -k 10 200 python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/${lib}.json" 2> "$OUT/${lib}.err"
  rc=$?; echo "$lib bench rc=$rc" >> "$OUT/status.txt"; case $rc in 124|134|137|139) exit $rc;; esac
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_${lib}" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/trace_${lib}.log" 2>&1)
  rc=$?; echo "$lib trace rc=$rc" >> "$OUT/status.txt"; case $rc in 124|134|137|139) exit $rc;; esac
done
