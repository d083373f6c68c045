#!/bin/bash
# GPU box: kernel trace of a short bench run and the per-launch gap table.  usage: tools/gpu_gaps.sh TAG [bench args]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-gaps}; shift || true
OUT=$R/gpurun_out/gaps_$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 "$@" > "$OUT/trace.log" 2>&1 || exit 1
python3 "$R/tools/gaps.py" "$OUT/trace/run_kernel_trace.csv" > "$OUT/gaps.txt"
