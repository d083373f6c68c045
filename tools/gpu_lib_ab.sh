#!/bin/bash
# Device-rate A/B of library variants (GPU box), interleaved passes, no profiler.
# usage: tools/gpu_lib_ab.sh PASSES lib1.so lib2.so ...   (BENCH_ARGS: extra bench.py arguments)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=$1; shift
OUT=$R/gpurun_out/lib_ab; mkdir -p "$OUT"; : > "$OUT/summary.txt"
for pass in $(seq 1 "$P"); do
  for lib in "$@"; do
    SHREDWORD_HIP_LIB=$R/shredword_amd/$lib timeout -k 10 200 python3 "$R/bench.py" --steps 20 --warmup 2 \
      --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS:-} > "$OUT/${lib}_p$pass.log" 2>&1 || exit 1
    grep '^{' "$OUT/${lib}_p$pass.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$pass $lib', d['value'], d['roofline']['kernel_ms'])" >> "$OUT/summary.txt"
  done
done
