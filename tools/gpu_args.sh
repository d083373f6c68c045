#!/bin/bash
# GPU box: one bench line + kernel trace per bench argument set.  usage: tools/gpu_args.sh tag "args1" "args2" ...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/args_$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for args in "$@"; do
  i=$((i+1))
  echo "$i: $args" >> "$OUT/index.txt"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline $args > "$OUT/b$i.log" 2>&1)
  rc=$?; echo "$i rc=$rc" >> "$OUT/status.txt"; case $rc in 124|134|137|139) exit $rc;; esac
done
