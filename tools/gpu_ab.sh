#!/bin/bash
# A/B of library variants on the bench workload (GPU box).  usage: tools/gpu_ab.sh tag lib1 lib2 ...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_$TAG; mkdir -p "$OUT"
for lib in "$@"; do
  for ct in 1 0; do
    extra=""; [ $ct = 0 ] && extra="--no-chunk-table"
    SHREDWORD_HIP_LIB=$R/shredword_amd/$lib timeout -k 10 200 python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline $extra > "$OUT/${lib}_ct$ct.json" 2> "$OUT/${lib}_ct$ct.err"
    rc=$?; echo "$lib ct=$ct rc=$rc" >> "$OUT/status.txt"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
