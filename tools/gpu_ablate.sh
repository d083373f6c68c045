#!/bin/bash
# kernel-time ablation: rocprofv3 kernel stats of bench.py with each library variant
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/abl_$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in "$@"; do
  cd /tmp && SHREDWORD_HIP_LIB=$R/shredword_amd/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$lib" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$lib.log" 2>&1
  rc=$?; echo "$lib rc=$rc" >> "$OUT/status.txt"; case $rc in 124|134|137|139) exit $rc;; esac
done
