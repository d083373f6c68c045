#!/bin/bash
# GPU box: per-phase cycle stamps (SW_STAMPS build) for the MIXED and the STRESS corpus.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for kind in mixed stress; do
  SHREDWORD_HIP_LIB=$R/shredword_amd/libshredword_hip_stamps.so timeout -k 10 200 python3 "$R/tools/phase_stamps.py" 250000 $kind > "$R/gpurun_out/stamps_$kind.log" 2>&1
  rc=$?; cat "$R/gpurun_out/stamps_$kind.log"; [ $rc -eq 0 ] || exit $rc
done
