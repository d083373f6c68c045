#!/bin/bash
# GPU-box profiling recipe (run through gpurun).  Kernel trace + stats, then one rocprofv3 pass
# per PMC counter group (never combined with trace domains).  Stops at the first step that
# times out / aborts / faults; a rejected counter name only skips that pass.
# usage: tools/profile_gpu.sh <tag> [bench args...]
set -u
TAG=${1:-r1}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH=(python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 --small-steps 0 "$@")
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2" >> "$OUT/status.txt"; exit $1;; esac; }
rocprofv3 -L > "$OUT/counters_available.txt" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc" >> "$OUT/status.txt"; fatal $rc trace
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i ($grp) rc=$rc" >> "$OUT/status.txt"; fatal $rc "pmc$i"
done
echo all-done >> "$OUT/status.txt"
