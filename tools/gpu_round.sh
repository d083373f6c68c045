#!/bin/bash
# GPU-box round check (run through gpurun): the -m gpu tests, smoke, the C2 bench line, the
# world-1 RCCL bench line with the reassembly in the step, and a kernel trace of the latter (the
# RCCL gathers and the reassembly pass on their own streams beside the next encode).  Every step
# has its own time limit; the script stops at the first failing step.
# usage: tools/gpu_round.sh <tag> [steps...]   steps: pytest smoke c2 gw1 trace_gw1 (default: all)
set -u
TAG=${1:-r3}; shift || true
STEPS=${*:-"pytest smoke c2 gw1 trace_gw1"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$O/status.txt"
  [ $rc -eq 0 ] || exit $rc
}
for s in $STEPS; do
  case $s in
    pytest) run pytest 1200 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ;;
    smoke) run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
    c2) run bench_c2 400 python -u bench.py --steps 20 --warmup 2 ;;
    c5) run bench_c5 400 python -u bench.py --steps 20 --warmup 2 --config c5 --no-cpu-baseline --e2e-steps 0 ;;
    c3) run bench_c3 400 python -u bench.py --steps 20 --warmup 2 --presplit host --no-cpu-baseline --e2e-steps 0 ;;
    gw1) run bench_gw1 400 python -u bench.py --steps 10 --warmup 2 --gather-world1 --no-cpu-baseline --e2e-steps 0 ;;
    trace_gw1) (cd /tmp && export TMPDIR=/tmp && run trace_gw1 400 rocprofv3 --kernel-trace --stats -d "$O/trace_gw1" \
                 -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --gather-world1 \
                 --no-cpu-baseline --e2e-steps 0) || exit $? ;;
    *) echo "unknown step $s" >> "$O/status.txt"; exit 2 ;;
  esac
done
echo all-done >> "$O/status.txt"
