#!/bin/bash
# GPU box: kernel-trace stats of a short bench run (no tests).  usage: tools/gpu_trace.sh TAG [bench args]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-tr}; shift || true
OUT=$R/gpurun_out/trace_$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc" > "$OUT/status.txt"
python3 - "$OUT" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1] + '/trace/run_kernel_stats.csv')):
    print('%-60s %8.4f ms x%s' % (r['Name'][:60], float(r['AverageNs'])/1e6, r['Calls']))
PY
grep '^{' "$OUT/trace.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])"
exit $rc
