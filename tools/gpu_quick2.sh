#!/bin/bash
# GPU box: the -m gpu suite (time-limited), then short C2 / C5 bench lines and a C5 kernel trace.
# usage: tools/gpu_quick2.sh TAG [pytest -k expression]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-q}; K=${2:-}
OUT=$R/gpurun_out/q_$TAG; mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest "$R/tests" -m gpu -x -v --timeout 150 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1
else
  timeout -k 10 500 python -u -m pytest "$R/tests" -m gpu -x -v --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1
fi
rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for cfg in c2 c5; do
  timeout -k 10 200 python3 -u "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --e2e-steps 0 --config ${cfg/c2/c3} > "$OUT/bench_$cfg.log" 2>&1
  rc=$?; echo "bench $cfg rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
  grep '^{' "$OUT/bench_$cfg.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
"$R/tools/gpu_trace.sh" "${TAG}_c5" --config c5
