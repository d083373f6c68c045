#!/bin/bash
# GPU box: per-kernel times of library variants on the bench workload (kernel trace, one pass
# per variant, in turn).  usage: tools/gpu_ab_trace.sh TAG spec1 spec2 ...
# spec: lib.so, or lib.so@arg1,arg2 for extra bench.py arguments of that run only (commas
# become spaces); lib: a file name under shredword_amd/, built with `make -C shredword_amd
# variant ...`.  BENCH_ARGS applies to every run.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/abt_$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
names=()
for spec in "$@"; do
  lib=${spec%%@*}
  extra=""
  [ "$lib" != "$spec" ] && extra=${spec#*@} && extra=${extra//,/ }
  name=$(echo "${spec%.so}" | tr -c 'A-Za-z0-9_\n' '_')
  name=${name//_so_/_}
  names+=("$name")
  SHREDWORD_HIP_LIB=$R/shredword_amd/$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --e2e-steps 0 --small-steps 0 ${BENCH_ARGS:-} $extra \
    > "$OUT/$name.log" 2>&1
  rc=$?; echo "$name rc=$rc" >> "$OUT/status.txt"
  [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" "${names[@]}" <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
for name in sys.argv[2:]:
    rows = list(csv.DictReader(open(glob.glob('%s/%s/**/run_kernel_stats.csv' % (out, name), recursive=True)[0])))
    line = [l for l in open('%s/%s.log' % (out, name)) if l.startswith('{')]
    d = json.loads(line[-1]) if line else {}
    print('== %s  value %s MB/s  kernel_ms %s' % (name, d.get('value'), d.get('roofline', {}).get('kernel_ms')))
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
        print('   %-50s %8.4f ms x%s' % (r['Name'][:50], float(r['AverageNs']) / 1e6, r['Calls']))
PY
