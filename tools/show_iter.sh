#!/bin/bash
D=gpurun_out/iter_$1
cat $D/status.txt; tail -3 $D/pytest_gpu.log
for f in $D/bench_ct*.json; do echo -n "$f "; tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('parity_vs_oracle_sample'))" 2>/dev/null || tail -3 ${f%.json}.err; done
python3 -c "
import csv
for r in csv.DictReader(open('$D/trace/run_kernel_stats.csv')):
    print('%-70s %8.4f ms x%s' % (r['Name'][:70], float(r['AverageNs'])/1e6, r['Calls']))
" 2>/dev/null
