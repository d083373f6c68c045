"""Summarise gpurun_out/args_<tag>: bench value and per-kernel average ms per argument set."""
import csv, json, os, sys
d = 'gpurun_out/args_' + sys.argv[1]
idx = [(l.split(':', 1)[0], l.split(':', 1)[1].strip()) for l in open(d + '/index.txt')]
rows = {}
for i, args in idx:
    try:
        j = [json.loads(l) for l in open('%s/b%s.log' % (d, i)) if l.startswith('{')][-1]
        print('%-3s %-40s %10.1f MB/s  %8.3f ms/step' % (i, args[:40], j['value'], j['ms_per_step']))
    except Exception as e:
        print(i, args, 'no bench line', e)
    f = '%s/trace_%s/run_kernel_stats.csv' % (d, i)
    if os.path.exists(f):
        for r in csv.DictReader(open(f)):
            rows.setdefault(r['Name'][:50], {})[i] = float(r['AverageNs']) / 1e6
ids = [i for i, _ in idx]
print('%-50s ' % 'kernel avg ms' + ' '.join('%8s' % i for i in ids))
for k, v in sorted(rows.items(), key=lambda kv: -max(kv[1].values())):
    if max(v.values()) < 0.03:
        continue
    print('%-50s ' % k + ' '.join('%8.3f' % v.get(i, float('nan')) for i in ids))
