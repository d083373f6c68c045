"""Summarise gpurun_out/cmp_<tag>: bench value per library and per-kernel average ms."""
import csv, glob, json, os, sys
d = 'gpurun_out/cmp_' + sys.argv[1]
libs = sorted(os.path.basename(p)[:-5] for p in glob.glob(d + '/*.so.json'))
for lib in libs:
    try:
        j = json.loads(open(f'{d}/{lib}.json').read().strip().splitlines()[-1])
        print('%-34s %10.1f MB/s  %8.3f ms/step  frac %.4f' % (lib, j['value'], j['ms_per_step'], j['roofline']['frac']))
    except Exception as e:
        print(lib, 'no bench line', e)
rows = {}
for lib in libs:
    f = f'{d}/trace_{lib}/run_kernel_stats.csv'
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        rows.setdefault(r['Name'][:58], {})[lib] = float(r['AverageNs']) / 1e6 * (2 if 'scan' in r['Name'] else 1)
print('%-58s ' % 'kernel (avg ms per launch; scans x2)' + ' '.join('%12s' % l.replace('libshredword_hip', '')[:12] for l in libs))
tot = {l: 0.0 for l in libs}
for k, v in sorted(rows.items(), key=lambda kv: -max(kv[1].values())):
    for l in libs:
        tot[l] += v.get(l, 0)
    if max(v.values()) < 0.02:
        continue
    print('%-58s ' % k + ' '.join('%12.3f' % v.get(l, float('nan')) for l in libs))
print('%-58s ' % 'TOTAL' + ' '.join('%12.3f' % tot[l] for l in libs))
