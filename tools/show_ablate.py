import csv, glob, os, sys
d = 'gpurun_out/abl_' + sys.argv[1]
rows = {}
libs = sorted(x for x in os.listdir(d) if os.path.isdir(os.path.join(d, x)))
for lib in libs:
    for r in csv.DictReader(open(os.path.join(d, lib, 'run_kernel_stats.csv'))):
        rows.setdefault(r['Name'][:60], {})[lib] = float(r['AverageNs']) / 1e6
print('%-60s ' % 'kernel' + ' '.join('%14s' % l[15:29] for l in libs))
for k, v in sorted(rows.items(), key=lambda kv: -max(kv[1].values())):
    if max(v.values()) < 0.05: continue
    print('%-60s ' % k + ' '.join('%14.3f' % v.get(l, float('nan')) for l in libs))
