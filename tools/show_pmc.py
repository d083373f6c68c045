"""Per-kernel mean of every counter in gpurun_out/pmc_<tag>/p*/run_counter_collection.csv."""
import csv, glob, sys, collections
d = 'gpurun_out/pmc_' + sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(d + '/p*/**/*counter_collection.csv', recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r['Kernel_Name'][:48], r['Counter_Name'], r['Dispatch_Id'])] += float(r['Counter_Value'])
    for (k, c, _), v in per.items():
        acc[k][c].append(v)
for k in sorted(acc):
    print(k)
    for c in sorted(acc[k]):
        v = acc[k][c]
        print('   %-40s %16.4g' % (c, sum(v) / len(v)))
