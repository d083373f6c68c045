#!/usr/bin/env python3
"""Per-kernel PMC means of tools/box.sh `fetch=` passes (FETCH_SIZE / WRITE_SIZE in KB -> GB per
dispatch, TCC hit rate).  usage: tools/fetch_summary.py gpurun_out/TAG [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
runs = collections.defaultdict(dict)
files = glob.glob(os.path.join(root, "fetch_*", "**", "*counter_collection.csv"), recursive=True)
files += glob.glob(os.path.join(root, "diag*", "**", "*counter_collection.csv"), recursive=True)
for f in sorted(files):
    name = os.path.relpath(f, root).split(os.sep)[0]
    var, grp = name.rsplit("_", 2)[0], name
    per = collections.defaultdict(float)
    kn = {}
    for r in csv.DictReader(open(f)):
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        kn[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0].replace("void ", "")
    acc = collections.defaultdict(list)
    for (d, c), v in per.items():
        acc[(kn[d], c)].append(v)
    for (k, c), vs in acc.items():
        runs[name.split("_so_")[0] if name.startswith("fetch_") else "diag"][(k, c)] = sum(vs) / len(vs)
for var, d in runs.items():
    print("==", var)
    if var == "diag":
        for k in sorted({k for k, _ in d if want in k}):
            print("  %s" % k[:60])
            for (kk, c), v in sorted(d.items()):
                if kk == k:
                    print("     %-40s %.4g" % (c, v))
        continue
    ks = sorted({k for k, _ in d if want in k})
    for k in ks:
        fb, wb = d.get((k, "FETCH_SIZE")), d.get((k, "WRITE_SIZE"))
        h, m = d.get((k, "TCC_HIT_sum")), d.get((k, "TCC_MISS_sum"))
        print("  %-48s fetch %s  write %s  l2hit %s" % (
            k[:48], "%.3f GB" % (fb * 1024 / 1e9) if fb is not None else "-",
            "%.3f GB" % (wb * 1024 / 1e9) if wb is not None else "-",
            "%.3f" % (h / (h + m)) if h is not None and m else "-"))
