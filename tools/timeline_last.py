#!/usr/bin/env python3
"""Print the kernel timeline of the second-to-last encode launch in a rocprofv3 kernel trace
(times relative to its k_tile_strings).  usage: tools/timeline_last.py <trace dir or csv>"""
import csv
import glob
import os
import sys

p = sys.argv[1]
f = p if p.endswith(".csv") else glob.glob(os.path.join(p, "**", "run_kernel_trace.csv"), recursive=True)[0]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
            for r in csv.DictReader(open(f)))
starts = [i for i, e in enumerate(ev) if "k_tile_strings" in e[2]]
i0, i1 = starts[-2], starts[-1]
t0 = ev[i0][0]
for a, b, n in ev[i0:i1]:
    print("%8.3f %8.3f %7.3f  %s" % ((a - t0) / 1e6, (b - t0) / 1e6, (b - a) / 1e6, n[:60]))
